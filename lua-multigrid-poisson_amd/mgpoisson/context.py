"""Thin object wrapper of one ``mgp_ctx`` (include/mgpoisson.h).

Host buffers are numpy arrays (C-contiguous, x fastest: shape (nz, ny, nx) or (ny, nx));
device buffers are passed as raw pointers (e.g. ``torch_tensor.data_ptr()``) with
``mem=MEM_DEVICE``.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L

SMOOTHERS = {"jacobi": L.JACOBI, "rbgs": L.RBGS, "gs_lex": L.GS_LEX}
CYCLES = {"V": L.CYCLE_V, "F": L.CYCLE_F}
PROLONGS = {"pc": L.PROLONG_PC, "linear": L.PROLONG_LINEAR}
COARSE_INITS = {"fresh": L.COARSE_FRESH, "warm": L.COARSE_WARM}
COARSE_BCS = {"zero": L.BC_ZERO, "consistent": L.BC_CONSISTENT}
RESTRICTIONS = {"average": L.RESTRICT_AVERAGE, "full_weighting": L.RESTRICT_FULL_WEIGHTING}
REALS = {"double": 8, "float": 4}
# real = float arithmetic: "real" = every operation in float (gpu.lua:32), "double" = float buffers with every
# expression in double, rounded at each store (cpu-raw.lua's real = 'float', cpu-raw.lua:142-153)
ARITHS = {"real": L.ARITH_REAL, "double": L.ARITH_DOUBLE}


def make_opts(dim=2, n=(8, 8, 1), real="double", nu1=7, nu2=7, smoother="jacobi", cycle="V",
              prolong="pc", coarse_init="fresh", coarse_bc="zero", coarse_sweeps=48, err_mode=1,
              device=-1, rank=0, world=1, gather_cells=32768, comm_id: bytes | None = None,
              restriction="average", arith="real") -> L.MGPOpts:
    """Build mgp_opts from keyword names (defaults = the reference cpu.lua configuration)."""
    o = L.default_opts()
    o.dim = dim
    nn = tuple(n) + (1,) * (3 - len(n))
    o.n[0], o.n[1], o.n[2] = nn[0], nn[1], (nn[2] if dim == 3 else 1)
    o.real_bytes = REALS[real] if isinstance(real, str) else int(real)
    o.nu1, o.nu2 = nu1, nu2
    o.smoother = SMOOTHERS[smoother] if isinstance(smoother, str) else smoother
    o.cycle = CYCLES[cycle] if isinstance(cycle, str) else cycle
    o.prolong = PROLONGS[prolong] if isinstance(prolong, str) else prolong
    o.coarse_init = COARSE_INITS[coarse_init] if isinstance(coarse_init, str) else coarse_init
    o.coarse_bc = COARSE_BCS[coarse_bc] if isinstance(coarse_bc, str) else coarse_bc
    o.coarse_sweeps = coarse_sweeps
    o.err_mode = err_mode
    o.device = device
    o.rank, o.world = rank, world
    o.gather_cells = gather_cells
    o.restriction = RESTRICTIONS[restriction] if isinstance(restriction, str) else restriction
    o.arith = ARITHS[arith] if isinstance(arith, str) else arith
    if comm_id is not None:
        ctypes.memmove(o.comm_id, comm_id, L.COMM_ID_BYTES)
    return o


class Loopback:
    """A loopback transport group (tests): `world` ranks as contexts of this process on one GPU,
    each driven from its own thread (see mgp_create_loopback)."""

    def __init__(self, world: int):
        h = ctypes.c_void_p()
        L.check(L.lib.mgp_loopback_create(ctypes.byref(h), world))
        self._h = h
        self.world = world

    def close(self):
        if getattr(self, "_h", None):
            L.lib.mgp_loopback_destroy(self._h)
            self._h = None


class Context:
    """Owns one mgp_ctx: the level hierarchy, its device buffers and stream."""

    def __init__(self, opts: L.MGPOpts, loopback: "Loopback | None" = None):
        self.opts = opts
        self.dtype = np.dtype(np.float64 if opts.real_bytes == 8 else np.float32)
        h = ctypes.c_void_p()
        if loopback is not None:
            L.check(L.lib.mgp_create_loopback(ctypes.byref(h), ctypes.byref(opts), loopback._h))
        else:
            L.check(L.lib.mgp_create(ctypes.byref(h), ctypes.byref(opts)))
        self._h = h
        self._read_levels()

    def _read_levels(self):
        self.levels = []
        info = (ctypes.c_int64 * 8)()
        for l in range(L.lib.mgp_num_levels(self._h)):
            L.check(L.lib.mgp_level_info(self._h, l, info), self._h)
            self.levels.append(dict(nx=info[0], ny=info[1], nz_global=info[2], nz_local=info[3],
                                    z0=info[4], distributed=bool(info[5]), tail=info[6] == 1,
                                    engine=("piece", "tail", "zs", "blk", "zpost")[info[6]], exchanges=info[7]))

    # -- lifecycle --
    def close(self):
        if getattr(self, "_h", None):
            L.lib.mgp_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _chk(self, rc):
        return L.check(rc, self._h)

    # -- shapes --
    def shape(self, level=0):
        lv = self.levels[level]
        if self.opts.dim == 3:
            return (lv["nz_local"], lv["ny"], lv["nx"])
        return (lv["ny"], lv["nx"])

    def count(self, level=0):
        return int(np.prod(self.shape(level)))

    # -- data --
    def init_point_charge(self):
        self._chk(L.lib.mgp_init_point_charge(self._h))

    def set_field(self, which, arr, level=0):
        a = np.ascontiguousarray(arr, dtype=self.dtype)
        if a.size != self.count(level):
            raise ValueError(f"expected {self.count(level)} elements, got {a.size}")
        self._chk(L.lib.mgp_set_field(self._h, level, which, a.ctypes.data, a.size, L.MEM_HOST))

    def get_field(self, which, level=0):
        out = np.empty(self.shape(level), dtype=self.dtype)
        self._chk(L.lib.mgp_get_field(self._h, level, which, out.ctypes.data, out.size, L.MEM_HOST))
        return out

    def get_planes(self, which, z_begin, nz, level=0):
        """Local planes [z_begin, z_begin + nz) of a field as an (nz, ny, nx) host array."""
        lv = self.levels[level]
        out = np.empty((nz, lv["ny"], lv["nx"]), dtype=self.dtype)
        self._chk(L.lib.mgp_get_planes(self._h, level, which, int(z_begin), int(nz), out.ctypes.data, L.MEM_HOST))
        return out

    def set_planes(self, which, z_begin, arr, level=0):
        lv = self.levels[level]
        a = np.ascontiguousarray(arr, dtype=self.dtype)
        if a.size % (lv["ny"] * lv["nx"]) != 0:
            raise ValueError("set_planes: the array must hold whole planes")
        nz = a.size // (lv["ny"] * lv["nx"])
        self._chk(L.lib.mgp_set_planes(self._h, level, which, int(z_begin), int(nz), a.ctypes.data, L.MEM_HOST))

    def field_stats(self, which=L.FIELD_U, level=0):
        """(hash, sum, sum of squares, max |x|) of this rank's part of a field, computed on the device."""
        h = ctypes.c_uint64()
        d = (ctypes.c_double * 3)()
        self._chk(L.lib.mgp_field_stats(self._h, level, which, ctypes.byref(h), d))
        return h.value, d[0], d[1], d[2]

    def set_psi(self, arr, level=0):
        self.set_field(L.FIELD_U, arr, level)

    def set_f(self, arr, level=0):
        self.set_field(L.FIELD_F, arr, level)

    def get_psi(self, level=0):
        return self.get_field(L.FIELD_U, level)

    def get_f(self, level=0):
        return self.get_field(L.FIELD_F, level)

    # -- cycles --
    def cycle(self) -> float:
        e = ctypes.c_double()
        self._chk(L.lib.mgp_cycle(self._h, ctypes.byref(e)))
        return e.value

    def cycles(self, k: int) -> np.ndarray:
        errs = np.zeros(k, dtype=np.float64)
        self._chk(L.lib.mgp_cycles(self._h, k, errs.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
        return errs

    def two_grid(self, h: float, u: np.ndarray, f: np.ndarray, size: int):
        """cpu-raw.lua:186 twoGrid(h, u, f, L) on host arrays; u updated in place."""
        if not (u.flags.c_contiguous and u.dtype == self.dtype):
            raise ValueError("u must be a C-contiguous array of the context's real type")
        fc = np.ascontiguousarray(f, dtype=self.dtype)
        lv = next((x for x in self.levels if x["nx"] == int(size)), None)
        need = None if lv is None else lv["nx"] * lv["ny"] * (lv["nz_local"] if self.opts.dim == 3 else 1)
        if need is not None and (u.size != need or fc.size != need):
            raise ValueError(f"two_grid: u and f must hold {need} reals each (got {u.size}, {fc.size})")
        self._chk(L.lib.mgp_two_grid(self._h, float(h), u.ctypes.data, fc.ctypes.data, int(size), L.MEM_HOST))

    def two_grid_ptr(self, h: float, u_ptr: int, f_ptr: int, size: int, mem=L.MEM_DEVICE):
        self._chk(L.lib.mgp_two_grid(self._h, float(h), u_ptr, f_ptr, int(size), mem))

    # -- level-granular pieces --
    def smooth(self, level, sweeps):
        self._chk(L.lib.mgp_smooth(self._h, level, sweeps))

    def residual_restrict(self, level):
        self._chk(L.lib.mgp_residual_restrict(self._h, level))

    def prolong_correct(self, level):
        self._chk(L.lib.mgp_prolong_correct(self._h, level))

    def coarse_solve(self):
        self._chk(L.lib.mgp_coarse_solve(self._h))

    def set_coarse_level(self, size: int):
        """Levels of nx <= size run in the one-launch LDS coarse engine (cpuDepth, cpu-gpu.lua:61)."""
        self._chk(L.lib.mgp_set_coarse_level(self._h, int(size)))
        self._read_levels()

    def set_coarse_handoff(self, size: int, engine):
        """cpu-gpu.lua:17-52: at the level of nx = size call engine(h, u, f, size) on host numpy views
        (u updated in place); engine=None removes the hand-off."""
        if engine is None:
            self._handoff = None
            self._chk(L.lib.mgp_set_coarse_handoff(self._h, int(size), L.COARSE_FN(), None))
            return
        lvl = next(i for i, lv in enumerate(self.levels) if lv["nx"] == size)
        shape = self.shape(lvl)
        count = int(np.prod(shape))
        dt = self.dtype

        def cb(user, h, u_ptr, f_ptr, n):
            try:
                u = np.ctypeslib.as_array((ctypes.c_char * (count * dt.itemsize)).from_address(u_ptr)).view(dt).reshape(shape)
                f = np.ctypeslib.as_array((ctypes.c_char * (count * dt.itemsize)).from_address(f_ptr)).view(dt).reshape(shape)
                engine(h, u, f, int(n))
                return 0
            except Exception:  # noqa: BLE001 - reported as a library error
                return 1

        self._handoff = L.COARSE_FN(cb)  # keep the trampoline alive
        self._chk(L.lib.mgp_set_coarse_handoff(self._h, int(size), self._handoff, None))

    def metrics(self):
        """(rel_err, count, frob) of the last outer iteration (gpu.lua:173-200, test-gpu-obj.lua:216-247)."""
        rel, n, frob = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
        self._chk(L.lib.mgp_metrics(self._h, ctypes.byref(rel), ctypes.byref(n), ctypes.byref(frob)))
        return rel.value, n.value, frob.value

    def residual_norm(self, level=0):
        """(||f - A u||_2, ||f||_2) of a level, reduced on the device (fp64)."""
        r, f = ctypes.c_double(), ctypes.c_double()
        self._chk(L.lib.mgp_residual_norm(self._h, level, ctypes.byref(r), ctypes.byref(f)))
        return r.value, f.value

    def cg_solve(self, epsilon=1e-20, maxiter=10000, history=False):
        """Device CG on the finest level (converge-multigrid-vs-krylov.lua:38-69): x0 = -f, b = f, stop at
        rSq / bSq < epsilon.  Returns (x, iterations, rSq / bSq[, |x|_inf per iteration])."""
        x = np.empty(self.shape(0), dtype=self.dtype)
        it, err = ctypes.c_int32(), ctypes.c_double()
        hist = np.zeros(maxiter, dtype=np.float64) if history else None
        self._chk(L.lib.mgp_cg_solve(self._h, float(epsilon), int(maxiter), x.ctypes.data, L.MEM_HOST, ctypes.byref(it),
                                     ctypes.byref(err),
                                     hist.ctypes.data_as(ctypes.POINTER(ctypes.c_double)) if history else None))
        if history:
            return x, it.value, err.value, hist[:it.value]
        return x, it.value, err.value

    def sync(self):
        self._chk(L.lib.mgp_sync(self._h))

    def set_debug(self, mode=1):
        """The reference's debugging check (cpu-raw.lua:126-140, gpu.lua:269-284): after every phase of a cycle its
        output is scanned on the device, and cycle() / cycles() raise MGPError naming the first phase that produced
        a NaN or inf ("found a nan").  mode 0 turns it off."""
        self._chk(L.lib.mgp_set_debug(self._h, int(mode)))

    # -- timing --
    def timing(self, enable=True):
        self._chk(L.lib.mgp_timing(self._h, 1 if enable else 0))

    def comm_log(self, reset=False, max_rows=1 << 16):
        """The exchanges / collectives this rank issued, in order: [(op, side, level, msgs, bytes)] with op one of
        "exchange" (msgs per neighbour and direction, bytes sent per neighbour), "allgather", "allreduce"; side 1 =
        the side stream's communicator (mgp_comm_log)."""
        rows = (ctypes.c_int64 * (5 * max_rows))()
        n = self._chk(L.lib.mgp_comm_log(self._h, rows, max_rows, 1 if reset else 0))
        return [(L.COMM_OPS[rows[5 * i]],) + tuple(rows[5 * i + k] for k in range(1, 5)) for i in range(min(n, max_rows))]

    def timing_read(self):
        """{kind name: (ms, launches / calls, bytes)} timed so far: the level-0 smoothing launches (algorithmic
        bytes) and every halo exchange / collective (bytes this rank sends)."""
        out = {}
        for kind, name in L.TIMING_KINDS.items():
            ms, n, by = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
            self._chk(L.lib.mgp_timing_read(self._h, kind, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(by)))
            out[name] = (ms.value, n.value, by.value)
        return out

    def timing_kernels(self):
        """{kind name: (kernel symbol as rocprofv3 prints it, grid in work-items)} of the last timed level-0 fused
        launch of each kind (mgp_timing_kernel); kinds without a timed launch are absent."""
        out = {}
        for kind, name in L.TIMING_KINDS.items():
            buf, grid = ctypes.create_string_buffer(128), ctypes.c_int64()
            if L.lib.mgp_timing_kernel(self._h, kind, buf, len(buf), ctypes.byref(grid)) == 0:
                out[name] = (buf.value.decode(), grid.value)
        return out


class Group:
    """One host process driving `ngpu` GPUs (mgp_group_create): one z-slab context per rank, RCCL
    communicators from ncclCommInitAll, every call run by one host thread per device inside the
    library.  devices all equal (e.g. [0] * 8) = the ranks share that GPU through the loopback
    transport (tests).  Field I/O is global (the whole box, x fastest)."""

    def __init__(self, opts: L.MGPOpts, ngpu: int, devices=None):
        self.opts = opts
        self.dtype = np.dtype(np.float64 if opts.real_bytes == 8 else np.float32)
        h = ctypes.c_void_p()
        devs = None if devices is None else (ctypes.c_int * ngpu)(*devices)
        L.check_group(L.lib.mgp_group_create(ctypes.byref(h), ctypes.byref(opts), ngpu, devs))
        self._h = h
        self.ngpu = ngpu
        self.ranks = [_RankView(L.lib.mgp_group_rank(h, r), opts) for r in range(ngpu)]
        self.levels = self.ranks[0].levels

    def close(self):
        if getattr(self, "_h", None):
            L.lib.mgp_group_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc):
        return L.check_group(rc, self._h)

    def shape(self, level=0):
        lv = self.levels[level]
        return (lv["nz_global"], lv["ny"], lv["nx"])

    def init_point_charge(self):
        self._chk(L.lib.mgp_group_init_point_charge(self._h))

    def cycle(self) -> float:
        e = ctypes.c_double()
        self._chk(L.lib.mgp_group_cycle(self._h, ctypes.byref(e)))
        return e.value

    def cycles(self, k: int) -> np.ndarray:
        errs = np.zeros(k, dtype=np.float64)
        self._chk(L.lib.mgp_group_cycles(self._h, k, errs.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
        return errs

    def get_field(self, which, level=0):
        out = np.empty(self.shape(level), dtype=self.dtype)
        self._chk(L.lib.mgp_group_get_field(self._h, level, which, out.ctypes.data, out.size, L.MEM_HOST))
        return out

    def set_field(self, which, arr, level=0):
        a = np.ascontiguousarray(arr, dtype=self.dtype)
        self._chk(L.lib.mgp_group_set_field(self._h, level, which, a.ctypes.data, a.size, L.MEM_HOST))

    def get_psi(self, level=0):
        return self.get_field(L.FIELD_U, level)

    def residual_norm(self, level=0):
        r, f = ctypes.c_double(), ctypes.c_double()
        self._chk(L.lib.mgp_group_residual_norm(self._h, level, ctypes.byref(r), ctypes.byref(f)))
        return r.value, f.value

    def field_stats(self, which=L.FIELD_U, level=0):
        h = ctypes.c_uint64()
        d = (ctypes.c_double * 3)()
        self._chk(L.lib.mgp_group_field_stats(self._h, level, which, ctypes.byref(h), d))
        return h.value, d[0], d[1], d[2]


class _RankView(Context):
    """A rank's context owned by a Group (not destroyed on its own)."""

    def __init__(self, handle, opts):  # noqa: D401 - no super().__init__: the group created it
        self.opts = opts
        self.dtype = np.dtype(np.float64 if opts.real_bytes == 8 else np.float32)
        self._h = ctypes.c_void_p(handle)
        self._read_levels()

    def close(self):
        self._h = None
