"""ctypes binding of the C oracle (oracle/build/libmgp_oracle.so) — TEST INFRASTRUCTURE ONLY.

Builds the oracle with `make -C oracle` on first use if it is not built yet.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "libmgp_oracle.so")

JACOBI, RBGS, GS_LEX = 0, 1, 2
SMOOTHERS = {"jacobi": JACOBI, "rbgs": RBGS, "gs_lex": GS_LEX}
CYCLES = {"V": 0, "F": 1}
PROLONGS = {"pc": 0, "linear": 1}
INITS = {"fresh": 0, "warm": 1}
BCS = {"zero": 0, "consistent": 1}
RESTRICTIONS = {"average": 0, "full_weighting": 1}
# real = float arithmetic: "real" = every operation in float (gpu.lua:32), "double" = float buffers with
# every expression in double (cpu-raw.lua's real = 'float', LuaJIT numbers)
ARITHS = {"real": 0, "double": 1}
F32_ARITH_F64 = 12  # real_bytes code of the stateless *_arr kernels for float arrays + double arithmetic


class Opts(ctypes.Structure):
    _fields_ = [("dim", ctypes.c_int), ("nx", ctypes.c_int64), ("ny", ctypes.c_int64), ("nz", ctypes.c_int64),
                ("real_bytes", ctypes.c_int), ("nu1", ctypes.c_int), ("nu2", ctypes.c_int),
                ("smoother", ctypes.c_int), ("cycle", ctypes.c_int), ("prolong", ctypes.c_int),
                ("coarse_init", ctypes.c_int), ("coarse_sweeps", ctypes.c_int), ("coarse_bc", ctypes.c_int),
                ("threads", ctypes.c_int), ("restriction", ctypes.c_int), ("arith", ctypes.c_int)]


def _load():
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-C", ORACLE_DIR], check=True, capture_output=True)
    lib = ctypes.CDLL(ORACLE_SO)
    vp, i64, d = ctypes.c_void_p, ctypes.c_int64, ctypes.c_double
    lib.mgo_opts_default.argtypes = [ctypes.POINTER(Opts)]
    lib.mgo_create.restype = vp
    lib.mgo_create.argtypes = [ctypes.POINTER(Opts)]
    lib.mgo_destroy.argtypes = [vp]
    lib.mgo_num_levels.argtypes = [vp]
    lib.mgo_init_point_charge.argtypes = [vp]
    lib.mgo_set_field.argtypes = [vp, ctypes.c_int, vp, i64]
    lib.mgo_get_field.argtypes = [vp, ctypes.c_int, vp, i64]
    lib.mgo_step.restype = d
    lib.mgo_step.argtypes = [vp]
    lib.mgo_solve.argtypes = [vp, ctypes.c_int, d, ctypes.POINTER(d)]
    lib.mgo_two_grid.argtypes = [vp, d, vp, vp, i64]
    lib.mgo_smooth_arr.argtypes = [ctypes.c_int, i64, i64, i64, ctypes.c_int, ctypes.c_int, ctypes.c_int, d, d, vp, vp]
    lib.mgo_residual_arr.argtypes = [ctypes.c_int, i64, i64, i64, ctypes.c_int, d, d, vp, vp, vp]
    lib.mgo_restrict_arr.argtypes = [ctypes.c_int, i64, i64, i64, ctypes.c_int, vp, vp]
    lib.mgo_residual_sumsq_arr.restype = d
    lib.mgo_residual_sumsq_arr.argtypes = [ctypes.c_int, i64, i64, i64, ctypes.c_int, d, d, vp, vp, i64, i64, ctypes.c_int]
    lib.mgo_restrict_fw_arr.argtypes = [ctypes.c_int, i64, i64, i64, ctypes.c_int, d, vp, vp]
    lib.mgo_prolong_correct_arr.argtypes = [ctypes.c_int, i64, i64, i64, ctypes.c_int, ctypes.c_int, d, vp, vp]
    lib.mgo_coarse_coef.restype = d
    lib.mgo_coarse_coef.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.mgo_err_arr.restype = d
    lib.mgo_err_arr.argtypes = [i64, ctypes.c_int, vp, vp]
    return lib


lib = _load()


class Oracle:
    """The C oracle configured like mgpoisson.make_opts (same keyword names)."""

    def __init__(self, dim=2, n=(8, 8, 1), real="double", nu1=7, nu2=7, smoother="jacobi", cycle="V",
                 prolong="pc", coarse_init="fresh", coarse_bc="zero", coarse_sweeps=48, threads=1,
                 restriction="average", arith="real"):
        o = Opts()
        lib.mgo_opts_default(ctypes.byref(o))
        nn = tuple(n) + (1,) * (3 - len(n))
        o.dim, o.nx, o.ny, o.nz = dim, nn[0], nn[1], (nn[2] if dim == 3 else 1)
        o.real_bytes = 8 if real == "double" else 4
        o.nu1, o.nu2 = nu1, nu2
        o.smoother, o.cycle, o.prolong = SMOOTHERS[smoother], CYCLES[cycle], PROLONGS[prolong]
        o.coarse_init, o.coarse_bc, o.coarse_sweeps, o.threads = INITS[coarse_init], BCS[coarse_bc], coarse_sweeps, threads
        o.restriction = RESTRICTIONS[restriction]
        o.arith = ARITHS[arith]
        self.o = o
        self.dtype = np.dtype(np.float64 if o.real_bytes == 8 else np.float32)
        self.shape = (o.nz, o.ny, o.nx) if dim == 3 else (o.ny, o.nx)
        self.h = lib.mgo_create(ctypes.byref(o))
        if not self.h:
            raise ValueError("oracle rejected the options")

    def __del__(self):
        if getattr(self, "h", None):
            lib.mgo_destroy(self.h)
            self.h = None

    def init_point_charge(self):
        lib.mgo_init_point_charge(self.h)

    def get(self, which=0):
        out = np.empty(self.shape, self.dtype)
        assert lib.mgo_get_field(self.h, which, out.ctypes.data, out.size) == 0
        return out

    def set(self, which, arr):
        a = np.ascontiguousarray(arr, self.dtype)
        assert lib.mgo_set_field(self.h, which, a.ctypes.data, a.size) == 0

    def step(self):
        return lib.mgo_step(self.h)

    def two_grid(self, h, u, f, size):
        """cpu-raw.lua:186 twoGrid(h, u, f, L) on host arrays of one level's size; u updated in place."""
        assert u.flags.c_contiguous and u.dtype == self.dtype
        fc = np.ascontiguousarray(f, self.dtype)
        assert lib.mgo_two_grid(self.h, h, u.ctypes.data, fc.ctypes.data, int(size)) == 0

    def levels(self):
        return lib.mgo_num_levels(self.h)


def _kind(a, arith):
    """real_bytes code of the stateless kernels: the element size, or F32_ARITH_F64 for float arrays with
    cpu-raw.lua's double arithmetic."""
    return F32_ARITH_F64 if (arith == "double" and a.itemsize == 4) else a.itemsize


def smooth_arr(dim, u, f, smoother, sweeps, h, cl=0.0, arith="real"):
    u = np.ascontiguousarray(u).copy()
    f = np.ascontiguousarray(f, u.dtype)
    nz, ny, nx = (u.shape if dim == 3 else (1,) + u.shape)
    lib.mgo_smooth_arr(dim, nx, ny, nz, _kind(u, arith), SMOOTHERS[smoother], sweeps, h, cl, u.ctypes.data,
                       f.ctypes.data)
    return u


def residual_arr(dim, u, f, h, cl=0.0, arith="real"):
    u = np.ascontiguousarray(u)
    f = np.ascontiguousarray(f, u.dtype)
    r = np.empty_like(u)
    nz, ny, nx = (u.shape if dim == 3 else (1,) + u.shape)
    lib.mgo_residual_arr(dim, nx, ny, nz, _kind(u, arith), h, cl, u.ctypes.data, f.ctypes.data, r.ctypes.data)
    return r


def residual_sumsq_arr(dim, u, f, h, cl=0.0, z_lo=0, z_hi=None, threads=1, arith="real"):
    """sum of (f - A u)^2 (fp64) over planes [z_lo, z_hi) of a 3D (nz, ny, nx) array; its ends are the ghost."""
    u = np.ascontiguousarray(u)
    f = np.ascontiguousarray(f, u.dtype)
    nz, ny, nx = (u.shape if dim == 3 else (1,) + u.shape)
    z_hi = nz if z_hi is None else z_hi
    return lib.mgo_residual_sumsq_arr(dim, nx, ny, nz, _kind(u, arith), h, cl, u.ctypes.data, f.ctypes.data, z_lo,
                                      z_hi, threads)


def restrict_arr(dim, r, arith="real"):
    r = np.ascontiguousarray(r)
    shp = tuple(s // 2 for s in r.shape)
    R = np.empty(shp, r.dtype)
    nz, ny, nx = (r.shape if dim == 3 else (1,) + r.shape)
    lib.mgo_restrict_arr(dim, nx, ny, nz, _kind(r, arith), r.ctypes.data, R.ctypes.data)
    return R


def restrict_fw_arr(dim, r, cl_coarse=0.0, arith="real"):
    """Full-weighting restriction (the adjoint of the linear prolongation), mgp_oracle_impl.h restrict_fw."""
    r = np.ascontiguousarray(r)
    shp = tuple(s // 2 for s in r.shape)
    R = np.empty(shp, r.dtype)
    nz, ny, nx = (r.shape if dim == 3 else (1,) + r.shape)
    lib.mgo_restrict_fw_arr(dim, nx, ny, nz, _kind(r, arith), cl_coarse, r.ctypes.data, R.ctypes.data)
    return R


def prolong_correct_arr(dim, u, V, prolong, cl_coarse=0.0, arith="real"):
    u = np.ascontiguousarray(u).copy()
    V = np.ascontiguousarray(V, u.dtype)
    nz, ny, nx = (u.shape if dim == 3 else (1,) + u.shape)
    lib.mgo_prolong_correct_arr(dim, nx, ny, nz, _kind(u, arith), PROLONGS[prolong], cl_coarse, u.ctypes.data,
                                V.ctypes.data)
    return u


def err_arr(psi, old, arith="real"):
    """sqrt(sum (psi - psiOld)^2 / N) as the oracle's step() computes it (cpu.lua:203, cpu-raw.lua:249-254)."""
    a = np.ascontiguousarray(psi)
    b = np.ascontiguousarray(old, a.dtype)
    return lib.mgo_err_arr(a.size, _kind(a, arith), a.ctypes.data, b.ctypes.data)


def coarse_coef(bc, level):
    return lib.mgo_coarse_coef(BCS[bc], level)
