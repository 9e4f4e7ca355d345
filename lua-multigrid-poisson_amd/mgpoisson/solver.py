"""Host-side mirror of the reference's two solver-call protocols, over libmgpoisson.so.

The reference's host language is Lua (no Lua runtime exists in this image), so the drop-in
host layer is written in Python with the same names, argument meanings and error behaviour;
the LuaJIT-FFI module a Lua user would load is lua/multigrid-poisson/hip.lua.

* :class:`MultigridHIP` — the ``cpu.lua`` table protocol:
  ``MultigridCPU{size=n, maxiter=?, epsilon=?, errorCallback=?, debug=?}`` then
  ``:solve()`` / ``:step()`` / ``:twoGrid(h, u, f)`` (cpu.lua:70, 173-216).
* :class:`MultigridHIPRaw` — the ``cpu-raw.lua`` / ``gpu.lua`` positional protocol:
  ``MultigridCPURaw(size, real)`` then ``:run()`` (2 outer iterations) and
  ``:twoGrid(h, uPtr, fPtr, L)`` (cpu-raw.lua:142, 186, 239-258; gpu.lua:26, 296, 348).
  ``real='float'`` follows cpu-raw.lua's arithmetic by default (float buffers, every expression in
  double: ``arith='double'``); ``arith='real'`` gives gpu.lua's float-rounded OpenCL arithmetic.
"""
from __future__ import annotations

import logging
import math

import numpy as np

from . import _lib as L
from ._lib import MGPError
from .context import Context, make_opts

log = logging.getLogger(__name__)


class _Smoother(str):
    """The values of ``inPlaceIterativeSolver`` (cpu.lua:56-57): ``MultigridHIP.Jacobi`` (the
    reference's active choice), ``MultigridHIP.GaussSeidel`` (cpu.lua:24-37's lexicographic in-place
    sweep, bit for bit: hyperplane-ordered on the GPU, one rank's box) or
    ``MultigridHIP.RedBlackGaussSeidel`` (the build's red/black form, which the temporally blocked
    engines run; gpu.lua:61-81's racy GPU variant is not offered)."""


class LevelFields:
    """``mg.rs[L]`` / ``mg.Rs[L]`` / ``mg.vs[L]`` / ``mg.Vs[L]`` of cpu-raw.lua:155-171: the field of the
    level of size L (a power of two, as the reference's table keys), downloaded from HBM."""

    def __init__(self, ctx_fn, which):
        self._ctx_fn = ctx_fn
        self._which = which

    def _level(self, size):
        ctx = self._ctx_fn()
        for l, lv in enumerate(ctx.levels):
            if lv["nx"] == int(size):
                return ctx, l
        raise KeyError(size)

    def __getitem__(self, size):
        ctx, l = self._level(size)
        return ctx.get_field(self._which, l)

    def __setitem__(self, size, value):
        ctx, l = self._level(size)
        if self._which not in (L.FIELD_U, L.FIELD_F):
            raise TypeError("rs / vs are computed views (read-only)")
        ctx.set_field(self._which, value, l)

    def keys(self):
        return [lv["nx"] for lv in self._ctx_fn().levels]


class _RawFields:
    """cpu-raw.lua's buffer fields on a context: psiOld, errorBuf, tmpU and the per-level rs/Rs/vs/Vs."""

    @property
    def psiOld(self):
        return self.ctx.get_field(L.FIELD_PSI_OLD, 0)

    @property
    def errorBuf(self):
        return self.ctx.get_field(L.FIELD_ERROR, 0)

    @property
    def tmpU(self):
        return self.ctx.get_field(L.FIELD_TMP, 0)

    @property
    def rs(self):
        return LevelFields(lambda: self.ctx, L.FIELD_RESIDUAL)

    @property
    def Rs(self):
        return LevelFields(lambda: self.ctx, L.FIELD_F)

    @property
    def vs(self):
        return LevelFields(lambda: self.ctx, L.FIELD_CORRECTION)

    @property
    def Vs(self):
        return LevelFields(lambda: self.ctx, L.FIELD_U)


class MultigridHIP(_RawFields):
    """Drop-in for ``MultigridCPU`` (cpu.lua:15-218), solving on the GPU.

    ``MultigridHIP({'size': n, 'maxiter': ..., 'epsilon': ..., 'errorCallback': fn,
    'debug': ...})`` or the same as keyword arguments.  A missing (None) field falls back to
    the class default exactly as the Lua ``self.maxiter = args.maxiter`` does (cpu.lua:174-177
    with the class fields of cpu.lua:18-22).  Build options beyond the reference's (``dim``,
    ``real``, ``smoother``, ``cycle``, ``prolong``, ``coarse_init``, ``coarse_bc``, ``restriction``)
    default to the reference configuration: 2D, double, Jacobi 7+7, V-cycle, injection, 2x2 average,
    fresh zero guess.
    """

    debug = False
    smooth = 7  # cpu.lua:20
    epsilon = 1e-10  # cpu.lua:21
    maxiter = 1000  # cpu.lua:22
    Jacobi = _Smoother("jacobi")  # cpu.lua:40-54
    GaussSeidel = _Smoother("gs_lex")  # cpu.lua:24-37, lexicographic, bit-identical
    RedBlackGaussSeidel = _Smoother("rbgs")  # build-defined red/black (the north-star smoother)

    def __init__(self, args=None, **kw):
        a = dict(args or {})
        a.update(kw)
        if "size" not in a:
            raise TypeError("MultigridHIP: 'size' is required (cpu.lua:178)")
        n = int(a["size"])
        for k in ("maxiter", "epsilon"):
            if a.get(k) is not None:
                setattr(self, k, a[k])
        self.errorCallback = a.get("errorCallback")
        if a.get("debug") is not None:
            self.debug = a["debug"]
        if a.get("smooth") is not None:
            self.smooth = int(a["smooth"])
        self.dim = int(a.get("dim", 2))
        self.size = (n,) * self.dim  # matrix{size, size} (cpu.lua:178)
        sm = a.get("inPlaceIterativeSolver", a.get("smoother", "jacobi"))
        self._build = dict(dim=self.dim, real=a.get("real", "double"), smoother=_smoother_name(sm),
                           cycle=a.get("cycle", "V"), prolong=a.get("prolong", "pc"),
                           coarse_init=a.get("coarse_init", "fresh"), coarse_bc=a.get("coarse_bc", "zero"),
                           restriction=a.get("restriction", "average"), device=a.get("device", -1))
        self._ctx = None
        self._ctx_smooth = None
        self._ensure_ctx()
        self._ctx.init_point_charge()  # f = point charge, psi = -f (cpu.lua:180-193)

    # The reference reads self.smooth inside every twoGrid call (cpu.lua:96, 161); the
    # sweep counts are baked into the device context, so a change rebuilds it, keeping psi/f.
    @property
    def inPlaceIterativeSolver(self):
        """cpu.lua:56-57's knob: MultigridHIP.Jacobi, .GaussSeidel or .RedBlackGaussSeidel (writable)."""
        return {"jacobi": self.Jacobi, "gs_lex": self.GaussSeidel}.get(self._build["smoother"], self.RedBlackGaussSeidel)

    @inPlaceIterativeSolver.setter
    def inPlaceIterativeSolver(self, value):
        name = _smoother_name(value)
        if name != self._build["smoother"]:
            self._build["smoother"] = name
            self._ctx_smooth = None  # rebuild on next use, keeping psi / f

    @property
    def ctx(self):
        self._ensure_ctx()
        return self._ctx

    def _ensure_ctx(self):
        if self._ctx is not None and self._ctx_smooth == self.smooth:
            return
        psi = f = None
        if self._ctx is not None:
            psi, f = self._ctx.get_psi(), self._ctx.get_f()
            self._ctx.close()
        n = self.size[0]
        opts = make_opts(n=(n, n, n if self.dim == 3 else 1), nu1=self.smooth, nu2=self.smooth, **self._build)
        self._ctx = Context(opts)
        self._ctx_smooth = self.smooth
        if psi is not None:
            self._ctx.set_psi(psi)
            self._ctx.set_f(f)

    @property
    def psi(self) -> np.ndarray:
        """Current solution as an (n, n[, n]) host array (downloaded from HBM)."""
        return self._ctx.get_psi()

    @psi.setter
    def psi(self, value):
        self._ctx.set_psi(value)

    @property
    def f(self) -> np.ndarray:
        return self._ctx.get_f()

    @f.setter
    def f(self, value):
        self._ctx.set_f(value)

    def step(self) -> float:
        """cpu.lua:196-206: psiOld = psi; twoGrid(1/n, psi, f); return RMS(psi - psiOld)."""
        self._ensure_ctx()
        err = self._ctx.cycle()
        if self.debug:
            print("err", err)
        return err

    def solve(self):
        """cpu.lua:208-216, including its break rules."""
        if self.debug:
            print("#iter", "err")
        for it in range(1, int(self.maxiter) + 1):
            err = self.step()
            if self.errorCallback and self.errorCallback(it, err):
                break
            if err < self.epsilon or not math.isfinite(err):
                break

    def twoGrid(self, h, u, f):
        """cpu.lua:70 twoGrid(h, u, f): u updated in place.  u / f are (L, L[, L]) host arrays, or
        cpu.lua-style 1-based-indexed nested lists u[i][j] (x = i), whose rows are updated in place."""
        self._ensure_ctx()
        if isinstance(u, np.ndarray):
            self._ctx.two_grid(h, u, f, u.shape[-1])
            return u
        # lua-matrix form: nested lists indexed [i][j] with x = i (cpu.lua:43-53)
        ua = np.ascontiguousarray(np.array(u, dtype=self._ctx.dtype).T)
        fa = np.ascontiguousarray(np.array(f, dtype=self._ctx.dtype).T)
        self._ctx.two_grid(h, ua, fa, ua.shape[-1])
        for i, row in enumerate(u):
            row[:] = ua[:, i].tolist()
        return u


def _smoother_name(v):
    if callable(v) and getattr(v, "__name__", "") in ("Jacobi", "GaussSeidel", "RedBlackGaussSeidel"):
        v = v.__name__
    v = str(v)
    names = {"jacobi": "jacobi", "Jacobi": "jacobi", "gs_lex": "gs_lex", "GaussSeidel": "gs_lex",
             "gaussseidel": "gs_lex", "rbgs": "rbgs", "RedBlackGaussSeidel": "rbgs"}
    if v not in names:
        raise ValueError(f"inPlaceIterativeSolver: {v!r} (Jacobi | GaussSeidel | RedBlackGaussSeidel)")
    return names[v]


class MultigridHIPRaw(_RawFields):
    """Drop-in for ``MultigridCPURaw`` / ``MultigridGPU`` (cpu-raw.lua:118-260, gpu.lua:18-375).

    ``MultigridHIPRaw(size, real='double')``; ``run()`` does the reference's two hard-coded
    outer iterations (cpu-raw.lua:245) printing ``#iter err`` lines; ``twoGrid(h, u, f, L)``
    takes host numpy arrays or integer device pointers (``mem=MEM_DEVICE``).  With ``real='float'`` the
    arithmetic is cpu-raw.lua's (LuaJIT doubles over float images: ``arith='double'``, the default of this
    protocol); ``arith='real'`` selects gpu.lua's (every operation rounded to float, gpu.lua:32).
    """

    debugging = False
    smooth = 7  # cpu-raw.lua:123
    accuracy = 1e-10  # cpu-raw.lua:124

    def __init__(self, size, real="double", cpuDepth=None, **build):
        self.real = real or "double"  # cpu-raw.lua:143
        self.size = int(size)
        self.cpuDepth = cpuDepth
        dim = int(build.pop("dim", 2))
        n = self.size
        self.arith = build.pop("arith", "double")  # cpu-raw.lua's LuaJIT arithmetic (no effect on double)
        opts = make_opts(dim=dim, n=(n, n, n if dim == 3 else 1), real=self.real, nu1=build.pop("nu1", self.smooth),
                         nu2=build.pop("nu2", self.smooth), coarse_init=build.pop("coarse_init", "warm"),
                         arith=self.arith, **build)
        self._ctx = Context(opts)
        if cpuDepth:  # cpu-gpu.lua:61: switch to the coarse engine at size 2^cpuDepth when it fits
            try:
                self._ctx.set_coarse_level(1 << int(cpuDepth))
            except MGPError as e:  # the default switch stays (cpu-raw arithmetic has no coarse engine)
                log.info("cpuDepth %s not applied: %s", cpuDepth, e)
        self._ctx.init_point_charge()  # call2D(initCells) (cpu-raw.lua:173)
        self.quiet = False

    @property
    def ctx(self):
        return self._ctx

    @property
    def psi(self):
        return self._ctx.get_psi()

    @property
    def f(self):
        return self._ctx.get_f()

    def twoGrid(self, h, u, f, L_, mem=None):
        if isinstance(u, np.ndarray):
            self._ctx.two_grid(h, u, f, L_)
        else:
            self._ctx.two_grid_ptr(h, int(u), int(f), L_, L.MEM_DEVICE if mem is None else mem)

    def run(self, iters: int = 2):
        """cpu-raw.lua:239-258 / gpu.lua:348-373 (2 outer iterations, printed).  With ``debugging`` set (class or
        instance field, cpu-raw.lua:121 / gpu.lua:21) every phase's output is checked for non-finite cells and the
        first one raises "found a nan" (cpu-raw.lua:135-139, gpu.lua:279-283)."""
        self._ctx.set_debug(1 if self.debugging else 0)
        if not self.quiet:
            print("#iter", "err")
        errs = []
        for it in range(1, iters + 1):
            err = self._ctx.cycle()
            errs.append(err)
            if not self.quiet:
                print(it, err)
            if err < self.accuracy or not math.isfinite(err):
                break
        return errs


class MultigridHIPHybrid(MultigridHIPRaw):
    """Drop-in for ``MultigridCPUGPU`` (cpu-gpu.lua:55-72): ``MultigridHIPHybrid(size, real,
    cpuDepth, engine)`` runs the fine levels on the GPU and hands the level of size 2^cpuDepth to
    ``engine(h, u, f, L)`` (a coarse twoGrid on host arrays, e.g. a CPU solver), then continues.
    Without an engine the hand-off goes to the GPU's own one-launch coarse engine."""

    def __init__(self, size, real="double", cpuDepth=3, engine=None, **build):
        super().__init__(size, real, cpuDepth if engine is None else None, **build)
        if engine is not None:
            self._ctx.set_coarse_handoff(1 << int(cpuDepth), engine)
