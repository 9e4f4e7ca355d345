"""Independent NumPy restatement of the reference multigrid cycle (TEST INFRASTRUCTURE ONLY).

Only tests/ and bench.py's cpu_baseline leg may import this module; it is the checker,
never the product.  It restates the same reference lines as ``mgp_oracle.c`` (see
``mgp_oracle.h``) with whole-array NumPy operations instead of per-cell loops, so that two
independent restatements must agree bit-for-bit in fp64 (and fp32) before either is trusted:

* ``cpu.lua:40-54`` Jacobi, ``cpu.lua:108-123`` residual, ``cpu.lua:127-135`` restriction,
  ``cpu.lua:138-158`` fresh-zero coarse guess + piecewise-constant prolongation + correction,
  ``cpu.lua:76-93`` 1-cell coarse solve, ``cpu.lua:180-206`` init / step / err,
  ``cpu-raw.lua:221`` warm (persistent) coarse buffers.
* Build-defined: 3D 7-point form, red/black GS, F-cycle, cell-centred linear prolongation.
* ``arith="double"`` with float32 arrays: ``cpu-raw.lua`` under ``real = 'float'`` (cpu-raw.lua:142-153) —
  float buffers read into LuaJIT numbers, so every expression is evaluated in float64 and rounded to
  float32 once, where the reference stores into a buffer (Jacobi :34-44, calcResidual :46-57,
  reduceResidual :59-63, expandResidual / addTo :65-85, calcFrobErr's errorBuf :96-100).  The default
  ``arith="real"`` rounds every operation to the array type (gpu.lua's OpenCL ``real``, gpu.lua:32).

Parity status: "parity unpinned" against the reference itself (no Lua runtime here, no
reference golden vectors); pinned by known-answer tests in tests/test_oracle.py.

Arrays are shaped (nz, ny, nx) — x fastest, the ``cpu-raw.lua`` layout ``i + L*j`` — with
nz = 1 for 2D.  Summation orders match the reference: ((xl + xr) + yl) + yr [+ zl + zr].
"""
from __future__ import annotations

import numpy as np

JACOBI, RBGS, GS_LEX = 0, 1, 2
CYCLE_V, CYCLE_F = 0, 1
PROLONG_PC, PROLONG_LINEAR = 0, 1
COARSE_FRESH, COARSE_WARM = 0, 1
BC_ZERO, BC_CONSISTENT = 0, 1
RESTRICT_AVERAGE, RESTRICT_FULL_WEIGHTING = 0, 1


def _nbsum(u: np.ndarray, dim: int) -> np.ndarray:
    p = np.pad(u, 1) if dim == 3 else np.pad(u, ((0, 0), (1, 1), (1, 1)))
    if dim == 3:
        c = p[1:-1, 1:-1, 1:-1]
        xl, xr = p[1:-1, 1:-1, :-2], p[1:-1, 1:-1, 2:]
        yl, yr = p[1:-1, :-2, 1:-1], p[1:-1, 2:, 1:-1]
        zl, zr = p[:-2, 1:-1, 1:-1], p[2:, 1:-1, 1:-1]
        del c
        return ((((xl + xr) + yl) + yr) + zl) + zr
    xl, xr = p[:, 1:-1, :-2], p[:, 1:-1, 2:]
    yl, yr = p[:, :-2, 1:-1], p[:, 2:, 1:-1]
    return ((xl + xr) + yl) + yr


def _consts(h: float, dim: int, dt):
    hh = dt.type(h)
    hsq = hh * hh
    adiag = dt.type(-2 * dim) / hsq
    return hsq, adiag


def nfaces(shape, dim, z0=0, gnz=None):
    """Boundary faces per cell (a 1-cell axis counts 2); z uses global index z0 + k of gnz."""
    nz, ny, nx = shape
    gnz = nz if gnz is None else gnz
    i = np.arange(nx)
    j = np.arange(ny)
    nb = ((i == 0).astype(np.int64) + (i == nx - 1))[None, None, :] + \
         ((j == 0).astype(np.int64) + (j == ny - 1))[None, :, None]
    if dim == 3:
        k = np.arange(nz) + z0
        nb = nb + ((k == 0).astype(np.int64) + (k == gnz - 1))[:, None, None]
    return np.broadcast_to(nb, shape)


def diag(shape, h, dim, dt, cl, z0=0, gnz=None):
    """Level operator diagonal: the reference adiag when cl = 0 (mgp_oracle_impl.h diag())."""
    hsq, adiag = _consts(h, dim, dt)
    c = dt.type(cl)
    if c == 0:
        return np.full(shape, adiag, dtype=dt)
    nb = nfaces(shape, dim, z0, gnz)
    dg = (dt.type(-2 * dim) - nb.astype(dt) * c) / hsq
    return np.where(nb == 0, adiag, dg).astype(dt)


def _relax(u, f, h, dim, cl=0.0, z0=0, gnz=None):
    hsq, _ = _consts(h, dim, u.dtype)
    return (f - _nbsum(u, dim) / hsq) / diag(u.shape, h, dim, u.dtype, cl, z0, gnz)


def color_mask(shape, z0: int = 0) -> np.ndarray:
    nz, ny, nx = shape
    k = np.arange(nz)[:, None, None] + z0
    j = np.arange(ny)[None, :, None]
    i = np.arange(nx)[None, None, :]
    return ((i + j + k) & 1) == 0  # red


def _cdt(dt, arith):
    """Type the expressions are evaluated in: float64 for float32 buffers under arith="double"."""
    return np.dtype(np.float64) if arith == "double" else np.dtype(dt)


def smooth(u, f, h, dim, smoother, sweeps, cl=0.0, z0=0, gnz=None, arith="real"):
    u = u.copy()
    dt, cdt = u.dtype, _cdt(u.dtype, arith)
    fc = f.astype(cdt)

    def relax(v):  # computed in cdt, stored (rounded) in the buffer type
        return _relax(v.astype(cdt), fc, h, dim, cl, z0, gnz).astype(dt)

    for _ in range(sweeps):
        if smoother == JACOBI:
            u = relax(u)
        elif smoother == RBGS:
            red = color_mask(u.shape, z0)
            u = np.where(red, relax(u), u)
            u = np.where(~red, relax(u), u)
        else:  # lexicographic, cpu.lua:26-27 order (x outer, y, z inner)
            hsq, _ = _consts(h, dim, cdt)
            dg = diag(u.shape, h, dim, cdt, cl, z0, gnz)
            nz, ny, nx = u.shape
            z = cdt.type(0)
            U = lambda k, j, i: cdt.type(u[k, j, i])  # noqa: E731
            for i in range(nx):
                for j in range(ny):
                    for k in range(nz):
                        s = (U(k, j, i - 1) if i > 0 else z) + (U(k, j, i + 1) if i < nx - 1 else z)
                        s = s + (U(k, j - 1, i) if j > 0 else z)
                        s = s + (U(k, j + 1, i) if j < ny - 1 else z)
                        if dim == 3:
                            s = s + (U(k - 1, j, i) if k > 0 else z)
                            s = s + (U(k + 1, j, i) if k < nz - 1 else z)
                        u[k, j, i] = (fc[k, j, i] - s / hsq) / dg[k, j, i]
    return u


def residual(u, f, h, dim, cl=0.0, z0=0, gnz=None, arith="real"):
    dt, cdt = u.dtype, _cdt(u.dtype, arith)
    uc = u.astype(cdt)
    hsq, _ = _consts(h, dim, cdt)
    askew = _nbsum(uc, dim) / hsq
    return (f.astype(cdt) - (askew + diag(u.shape, h, dim, cdt, cl, z0, gnz) * uc)).astype(dt)


def restrict(r, dim, arith="real"):
    if arith == "double" and r.dtype != np.float64:
        return restrict(r.astype(np.float64), dim).astype(r.dtype)
    if dim == 2:
        s = r[:, 0::2, 0::2] + r[:, 0::2, 1::2]
        s = s + r[:, 1::2, 0::2]
        s = s + r[:, 1::2, 1::2]
        return r.dtype.type(0.25) * s
    s = r[0::2, 0::2, 0::2] + r[0::2, 0::2, 1::2]
    s = s + r[0::2, 1::2, 0::2]
    s = s + r[0::2, 1::2, 1::2]
    s = s + r[1::2, 0::2, 0::2]
    s = s + r[1::2, 0::2, 1::2]
    s = s + r[1::2, 1::2, 0::2]
    s = s + r[1::2, 1::2, 1::2]
    return r.dtype.type(0.125) * s


def restrict_fw(r, dim, clc=0.0, arith="real"):
    """Full weighting (build-defined option): the cell-centred adjoint of the linear prolongation.

    Per axis, coarse cell I gets fine cells 2I-1 .. 2I+2 as ((r_a + w_b r_b) + w_c r_c) + r_d with
    w = 3, or 3 - clc next to a box face (I = 0 for 2I, I = m-1 for 2I+1); fine cells outside the box
    are +0.  x, then y, then z; finally times 1/8^d (mgp_oracle_impl.h restrict_fw()).
    """
    if arith == "double" and r.dtype != np.float64:
        return restrict_fw(r.astype(np.float64), dim, clc).astype(r.dtype)
    dt = r.dtype.type
    w3, wf = dt(3), dt(3) - dt(clc)
    axes = (2, 1, 0) if dim == 3 else (2, 1)
    p = np.pad(r, 1) if dim == 3 else np.pad(r, ((0, 0), (1, 1), (1, 1)))
    for ax in axes:
        n = p.shape[ax] - 2
        m = n // 2
        take = lambda off: np.take(p, np.arange(m) * 2 + off, axis=ax)  # noqa: E731
        wb = np.full(m, w3, r.dtype)
        wc = np.full(m, w3, r.dtype)
        wb[0] = wf
        wc[m - 1] = wf
        shp = [1, 1, 1]
        shp[ax] = m
        wb, wc = wb.reshape(shp), wc.reshape(shp)
        s = take(0) + wb * take(1)
        s = s + wc * take(2)
        p = s + take(3)  # the axes still to be reduced keep their zero border
    scale = dt(1.0 / 512.0) if dim == 3 else dt(1.0 / 64.0)
    return scale * p


def _axis_idx(n_fine, n_coarse):
    idx = np.arange(n_fine)
    parent = idx >> 1
    nb = np.where(idx & 1, parent + 1, parent - 1)
    out = (nb < 0) | (nb >= n_coarse)
    return parent, np.clip(nb, 0, n_coarse - 1), out


def prolong(V, fine_shape, dim, kind, cl=0.0, arith="real"):
    """PC injection (cpu.lua:142-150) or cell-centred separable linear (build-defined).

    Linear: each coarse sample outside the box is -cl times the nearest inside value, with
    the factor built per axis in x, y, z order (mgp_oracle_impl.h cval()); then x-, y-, z-
    interpolation with weights 3/4 (parent) and 1/4 (neighbour).  The result is in V's type (the
    reference's real buffer vs[L], cpu-raw.lua:226).
    """
    if arith == "double" and V.dtype != np.float64:
        return prolong(V.astype(np.float64), fine_shape, dim, kind, cl).astype(V.dtype)
    nz, ny, nx = fine_shape
    if kind == PROLONG_PC:
        v = np.repeat(np.repeat(V, 2, axis=2), 2, axis=1)
        if dim == 3:
            v = np.repeat(v, 2, axis=0)
        return v
    dt = V.dtype.type
    w0, w1, c = dt(0.75), dt(0.25), dt(cl)
    cz, cy, cx = V.shape
    xi = _axis_idx(nx, cx)
    yi = _axis_idx(ny, cy)
    zi = _axis_idx(nz, cz) if dim == 3 else (np.zeros(1, np.int64),) * 2 + (np.zeros(1, bool),)

    def val(px, py, pz):
        I = xi[px][None, None, :]
        J = yi[py][None, :, None]
        K = zi[pz][:, None, None]
        s = np.ones((len(zi[0]), ny, nx), dtype=V.dtype)
        if px:
            s = np.where(xi[2][None, None, :], -c * s, s)
        if py:
            s = np.where(yi[2][None, :, None], -c * s, s)
        if pz:
            s = np.where(zi[2][:, None, None], -c * s, s)
        return s * V[K, J, I]

    if dim == 2:
        a0 = w0 * val(0, 0, 0) + w1 * val(1, 0, 0)
        a1 = w0 * val(0, 1, 0) + w1 * val(1, 1, 0)
        return w0 * a0 + w1 * a1
    a00 = w0 * val(0, 0, 0) + w1 * val(1, 0, 0)
    a10 = w0 * val(0, 1, 0) + w1 * val(1, 1, 0)
    a01 = w0 * val(0, 0, 1) + w1 * val(1, 0, 1)
    a11 = w0 * val(0, 1, 1) + w1 * val(1, 1, 1)
    b0 = w0 * a00 + w1 * a10
    b1 = w0 * a01 + w1 * a11
    return w0 * b0 + w1 * b1


def add_to(u, v, arith="real"):
    """addTo u + v (cpu-raw.lua:83-85), evaluated in the compute type and stored in u's type."""
    cdt = _cdt(u.dtype, arith)
    return (u.astype(cdt) + v.astype(cdt)).astype(u.dtype)


def err_sum(psi, old, arith="real"):
    """sum (psi - psiOld)^2 in float64 (cpu.lua:203); arith="double": each square first stored in the
    float errorBuf (cpu-raw.lua:96-100, 249-253)."""
    d = psi.astype(np.float64) - old.astype(np.float64)
    sq = d * d
    if arith == "double" and psi.dtype != np.float64:
        sq = sq.astype(psi.dtype).astype(np.float64)
    return float(np.sum(sq))


def coarse_coef(coarse_bc: int, level: int) -> float:
    """c_l of MGO_BC_CONSISTENT: (2^l - 1)/(2^l + 1); 0 on level 0 and for the reference."""
    if coarse_bc != BC_CONSISTENT or level <= 0:
        return 0.0
    p = float(2 ** level)
    return (p - 1.0) / (p + 1.0)


class Multigrid:
    """cpu.lua semantics: ``Multigrid(dim, n, ...)``; ``step()`` returns the RMS update."""

    def __init__(self, dim=2, n=(8, 8, 1), dtype=np.float64, nu1=7, nu2=7, smoother=JACOBI,
                 cycle=CYCLE_V, prolong_kind=PROLONG_PC, coarse_init=COARSE_FRESH,
                 coarse_sweeps=48, coarse_bc=BC_ZERO, restriction=RESTRICT_AVERAGE, arith="real"):
        nx, ny, nz = n
        if dim == 2:
            nz = 1
        self.dim, self.dtype = dim, np.dtype(dtype)
        self.nu1, self.nu2, self.smoother, self.cycle = nu1, nu2, smoother, cycle
        self.prolong_kind, self.coarse_init, self.coarse_sweeps = prolong_kind, coarse_init, coarse_sweeps
        self.coarse_bc = coarse_bc
        self.restriction = restriction
        self.arith = arith
        shapes = []
        s = (nz, ny, nx)
        while True:
            shapes.append(s)
            more = s[2] >= 2 and s[1] >= 2 and (dim == 2 or s[0] >= 2)
            if not more:
                break
            s = (s[0] // 2 if dim == 3 else 1, s[1] // 2, s[2] // 2)
        self.shapes = shapes
        self.V = [np.zeros(sh, self.dtype) for sh in shapes]  # warm-start buffers
        self.f = np.zeros(shapes[0], self.dtype)
        self.psi = np.zeros(shapes[0], self.dtype)

    def init_point_charge(self):
        nz, ny, nx = self.shapes[0]
        self.f[...] = 0
        c = (nz // 2 if self.dim == 3 else 0, ny // 2, nx // 2)
        self.f[c] = self.dtype.type(-1e6 / 1.0)
        self.psi = -self.f

    def _cycle(self, l, u, f, h, fcycle):
        cl = coarse_coef(self.coarse_bc, l)
        ar = self.arith
        if l == len(self.shapes) - 1:
            sweeps = 1 if u.size == 1 else self.coarse_sweeps
            return smooth(u, f, h, self.dim, self.smoother, sweeps, cl, arith=ar)
        u = smooth(u, f, h, self.dim, self.smoother, self.nu1, cl, arith=ar)
        r = residual(u, f, h, self.dim, cl, arith=ar)
        if self.restriction == RESTRICT_FULL_WEIGHTING:
            R = restrict_fw(r, self.dim, coarse_coef(self.coarse_bc, l + 1), arith=ar)
        else:
            R = restrict(r, self.dim, arith=ar)
        V = np.zeros_like(R) if self.coarse_init == COARSE_FRESH else self.V[l + 1]
        if fcycle:
            V = self._cycle(l + 1, V, R, 2 * h, True)
        V = self._cycle(l + 1, V, R, 2 * h, False)
        self.V[l + 1] = V
        u = add_to(u, prolong(V, u.shape, self.dim, self.prolong_kind, coarse_coef(self.coarse_bc, l + 1), arith=ar),
                   arith=ar)
        return smooth(u, f, h, self.dim, self.smoother, self.nu2, cl, arith=ar)

    def step(self) -> float:
        h = 1.0 / self.shapes[0][2]
        old = self.psi.copy()
        self.psi = self._cycle(0, self.psi, self.f, h, self.cycle == CYCLE_F)
        return float(np.sqrt(err_sum(self.psi, old, self.arith) / self.psi.size))


def dst_exact(f: np.ndarray, h: float, dim: int) -> np.ndarray:
    """Exact solution of the discrete system A u = f (ghost-zero Dirichlet) by DST-I.

    Eigenvalues of the 1D operator (u_{i-1} - 2u_i + u_{i+1})/h^2 with zero ghosts are
    (2cos(pi k/(n+1)) - 2)/h^2 — the same system CG solves in
    converge-multigrid-vs-krylov.lua:48-58.
    """
    from scipy.fft import dstn, idstn

    f64 = f.astype(np.float64)
    axes = (0, 1, 2) if dim == 3 else (1, 2)
    F = dstn(f64, type=1, axes=axes)
    lam = np.zeros(f64.shape)
    for ax in axes:
        n = f64.shape[ax]
        k = np.arange(1, n + 1)
        l1 = (2 * np.cos(np.pi * k / (n + 1)) - 2) / (h * h)
        shp = [1, 1, 1]
        shp[ax] = n
        lam = lam + l1.reshape(shp)
    return idstn(F / lam, type=1, axes=axes)
