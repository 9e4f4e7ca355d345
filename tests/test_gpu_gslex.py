"""GPU: cpu.lua's lexicographic Gauss-Seidel (cpu.lua:24-37, inPlaceIterativeSolver = GaussSeidel).

The reference's sweep updates u in place in ascending lexicographic order.  The GPU runs it hyperplane by
hyperplane (cells with i + j + k = s read the new values of hyperplane s - 1 and the old ones of s + 1), tiled
in tile-hyperplanes (k_gslex), which is the same arithmetic on the same operands.  Bar: psi BIT-IDENTICAL to the
oracle's sequential sweep (oracle/mgp_oracle_impl.h gslex) after single sweeps of random fields on square,
non-square, tile-sized and sub-tile levels (fp32, fp64, with and without the consistent coarse boundary), and
after whole cycles: the verdict's 2D 256^2 7+7 V-cycle (the reference configuration with GaussSeidel selected)
and 3D 32^3; err to the usual summation-order tolerance.  The cpu.lua protocol (MultigridHIP.GaussSeidel) runs it,
and red/black keeps a name of its own (MultigridHIP.RedBlackGaussSeidel)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle_lib import Oracle, coarse_coef, smooth_arr  # noqa: E402
from test_gpu_parity import REAL, _check_err, _ctx, _mg, _rand  # noqa: E402

SHAPES = [
    (2, (256, 256, 1)), (2, (64, 32, 1)), (2, (32, 128, 1)), (2, (32, 32, 1)), (2, (4, 4, 1)), (2, (1, 1, 1)),
    (3, (32, 32, 32)), (3, (16, 8, 32)), (3, (8, 8, 8)), (3, (64, 64, 64)), (3, (2, 2, 2)),
]


@pytest.mark.parametrize("dim,n", SHAPES, ids=[f"{d}d-{n[0]}x{n[1]}x{n[2]}" for d, n in SHAPES])
@pytest.mark.parametrize("real", ["double", "float"])
@pytest.mark.parametrize("level,bc", [(0, "zero"), (1, "consistent")])
def test_gslex_sweeps_match_oracle(dim, n, real, level, bc):
    if level >= 1 and min(n[:dim]) < 2:
        pytest.skip("no level 1")
    ctx = _ctx(dim=dim, n=n, real=real, smoother="gs_lex", coarse_bc=bc)
    shp = ctx.shape(level)
    u = _rand(shp, REAL[real], 11)
    f = _rand(shp, REAL[real], 12)
    ctx.set_psi(u, level)
    ctx.set_f(f, level)
    h = (2.0 ** level) / n[0]
    ref = u.copy()
    for sweeps in (1, 2):
        ctx.smooth(level, sweeps)
        ref = smooth_arr(dim, ref, f, "gs_lex", sweeps, h, coarse_coef(bc, level))
        assert np.array_equal(ctx.get_psi(level), ref)
    # it is the lexicographic sweep, not red/black: the two differ after one sweep
    rb = smooth_arr(dim, u.copy(), f, "rbgs", 1, h, coarse_coef(bc, level))
    lx = smooth_arr(dim, u.copy(), f, "gs_lex", 1, h, coarse_coef(bc, level))
    if u.size > 2:
        assert not np.array_equal(rb, lx)


CYCLES = [
    # the verdict's cases: the reference configuration (2D, Jacobi's 7+7 V-cycle, injection, ghost 0) with
    # GaussSeidel selected, at 256^2; 3D 32^3
    dict(dim=2, n=(256, 256, 1), real="double", nu1=7, nu2=7),
    dict(dim=3, n=(32, 32, 32), real="double", nu1=7, nu2=7),
    dict(dim=3, n=(32, 32, 32), real="float", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(dim=2, n=(64, 64, 1), real="float", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent", cycle="F"),
    dict(dim=3, n=(16, 16, 16), real="double", nu1=2, nu2=2, coarse_init="warm"),
    dict(dim=3, n=(32, 16, 8), real="double", nu1=3, nu2=3),
]


@pytest.mark.parametrize("cfg", CYCLES, ids=["2d256-7+7", "3d32-7+7", "3d32-f32-2+2-lin", "2d64-F", "3d16-warm",
                                             "3d-noncubic"])
def test_gslex_cycles_match_oracle(cfg):
    kw = dict(cfg, smoother="gs_lex")
    ctx = _ctx(**kw)
    ctx.init_point_charge()
    o = Oracle(**kw)
    o.init_point_charge()
    for _ in range(3):
        old = o.get(0).copy()
        e = ctx.cycle()
        eo = o.step()
        assert np.array_equal(ctx.get_psi(), o.get(0))
        _check_err(e, eo, o.get(0), old)
    assert all(lv["engine"] == "piece" for lv in ctx.levels)


def test_cpu_lua_protocol_gauss_seidel():
    """cpu.lua:56-57 with GaussSeidel selected: MultigridHIP(size, inPlaceIterativeSolver = GaussSeidel) steps
    bit-identically to the oracle's lexicographic sweep; switching to RedBlackGaussSeidel rebuilds with psi kept."""
    mg = _mg()
    s = mg.MultigridHIP(size=64, inPlaceIterativeSolver=mg.MultigridHIP.GaussSeidel)
    assert s.inPlaceIterativeSolver == mg.MultigridHIP.GaussSeidel
    o = Oracle(dim=2, n=(64, 64, 1), smoother="gs_lex")
    o.init_point_charge()
    for _ in range(3):
        s.step()
        o.step()
        assert np.array_equal(s.psi, o.get(0))
    s.inPlaceIterativeSolver = mg.MultigridHIP.RedBlackGaussSeidel
    o2 = Oracle(dim=2, n=(64, 64, 1), smoother="rbgs")
    o2.set(0, s.psi)
    o2.set(1, s.f)
    s.step()
    o2.step()
    assert np.array_equal(s.psi, o2.get(0))


@pytest.mark.parametrize("dim,n", [(2, (64, 64, 1)), (2, (32, 16, 1)), (3, (16, 16, 16))])
def test_gslex_cpu_raw_float_arithmetic(dim, n):
    """cpu-raw.lua's own GaussSeidel (cpu-raw.lua:22-32) under real = 'float': float images, every update evaluated
    in LuaJIT doubles and rounded once at the store (mgp_opts.arith = MGP_ARITH_DOUBLE): sweeps and whole cycles
    bit-identical to the oracle's arith="double" mode, and different from gpu.lua's all-float arithmetic."""
    kw = dict(dim=dim, n=n, real="float", smoother="gs_lex", nu1=7, nu2=7, coarse_init="warm")
    ctx = _ctx(arith="double", **kw)
    u = _rand(ctx.shape(0), np.float32, 31)
    f = _rand(ctx.shape(0), np.float32, 32)
    ctx.set_psi(u, 0)
    ctx.set_f(f, 0)
    ctx.smooth(0, 2)
    ref = smooth_arr(dim, u.copy(), f, "gs_lex", 2, 1.0 / n[0], 0.0, arith="double")
    assert np.array_equal(ctx.get_psi(0), ref)
    assert not np.array_equal(ref, smooth_arr(dim, u.copy(), f, "gs_lex", 2, 1.0 / n[0], 0.0))
    c2 = _ctx(arith="double", **kw)
    c2.init_point_charge()
    o = Oracle(arith="double", **kw)
    o.init_point_charge()
    for _ in range(2):
        c2.cycle()
        o.step()
        assert np.array_equal(c2.get_psi(), o.get(0))
