"""GPU parity of the full-weighting restriction option (mgp_opts.restriction = MGP_RESTRICT_FULL_WEIGHTING).

north_star names "full-weighting restriction"; the reference restricts by the 2x2 cell average
(cpu.lua:127-135), which stays the default.  The option is the cell-centred adjoint of the linear
prolongation (oracle: restrict_fw in oracle/mgp_oracle_impl.h, C and NumPy bit-identical, pinned by the
adjoint and known-answer tests of tests/test_oracle.py).  Bar: psi and the restricted right-hand sides
bit-identical to the C oracle on every engine (one launch per piece, the 3D-/2D-tiled phases k_blk, the
temporally blocked k_zs, both coarse tails) and through the slab decomposition; err to summation order.
"""
import numpy as np
import pytest

from oracle_lib import Oracle, coarse_coef, residual_arr, restrict_fw_arr
from test_gpu_parity import _check_err, _loopback_run

pytestmark = pytest.mark.gpu

REAL = {"double": np.float64, "float": np.float32}


def _ctx(**kw):
    import mgpoisson

    return mgpoisson.Context(mgpoisson.make_opts(**kw))


def _n3(dim, n):
    return (n, n, n if dim == 3 else 1)


@pytest.mark.parametrize("dim,n", [(2, 8), (2, 64), (2, 256), (3, 8), (3, 32), (3, 64)])
@pytest.mark.parametrize("real", ["double", "float"])
@pytest.mark.parametrize("level,bc", [(0, "zero"), (1, "consistent"), (2, "consistent")])
def test_fw_residual_restrict_kernel(dim, n, real, level, bc):
    """mgp_residual_restrict with full weighting (vector and scalar kernels) == the oracle's r -> R."""
    ctx = _ctx(dim=dim, n=_n3(dim, n), real=real, coarse_bc=bc, restriction="full_weighting")
    if level + 1 >= len(ctx.levels):
        pytest.skip("no coarser level")
    shp = ctx.shape(level)
    rng = np.random.default_rng(31 + level)
    u = rng.uniform(-1, 1, shp).astype(REAL[real])
    f = rng.uniform(-1, 1, shp).astype(REAL[real])
    ctx.set_psi(u, level)
    ctx.set_f(f, level)
    ctx.residual_restrict(level)
    h = (2.0 ** level) / n
    ref = restrict_fw_arr(dim, residual_arr(dim, u, f, h, coarse_coef(bc, level)), coarse_coef(bc, level + 1))
    assert np.array_equal(ctx.get_f(level + 1), ref)


# engine settings: (name, env)
ENGINES = [
    ("piece", {"MGP_BLK": "0", "MGP_TAIL": "0", "MGP_FUSED": "0"}),
    ("default", {}),
    ("generic-tail", {"MGP_TAIL_CUBIC": "0"}),
    ("zs", {"MGP_FUSED": "1", "MGP_FUSED_MIN_CELLS": "65536", "MGP_YS_MIN_CELLS": "65536"}),
]

FW_CONFIGS = [
    dict(dim=3, n=(64, 64, 64), real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(dim=3, n=(128, 64, 64), real="double", smoother="rbgs", nu1=2, nu2=2, cycle="F", prolong="linear",
         coarse_bc="consistent"),
    dict(dim=3, n=(64, 64, 128), real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="zero"),
    dict(dim=3, n=(32, 32, 32), real="double", smoother="rbgs", nu1=1, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(dim=3, n=(32, 32, 32), real="double", smoother="jacobi", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(dim=2, n=(512, 512, 1), real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(dim=2, n=(256, 128, 1), real="double", smoother="rbgs", nu1=2, nu2=2, cycle="F", prolong="linear",
         coarse_bc="zero"),
    dict(dim=2, n=(1024, 1024, 1), real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
    # zs engine: level 1 (64^3, cl = 0, a fresh guess) also runs the fused full weighting (k_zs PRE, LINEAR 2, ZSRC)
    dict(dim=3, n=(128, 128, 128), real="float", smoother="rbgs", nu1=2, nu2=2, prolong="pc", coarse_bc="zero"),
]


def _id(c):
    return "-".join(f"{k}{v}" for k, v in c.items()).replace(" ", "").replace("(", "").replace(")", "").replace(",", "x")


@pytest.mark.parametrize("engine", ENGINES, ids=[e[0] for e in ENGINES])
@pytest.mark.parametrize("cfg", FW_CONFIGS, ids=_id)
def test_fw_cycles_match_oracle(cfg, engine, monkeypatch):
    name, env = engine
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    kw = dict(restriction="full_weighting", **cfg)
    ctx = _ctx(**kw)
    engines = [lv["engine"] for lv in ctx.levels]
    if name == "zs" and not (cfg["smoother"] == "rbgs" and cfg["nu1"] == cfg["nu2"] == 2 and
                             (cfg["dim"] == 3 or cfg["n"][0] >= 1024)):
        pytest.skip("the temporally blocked phases run RB-GS 2+2 (2D: rows of >= 1024 cells)")
    if name == "zs":
        assert engines[0] == "zs", engines
    if name == "piece":
        assert set(engines) == {"piece"}, engines
    o = Oracle(threads=8, **kw)
    ctx.init_point_charge()
    o.init_point_charge()
    for it in range(3):
        old = o.get(0)
        e_gpu, e_ref = ctx.cycle(), o.step()
        new = o.get(0)
        assert np.array_equal(ctx.get_psi(), new), f"psi differs after cycle {it + 1} ({name}: {engines})"
        _check_err(e_gpu, e_ref, new, old)


def test_fw_blk_levels_present():
    """The tiled one-launch phases run with full weighting (its PRE restricts inside the tile)."""
    ctx = _ctx(dim=3, n=(128, 128, 128), real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear",
               coarse_bc="consistent", restriction="full_weighting")
    assert [lv["engine"] for lv in ctx.levels][1:3] == ["blk", "blk"]


@pytest.mark.parametrize("box,world,gather,cfg,fused", [
    ((64, 64, 128), 2, 4096, dict(real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear",
                                  coarse_bc="consistent"), False),
    ((64, 64, 128), 4, 4096, dict(real="double", smoother="rbgs", nu1=2, nu2=2, prolong="linear",
                                  coarse_bc="consistent", cycle="F"), False),
    ((64, 64, 128), 2, 4096, dict(real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear",
                                  coarse_bc="consistent"), True),
    ((32, 64, 64), 2, 512, dict(real="double", smoother="jacobi", nu1=2, nu2=2, prolong="linear",
                                coarse_bc="zero"), False),
], ids=["w2-f32", "w4-F-f64", "w2-zs-f32", "w2-jacobi"])
def test_fw_slab_decomposition_loopback(box, world, gather, cfg, fused, monkeypatch):
    """Full weighting on slab levels: the residual's ghost plane comes from the z-neighbour (one exchange of
    r per restriction).  Gathered psi == the single-domain run == the oracle, bit for bit."""
    if fused:
        monkeypatch.setenv("MGP_FUSED", "1")
        monkeypatch.setenv("MGP_FUSED_MIN_CELLS", "65536")
    cfg = dict(restriction="full_weighting", **cfg)
    psi, _, dist = _loopback_run(box, world, gather, cfg, cycles=2)
    assert dist[0] and dist[1]
    single = _ctx(dim=3, n=box, gather_cells=gather, **cfg)
    single.init_point_charge()
    single.cycles(2)
    assert np.array_equal(psi, single.get_psi())
    o = Oracle(dim=3, n=box, threads=8, **cfg)
    o.init_point_charge()
    o.step()
    o.step()
    assert np.array_equal(psi, o.get(0))


@pytest.mark.parametrize("n,cycle", [((512, 512, 512), "V"), ((256, 128, 256), "F")], ids=["512-V", "256x128x256-F"])
def test_fw_fused_pre_equals_restriction_after_phase(n, cycle, monkeypatch):
    """The full weighting fused into k_zs PRE (LINEAR 2: level 0 of an fp32 box, the bench's 512^3 among them) ==
    the same phase followed by k_resfw (MGP_ZS_FWF=0, read at creation), bit for bit, on a random field."""
    kw = dict(dim=3, n=n, real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent",
              restriction="full_weighting", cycle=cycle)
    if n[0] < 512:
        monkeypatch.setenv("MGP_FUSED_MIN_CELLS", "65536")
    rng = np.random.default_rng(7)
    f = rng.uniform(-1, 1, (n[2], n[1], n[0])).astype(np.float32)
    out = []
    for fwf in ("1", "0"):
        monkeypatch.setenv("MGP_ZS_FWF", fwf)
        ctx = _ctx(**kw)
        assert ctx.levels[0]["engine"] == "zs"
        ctx.set_f(f, 0)
        errs = [ctx.cycle() for _ in range(2)]
        out.append((ctx.get_psi(), errs))
        ctx.close()
    assert np.array_equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1]
