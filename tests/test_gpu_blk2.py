"""GPU: PRE of two consecutive small 2D levels in one launch (k_blk2_pre, round 6).

A V-cycle runs level l + 1's pre-smoothing right after level l's restriction (cpu.lua:138-139), so one workgroup
can smooth its fine box, restrict the fine residuals onto its coarse box (the coarse tile and its halo), and smooth
and restrict that too (cpu.lua:40-54, 108-135): one launch for two k_blk PRE launches.
k_blk2_post likewise runs POST of level l + 1 and then of level l (prolong_correct + nu2 sweeps each, cpu.lua:142-158).
Bar: psi, and every level's u and f, bit-identical to the oracle and to one k_blk launch per level (MGP_BLK2=0) after
whole cycles, on square and non-square boxes, fp32 (32- and 16-cell tiles) and fp64 (16-cell tiles), both coarse
boundaries and prolongations, fresh and warm coarse guesses, 1 and 2 pre-/post-sweeps, V- and F-cycles (the F-cycle's
first descent keeps one launch per level)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle_lib import Oracle  # noqa: E402
from test_gpu_parity import _check_err, _ctx  # noqa: E402

RB = dict(smoother="rbgs", nu1=2, nu2=2)
CASES = [
    dict(dim=2, n=(512, 512, 1), real="float", prolong="linear", coarse_bc="consistent", **RB),
    dict(dim=2, n=(1024, 1024, 1), real="float", prolong="linear", coarse_bc="consistent", **RB),
    dict(dim=2, n=(2048, 2048, 1), real="float", prolong="linear", coarse_bc="consistent", **RB),
    dict(dim=2, n=(512, 256, 1), real="float", prolong="pc", coarse_bc="zero", **RB),
    dict(dim=2, n=(512, 512, 1), real="float", prolong="linear", coarse_bc="consistent", coarse_init="warm", **RB),
    dict(dim=2, n=(1024, 1024, 1), real="float", prolong="linear", coarse_bc="consistent", smoother="rbgs", nu1=1,
         nu2=3),
    dict(dim=2, n=(1024, 1024, 1), real="float", prolong="linear", coarse_bc="consistent", cycle="F", **RB),
    dict(dim=2, n=(512, 512, 1), real="double", prolong="linear", coarse_bc="consistent", **RB),
    dict(dim=2, n=(2048, 1024, 1), real="double", prolong="pc", coarse_bc="zero", smoother="rbgs", nu1=2, nu2=1),
]


@pytest.mark.parametrize("cfg", CASES, ids=["512", "1024", "2048", "512x256-pc-zero", "512-warm", "1024-1+3",
                                            "1024-F", "512-f64", "2048x1024-f64-2+1"])
def test_blk2_cycles_match_oracle_and_single_level_launches(cfg, monkeypatch):
    monkeypatch.setenv("MGP_BLK2", "1")
    ctx = _ctx(**cfg)
    ctx.init_point_charge()
    monkeypatch.setenv("MGP_BLK2", "0")
    ref = _ctx(**cfg)
    ref.init_point_charge()
    o = Oracle(**cfg)
    o.init_point_charge()
    for _ in range(2):
        old = o.get(0).copy()
        e, er, eo = ctx.cycle(), ref.cycle(), o.step()
        assert np.array_equal(ctx.get_psi(), o.get(0))
        assert np.array_equal(ref.get_psi(), o.get(0))
        assert e == er
        _check_err(e, eo, o.get(0), old)
    # every level's u and f equal the unpaired path's
    for lv in range(1, len(ctx.levels)):
        assert np.array_equal(ctx.get_psi(lv), ref.get_psi(lv)), lv
        assert np.array_equal(ctx.get_f(lv), ref.get_f(lv)), lv
