"""GPU: the pre-smoothing's last black half-sweep fused with calcResidual + reduceResidual (k_bres).

A red/black sweep's black half reads only red cells, so one pass can relax the black cells, form the residual
of both colours and restrict it (cpu.lua:40-54 update, cpu.lua:108-135); it replaces k_half (black) +
k_resrestrict_s on every replicated per-piece level of a red/black cycle with >= 2 pre-sweeps and the average
restriction.  Bar: psi bit-identical to the oracle and to the unfused pieces (MGP_BRES=0) after whole cycles, on
cubic / square / non-cubic boxes, fp32 / fp64, both coarse boundaries, V and F, fresh and warm coarse guesses."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle_lib import Oracle  # noqa: E402
from test_gpu_parity import _check_err, _ctx  # noqa: E402

RB = dict(smoother="rbgs", nu1=2, nu2=2)
CASES = [
    dict(dim=3, n=(64, 64, 64), real="float", prolong="linear", coarse_bc="consistent", **RB),
    dict(dim=3, n=(64, 64, 64), real="double", prolong="linear", coarse_bc="consistent", cycle="F", **RB),
    dict(dim=3, n=(64, 32, 16), real="double", prolong="pc", coarse_bc="zero", **RB),
    dict(dim=3, n=(32, 32, 32), real="float", prolong="linear", coarse_bc="consistent", coarse_init="warm", **RB),
    dict(dim=2, n=(256, 256, 1), real="float", prolong="linear", coarse_bc="consistent", **RB),
    dict(dim=2, n=(128, 64, 1), real="double", prolong="pc", coarse_bc="zero", smoother="rbgs", nu1=3, nu2=1),
]


@pytest.mark.parametrize("cfg", CASES, ids=["3d64-f32", "3d64-f64-F", "3d-noncubic", "3d32-warm", "2d256", "2d-3+1"])
def test_bres_cycles_match_oracle_and_pieces(cfg, monkeypatch):
    monkeypatch.setenv("MGP_TAIL", "0")  # every level below the finest runs its own pieces
    monkeypatch.setenv("MGP_BLK", "0")
    monkeypatch.setenv("MGP_FUSED", "0")
    ctx = _ctx(**cfg)
    ctx.init_point_charge()
    monkeypatch.setenv("MGP_BRES", "0")
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


def test_bres_default_engines_512_box_levels():
    """With the default engines the 512^3 box runs k_bres on its per-piece PRE levels (256^3 zpost, 128^3):
    one cycle of a 128^3 box (its 64^3 and 32^3 levels per piece / tiled) still equals the oracle."""
    cfg = dict(dim=3, n=(128, 128, 128), real="float", prolong="linear", coarse_bc="consistent", **RB)
    ctx = _ctx(**cfg)
    ctx.init_point_charge()
    o = Oracle(**cfg)
    o.init_point_charge()
    ctx.cycle()
    o.step()
    assert np.array_equal(ctx.get_psi(), o.get(0))
