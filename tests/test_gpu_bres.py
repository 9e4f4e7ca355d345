"""GPU: fused passes of the per-piece red/black levels below the finest (round 6).

- k_bres: the pre-smoothing's last black half-sweep + calcResidual + reduceResidual in one pass.  A red/black
  sweep's black half reads only red cells, so one pass can relax the black cells, form the residual of both
  colours and restrict it (cpu.lua:40-54 update, cpu.lua:108-135).
- k_rbsweep (opt-in, MGP_RBSWEEP=1: measured slower than the k_half pair): a whole red/black sweep in one
  out-of-place pass (u -> t, swapped), the red cells the black half reads recomputed at the block edge; only the
  last sweep of a run stores its red cells.
Bar: psi bit-identical to the oracle and to the separate pieces (MGP_BRES=0 MGP_RBSWEEP=0) after whole cycles, on
cubic / square / non-cubic boxes, fp32 / fp64, both coarse boundaries, V and F, fresh and warm coarse guesses, odd
and even sweep counts; and single smoothing calls on levels 1 and 2 against the oracle's sweeps."""
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
    dict(dim=3, n=(32, 32, 32), real="float", prolong="linear", coarse_bc="consistent", smoother="rbgs", nu1=4, nu2=3),
    dict(dim=2, n=(64, 64, 1), real="float", prolong="linear", coarse_bc="consistent", smoother="rbgs", nu1=1, nu2=1,
         cycle="F"),
]


@pytest.mark.parametrize("cfg", CASES, ids=["3d64-f32", "3d64-f64-F", "3d-noncubic", "3d32-warm", "2d256", "2d-3+1",
                                            "3d-4+3", "2d-1+1-F"])
def test_bres_cycles_match_oracle_and_pieces(cfg, monkeypatch):
    monkeypatch.setenv("MGP_TAIL", "0")  # every level below the finest runs its own pieces
    monkeypatch.setenv("MGP_BLK", "0")
    monkeypatch.setenv("MGP_FUSED", "0")
    monkeypatch.setenv("MGP_RBSWEEP", "1")  # (opt-in: measured slower than the k_half pair)
    ctx = _ctx(**cfg)
    ctx.init_point_charge()
    monkeypatch.setenv("MGP_BRES", "0")
    monkeypatch.setenv("MGP_RBSWEEP", "0")
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


@pytest.mark.parametrize("dim,n", [(3, (32, 32, 32)), (3, (16, 32, 64)), (2, (128, 128, 1)), (2, (64, 16, 1))])
@pytest.mark.parametrize("real", ["float", "double"])
@pytest.mark.parametrize("level", [1, 2])
def test_rbsweep_smoothing_calls_match_oracle(dim, n, real, level, monkeypatch):
    """mgp_smooth on a level below the finest runs k_rbsweep for every sweep (the last one stores both colours):
    1, 2 and 3 sweeps of random fields equal the oracle's red/black sweeps with the consistent boundary."""
    from oracle_lib import coarse_coef, smooth_arr
    from test_gpu_parity import REAL, _rand

    monkeypatch.setenv("MGP_RBSWEEP", "1")
    ctx = _ctx(dim=dim, n=n, real=real, smoother="rbgs", nu1=2, nu2=2, coarse_bc="consistent")
    shp = ctx.shape(level)
    u = _rand(shp, REAL[real], 21)
    f = _rand(shp, REAL[real], 22)
    ctx.set_psi(u, level)
    ctx.set_f(f, level)
    ref = u
    h = (2.0 ** level) / n[0]
    for sweeps in (1, 2, 3):
        ctx.smooth(level, sweeps)
        ref = smooth_arr(dim, ref, f, "rbgs", sweeps, h, coarse_coef("consistent", level))
        assert np.array_equal(ctx.get_psi(level), ref)
