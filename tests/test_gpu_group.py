"""The single-process multi-GPU group (mgp_group_create): one host process, one context per rank,
the ranks' work run by one host thread per device inside the library (the Lua
host of north_star drives the node's GPUs this way).  On the one-GPU test box every rank sits on
device 0 and the group uses the loopback transport; with distinct devices it builds its RCCL
communicators with ncclCommInitAll.  Bar: the group's global psi and err == the single-domain run,
bit for bit (err to summation order)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _mg():
    import mgpoisson

    return mgpoisson


CASES = [
    ((64, 64, 128), 2, dict(real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"), None),
    ((64, 64, 256), 8, dict(real="double", smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent",
                            cycle="F", gather_cells=4096), None),
    ((128, 128, 128), 8, dict(real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
     "65536"),
    ((32, 32, 64), 2, dict(real="double", smoother="jacobi", nu1=3, nu2=3, prolong="pc", coarse_init="warm"), None),
]


@pytest.mark.parametrize("box,world,cfg,fused", CASES, ids=["w2-f32", "w8-F-f64", "w8-fused-f32", "w2-jacobi-warm"])
def test_group_equals_single_domain(box, world, cfg, fused, monkeypatch):
    mg = _mg()
    if fused:
        monkeypatch.setenv("MGP_FUSED", "1")
        monkeypatch.setenv("MGP_FUSED_MIN_CELLS", fused)
    g = mg.Group(mg.make_opts(dim=3, n=box, **cfg), world, devices=[0] * world)
    assert len(g.ranks) == world
    assert all(r.levels[0]["distributed"] for r in g.ranks)
    assert [r.levels[0]["z0"] for r in g.ranks] == [k * box[2] // world for k in range(world)]
    g.init_point_charge()
    ref = mg.Context(mg.make_opts(dim=3, n=box, **cfg))
    ref.init_point_charge()
    eg = np.concatenate([g.cycles(2), [g.cycle()]])
    er = ref.cycles(3)
    assert np.array_equal(g.get_psi(), ref.get_psi())
    np.testing.assert_allclose(eg, er, rtol=1e-12, atol=0)
    assert g.field_stats()[0] == ref.field_stats()[0]
    np.testing.assert_allclose(g.residual_norm(), ref.residual_norm(), rtol=1e-12, atol=0)
    # global field I/O round trip through the ranks' slabs
    u = np.random.default_rng(1).uniform(-1, 1, g.shape(0)).astype(g.dtype)
    g.set_field(0, u)
    assert np.array_equal(g.get_psi(), u)
    g.close()


def test_group_rejects_bad_split():
    mg = _mg()
    with pytest.raises(mg.MGPError):
        mg.Group(mg.make_opts(dim=3, n=(16, 16, 16)), 16, devices=[0] * 16)


@pytest.mark.parametrize("world", [2, 4])
def test_group_rank_failure_aborts_instead_of_hanging(world, monkeypatch):
    """a rank that fails before its exchange must not leave the other ranks blocked in it.
    One rank fails at once (test hook MGP_TEST_FAIL_RANK); the call returns the error within seconds (not the
    loopback barrier's 120 s), the group is marked unusable, and the caller's device is unchanged."""
    import time

    import torch

    mg = _mg()
    cfg = dict(real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent")
    g = mg.Group(mg.make_opts(dim=3, n=(64, 64, 128), **cfg), world, devices=[0] * world)
    g.init_point_charge()
    g.cycles(1)  # healthy first
    monkeypatch.setenv("MGP_TEST_FAIL_RANK", str(world - 1))
    t0 = time.perf_counter()
    with pytest.raises(mg.MGPError, match="injected failure"):
        g.cycles(3)
    assert time.perf_counter() - t0 < 30
    monkeypatch.delenv("MGP_TEST_FAIL_RANK")
    with pytest.raises(mg.MGPError, match="aborted"):
        g.cycle()
    assert torch.cuda.current_device() == 0
    g.close()


def test_group_debug_nan_keeps_group_usable():
    """the debugging check's "found a nan" is raised after a rank's final synchronisation, when every
    collective of the call has completed on every rank, so the group's call sequences still match: it is reported,
    and the group is not aborted (a clean call afterwards runs and equals the single domain)."""
    mg = _mg()
    cfg = dict(real="double", smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent")
    box = (32, 32, 64)
    g = mg.Group(mg.make_opts(dim=3, n=box, **cfg), 2, devices=[0, 0])
    for r in g.ranks:
        r.set_debug(1)
    g.init_point_charge()
    f = g.get_field(mg.FIELD_F)
    f[box[2] - 3, 5, 7] = np.nan  # in rank 1's slab
    g.set_field(mg.FIELD_F, f)
    with pytest.raises(mg.MGPError, match="found a nan"):
        g.cycles(1)
    g.init_point_charge()
    ref = mg.Context(mg.make_opts(dim=3, n=box, **cfg))
    ref.init_point_charge()
    np.testing.assert_allclose(g.cycles(2), ref.cycles(2), rtol=1e-12, atol=0)
    assert np.array_equal(g.get_psi(), ref.get_psi())
    g.close()
