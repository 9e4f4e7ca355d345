"""CPU tests of the engine planning (host logic, no device): mgp_plan reports, per level, how mgp_create
would run its smoothing phases — one launch per piece, the one-launch coarse tail, the temporally blocked
phases (k_zs; "zpost": POST only) or the tiled one-launch phases (k_blk).  The GPU tests prove every engine bit-exact against
the oracle; these pin which engine each BASELINE workload gets."""
import pytest

from mgpoisson import _lib

import mgpoisson as mg

NS = dict(smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent")


def engines(**kw):
    return [d["engine"] for d in _lib.plan(mg.make_opts(**kw))]


def test_bench_config_512_cube():
    """configs[2]: k_zs on 512^3, 256^3 PRE per piece and POST k_zs, 128^3 per piece, 64^3 and 32^3 tiled, 16^3 .. 1
    in the tail."""
    for real in ("float", "double"):
        assert engines(dim=3, n=(512, 512, 512), real=real, **NS) == ["zs", "zpost", "piece", "blk", "blk"] + ["tail"] * 5


def test_2d_config_4096():
    """configs[1]: 4096^2 temporally blocked (k_ys, rows streamed), 2048^2 per piece, 1024^2 .. 128^2 tiled (32 x 32
    tiles), 64^2 .. 1 in the tail; fp64 too."""
    for real in ("float", "double"):
        assert engines(dim=2, n=(4096, 4096, 1), real=real, **NS) == ["zs", "piece"] + ["blk"] * 4 + ["tail"] * 7


def test_config5_rank_slab_f_cycle():
    """configs[4] rank slab 4096 x 4096 x 512: three temporally blocked levels, 512 x 512 x 64 with POST temporally
    blocked, tiled 128 x 128 x 16 and 64 x 64 x 8, the tail from 32 x 32 x 4."""
    e = engines(dim=3, n=(4096, 4096, 512), real="float", cycle="F", **NS)
    assert e == ["zs"] * 3 + ["zpost", "piece"] + ["blk"] * 2 + ["tail"] * 3


def test_weak_scaling_rank_of_eight():
    """bench --gpus 8 (512 x 512 x 4096): distributed levels never tile (their halos come from the
    neighbours), the first replicated level after the all-gather does."""
    p = _lib.plan(mg.make_opts(dim=3, n=(512, 512, 4096), real="float", rank=3, world=8, comm_id=b"\0" * 128, **NS))
    assert [d["engine"] for d in p] == ["zs", "zpost"] + ["piece"] * 3 + ["blk"] + ["tail"] * 4
    assert all(d["distributed"] for d in p[:5]) and not any(d["distributed"] for d in p[5:])


@pytest.mark.parametrize("kw", [
    dict(smoother="jacobi", prolong="pc"),  # Jacobi: no RB-GS engines, the generic tail
    dict(smoother="rbgs", nu1=3, nu2=1),    # k_zs needs 2 + 2, k_blk at most 2 sweeps per phase
])
def test_engines_follow_the_smoother(kw):
    e = engines(dim=3, n=(128, 128, 128), real="float", **kw)
    assert e == ["piece"] * 3 + ["tail"] * 5


def test_engine_switches(monkeypatch):
    monkeypatch.setenv("MGP_BLK", "0")
    monkeypatch.setenv("MGP_FUSED", "0")
    assert engines(dim=3, n=(512, 512, 512), real="float", **NS) == ["piece"] * 5 + ["tail"] * 5
    monkeypatch.setenv("MGP_TAIL", "0")
    assert engines(dim=3, n=(512, 512, 512), real="float", **NS) == ["piece"] * 10
