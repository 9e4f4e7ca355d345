"""GPU tests of the 3D-tiled one-launch smoothing phases of small levels (k_blk).

Below ~128^3 a cycle's pieces are launch-bound, so a level's PRE phase (nu1 RB-GS sweeps +
calcResidual + reduceResidual, cpu.lua:108-135) and POST phase (expandResidual + addTo + nu2 sweeps,
cpu.lua:142-158) each run as one launch with the tile and its halo in LDS.  The bar is the same as
for every other engine: psi bit-identical to the C oracle and to one launch per piece (MGP_BLK=0) on
every level, err to summation order.
"""
import numpy as np
import pytest

from oracle_lib import Oracle
from test_gpu_parity import _check_err

pytestmark = pytest.mark.gpu


def _mg():
    import mgpoisson

    return mgpoisson


def _ctx(**kw):
    mg = _mg()
    return mg.Context(mg.make_opts(**kw))


BLK_CONFIGS = [
    # the bench's family: levels 64^3 and 32^3 tiled, 16^3 and below in the coarse tail
    dict(n=(64, 64, 64), real="float", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(n=(128, 128, 128), real="float", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(n=(64, 64, 64), real="double", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent", cycle="F"),
    # non-cubic boxes (tiles clipped per axis), injection, zero coarse boundary, warm coarse guesses
    dict(n=(128, 64, 32), real="double", nu1=2, nu2=2, prolong="pc", coarse_bc="zero"),
    dict(n=(32, 64, 128), real="float", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent", coarse_init="warm"),
    # one sweep per phase / unequal phases
    dict(n=(64, 64, 64), real="float", nu1=1, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(n=(64, 32, 64), real="double", nu1=2, nu2=1, prolong="linear", coarse_bc="consistent", cycle="F"),
    # no coarse tail: tiled levels down to 4 x 4 x 4 (tiles smaller than the halo, every cell on the box)
    dict(n=(32, 32, 32), real="float", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent", tail=0),
    dict(n=(64, 16, 32), real="double", nu1=1, nu2=1, prolong="pc", coarse_bc="consistent", tail=0),
    # 2D: 32 x 32 tiles (configs[1] family: RB-GS 2+2, linear, consistent coarse boundary)
    dict(dim=2, n=(512, 512, 1), real="float", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(dim=2, n=(256, 256, 1), real="double", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent", cycle="F"),
    dict(dim=2, n=(256, 128, 1), real="float", nu1=1, nu2=2, prolong="pc", coarse_bc="zero", coarse_init="warm"),
    dict(dim=2, n=(128, 128, 1), real="double", nu1=2, nu2=1, prolong="linear", coarse_bc="consistent", tail=0),
]


def _id(c):
    return "-".join(f"{k}{v}" for k, v in c.items()).replace(" ", "").replace("(", "").replace(")", "").replace(",", "x")


@pytest.mark.parametrize("cfg", BLK_CONFIGS, ids=_id)
def test_block_phases_match_oracle(cfg, monkeypatch):
    cfg = dict(cfg)
    tail = cfg.pop("tail", 1)
    kw = dict(smoother="rbgs", **cfg)
    kw.setdefault("dim", 3)
    if not tail:
        monkeypatch.setenv("MGP_TAIL", "0")
    monkeypatch.setenv("MGP_BLK", "1")
    a = _ctx(**kw)
    monkeypatch.setenv("MGP_BLK", "0")
    b = _ctx(**kw)
    assert any(lv["engine"] == "blk" for lv in a.levels), a.levels
    assert not any(lv["engine"] == "blk" for lv in b.levels)
    assert a.levels[0]["engine"] != "blk"
    o = Oracle(threads=8, **kw)
    for x in (a, b, o):
        x.init_point_charge()
    for it in range(3):
        old = o.get(0)
        ea, eb, eo = a.cycle(), b.cycle(), o.step()
        new = o.get(0)
        assert np.array_equal(a.get_psi(), new), f"tiled psi differs from the oracle after cycle {it + 1}"
        assert np.array_equal(b.get_psi(), new), f"per-piece psi differs from the oracle after cycle {it + 1}"
        _check_err(ea, eo, new, old)
        assert abs(ea - eb) <= 1e-12 * abs(eb)
    for level in range(len(a.levels)):
        assert np.array_equal(a.get_psi(level), b.get_psi(level)), f"psi level {level}"
        assert np.array_equal(a.get_f(level), b.get_f(level)), f"f level {level}"


def test_block_graph_replay_equals_eager(monkeypatch):
    """The tiled phases swap u / t per phase: graph replay (cached per pointer state) == eager."""
    kw = dict(dim=3, n=(128, 128, 128), real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear",
              coarse_bc="consistent", cycle="F")
    g = _ctx(**kw)
    monkeypatch.setenv("MGP_GRAPH", "0")
    e = _ctx(**kw)
    assert [lv["engine"] for lv in g.levels][1:3] == ["blk", "blk"]
    g.init_point_charge()
    e.init_point_charge()
    eg = np.concatenate([g.cycles(3), g.cycles(4)])
    ee = np.concatenate([e.cycles(3), e.cycles(4)])
    assert np.array_equal(g.get_psi(), e.get_psi())
    assert np.array_equal(eg, ee)


def test_block_levels_of_the_2d_config():
    """4096^2 RB-GS 2+2 (configs[1]): 4096^2 temporally blocked (k_ys), 2048^2 per piece, 1024^2 .. 128^2 tiled,
    64^2 and below in the tail."""
    ctx = _ctx(dim=2, n=(4096, 4096, 1), real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear",
               coarse_bc="consistent")
    eng = [lv["engine"] for lv in ctx.levels]
    assert eng[:6] == ["zs", "piece", "blk", "blk", "blk", "blk"] and eng[6] == "tail", eng


def test_block_levels_of_the_bench_config():
    """512^3 fp32 RB-GS 2+2: level 0 temporally blocked, 256^3 PRE per piece and POST temporally blocked, 128^3 per
    piece, 64^3 and 32^3 tiled, then the tail."""
    ctx = _ctx(dim=3, n=(512, 512, 512), real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear",
               coarse_bc="consistent")
    eng = [lv["engine"] for lv in ctx.levels]
    assert eng[:5] == ["zs", "zpost", "piece", "blk", "blk"] and eng[5] == "tail", eng


FRESH_CONFIGS = [
    dict(dim=3, n=(64, 64, 64), real="double", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(dim=3, n=(128, 64, 32), real="float", nu1=2, nu2=2, prolong="pc", coarse_bc="zero", cycle="F"),
    dict(dim=3, n=(32, 64, 128), real="float", nu1=1, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(dim=2, n=(256, 256, 1), real="double", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent", cycle="F"),
    dict(dim=2, n=(128, 128, 1), real="float", nu1=1, nu2=1, prolong="pc", coarse_bc="zero"),
]


@pytest.mark.parametrize("cfg", FRESH_CONFIGS, ids=_id)
def test_fresh_first_sweep_matches_oracle(cfg, monkeypatch):
    """k_fresh (the first RB-GS sweep of a fresh coarse guess from f alone, cpu.lua:138) == the two
    half-sweeps reading a zero black input == the oracle, on every level (tiled phases off, so every
    level above the tail sweeps per piece)."""
    kw = dict(smoother="rbgs", **cfg)
    monkeypatch.setenv("MGP_BLK", "0")
    monkeypatch.setenv("MGP_FRESH", "1")
    a = _ctx(**kw)
    monkeypatch.setenv("MGP_FRESH", "0")
    b = _ctx(**kw)
    o = Oracle(threads=8, **kw)
    for x in (a, b, o):
        x.init_point_charge()
    for it in range(3):
        old = o.get(0)
        ea, eb, eo = a.cycle(), b.cycle(), o.step()
        new = o.get(0)
        assert np.array_equal(a.get_psi(), new), f"psi differs from the oracle after cycle {it + 1}"
        assert np.array_equal(b.get_psi(), new)
        _check_err(ea, eo, new, old)
    for level in range(len(a.levels)):
        assert np.array_equal(a.get_psi(level), b.get_psi(level)), f"psi level {level}"


CUBIC_TAIL_CONFIGS = [
    dict(n=(64, 64, 64), real="float", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(n=(32, 32, 32), real="double", nu1=2, nu2=2, prolong="pc", coarse_bc="zero", cycle="F", coarse_init="warm"),
    dict(n=(128, 128, 128), real="float", nu1=1, nu2=3, prolong="linear", coarse_bc="consistent", cycle="F"),
    dict(n=(32, 32, 32), real="double", nu1=2, nu2=1, prolong="linear", coarse_bc="consistent", coarse_sweeps=3),
    # 2D: levels 64^2 .. 1
    dict(dim=2, n=(256, 256, 1), real="float", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(dim=2, n=(128, 128, 1), real="double", nu1=2, nu2=2, prolong="pc", coarse_bc="zero", cycle="F", coarse_init="warm"),
    # the slab tails: a configs[3] / configs[4] rank slab's ratio 8:8:1 ends in 32 x 32 x 4 ..
    # 8 x 8 x 1 (64 cells, coarse_sweeps sweeps); the weak-scaling box 512 x 512 x 512 N in 8 x 8 x 8 N .. 1 x 1 x N
    dict(n=(256, 256, 32), real="float", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent", tail=(32, 32, 4)),
    dict(n=(128, 128, 16), real="double", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent", cycle="F",
         tail=(32, 32, 4)),
    dict(n=(64, 64, 512), real="float", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent", tail=(8, 8, 64)),
    dict(n=(32, 32, 64), real="double", nu1=2, nu2=2, prolong="pc", coarse_bc="zero", cycle="F", coarse_init="warm",
         tail=(8, 8, 16)),
    dict(n=(64, 64, 256), real="float", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent", cycle="F",
         restriction="full_weighting", tail=(8, 8, 32)),
]


@pytest.mark.parametrize("cfg", CUBIC_TAIL_CONFIGS, ids=_id)
def test_cubic_tail_equals_generic_tail_and_oracle(cfg, monkeypatch):
    """k_tail_c (compile-time tail shapes: 16^3 .. 1 in 3D, 64^2 .. 1 in 2D, the slab tails 32 x 32 x 4 .. 8 x 8 x 1
    and 8 x 8 x 8N .. 1 x 1 x N; zero-halo LDS levels) == the generic k_tail == the oracle: psi and f bit-identical
    on every level."""
    kw = dict(smoother="rbgs", **cfg)
    kw.setdefault("dim", 3)
    top = kw.pop("tail", (16, 16, 16) if kw["dim"] == 3 else (64, 64, 1))
    monkeypatch.setenv("MGP_TAIL_CUBIC", "1")
    a = _ctx(**kw)
    monkeypatch.setenv("MGP_TAIL_CUBIC", "0")
    b = _ctx(**kw)
    tl = [(lv["nx"], lv["ny"], lv["nz_global"]) for lv in a.levels if lv["tail"]]
    nl = min(top[:kw["dim"]]).bit_length()
    assert tl == [tuple(max(1, t >> l) if (d < kw["dim"]) else 1 for d, t in enumerate(top)) for l in range(nl)]
    o = Oracle(threads=8, **kw)
    for x in (a, b, o):
        x.init_point_charge()
    for it in range(3):
        old = o.get(0)
        monkeypatch.setenv("MGP_TAIL_CUBIC", "1")
        ea = a.cycle()
        monkeypatch.setenv("MGP_TAIL_CUBIC", "0")
        eb = b.cycle()
        eo = o.step()
        new = o.get(0)
        assert np.array_equal(a.get_psi(), new), f"psi differs from the oracle after cycle {it + 1}"
        assert np.array_equal(b.get_psi(), new)
        _check_err(ea, eo, new, old)
    for level in range(len(a.levels)):
        assert np.array_equal(a.get_psi(level), b.get_psi(level)), f"psi level {level}"
        assert np.array_equal(a.get_f(level), b.get_f(level)), f"f level {level}"


POST1_CONFIGS = [
    dict(dim=3, n=(64, 64, 64), real="double", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(dim=3, n=(128, 64, 32), real="float", nu1=2, nu2=2, prolong="pc", coarse_bc="zero", cycle="F"),
    dict(dim=3, n=(32, 64, 128), real="float", nu1=1, nu2=3, prolong="linear", coarse_bc="consistent",
         coarse_init="warm"),
    dict(dim=2, n=(256, 256, 1), real="float", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(dim=2, n=(256, 128, 1), real="double", nu1=2, nu2=1, prolong="linear", coarse_bc="consistent", cycle="F"),
]


@pytest.mark.parametrize("cfg", POST1_CONFIGS, ids=_id)
def test_post_first_half_sweep_matches_oracle(cfg, monkeypatch):
    """k_post1 (prolongation + correction fused into the first post red half-sweep; u + P V of the
    black cells never stored) == prolong_correct + smooth == the oracle, psi on every level, err to
    summation order (tiled phases off, so every level above the tail runs per piece; 2D level 0 too)."""
    kw = dict(smoother="rbgs", **cfg)
    monkeypatch.setenv("MGP_BLK", "0")
    monkeypatch.setenv("MGP_POST1", "1")
    a = _ctx(**kw)
    monkeypatch.setenv("MGP_POST1", "0")
    b = _ctx(**kw)
    o = Oracle(threads=8, **kw)
    for x in (a, b, o):
        x.init_point_charge()
    for it in range(3):
        old = o.get(0)
        ea, eb, eo = a.cycle(), b.cycle(), o.step()
        new = o.get(0)
        assert np.array_equal(a.get_psi(), new), f"psi differs from the oracle after cycle {it + 1}"
        assert np.array_equal(b.get_psi(), new)
        _check_err(ea, eo, new, old)
    for level in range(len(a.levels)):
        assert np.array_equal(a.get_psi(level), b.get_psi(level)), f"psi level {level}"


@pytest.mark.parametrize("cfg", FRESH_CONFIGS + [
    dict(dim=3, n=(64, 64, 64), real="float", nu1=2, nu2=1, prolong="pc", coarse_bc="consistent", coarse_init="warm"),
], ids=_id)
def test_black_only_prolongation_matches_oracle(cfg, monkeypatch):
    """The cycle's prolongation corrects only the black cells before a red/black post-smoothing (its red
    half-sweep replaces every red cell without reading it): == correcting both colours == the oracle."""
    kw = dict(smoother="rbgs", **cfg)
    monkeypatch.setenv("MGP_BLK", "0")
    monkeypatch.setenv("MGP_POST_BLACK", "1")
    a = _ctx(**kw)
    monkeypatch.setenv("MGP_POST_BLACK", "0")
    b = _ctx(**kw)
    o = Oracle(threads=8, **kw)
    for x in (a, b, o):
        x.init_point_charge()
    for it in range(3):
        old = o.get(0)
        ea, eb, eo = a.cycle(), b.cycle(), o.step()
        new = o.get(0)
        assert np.array_equal(a.get_psi(), new), f"psi differs from the oracle after cycle {it + 1}"
        assert np.array_equal(b.get_psi(), new)
        _check_err(ea, eo, new, old)
    for level in range(len(a.levels)):
        assert np.array_equal(a.get_psi(level), b.get_psi(level)), f"psi level {level}"
