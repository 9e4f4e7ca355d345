"""GPU parity of cpu-raw.lua's real = 'float' arithmetic (mgp_opts.arith = MGP_ARITH_DOUBLE).

cpu-raw.lua keeps float images (cpu-raw.lua:142-153) but evaluates every kernel body in LuaJIT numbers
(doubles), so each expression is double and only the store into a float buffer rounds: Jacobi
(:34-44), calcResidual (:46-57), reduceResidual (:59-63), expandResidual / addTo (:65-85), and
calcFrobErr's float errorBuf (:96-100) summed in double (:249-254).  gpu.lua's `real = float` rounds
every operation instead (gpu.lua:32) — the library's default (arith = MGP_ARITH_REAL).

Bar: psi BIT-IDENTICAL to the oracle's arith="double" mode (oracle/mgp_oracle_impl.h, MGO_S fd) after
every piece and every cycle, and to the committed golden fixtures of MultigridCPURaw(n, 'float'):run()
(tests/golden/rawf2d_n*.npz).  err: the GPU sums the float-rounded squares in a fixed tree order, the
oracle sequentially — the same 1e-12 relative bound as tests/test_gpu_parity.py.
"""
import glob
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle_lib import (Oracle, coarse_coef, err_arr, prolong_correct_arr, residual_arr, residual_sumsq_arr,  # noqa: E402
                        restrict_arr, restrict_fw_arr, smooth_arr)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
RAW = dict(real="float", arith="double")


def _mg():
    import mgpoisson

    return mgpoisson


def _ctx(**kw):
    mg = _mg()
    return mg.Context(mg.make_opts(**kw))


def _n3(dim, n):
    return (n, n, n if dim == 3 else 1)


def _rand(shape, seed):
    return np.random.default_rng(seed).uniform(-1.0, 1.0, size=shape).astype(np.float32)


def _err_ok(e_gpu, psi_new, psi_old):
    """sqrt(sum float(d^2) / N), d in double (cpu-raw.lua:96-100, 249-254), against a pairwise numpy sum."""
    d = psi_new.astype(np.float64) - psi_old.astype(np.float64)
    sq = (d * d).astype(np.float32).astype(np.float64)
    ref = float(np.sqrt(np.sum(sq) / d.size))
    assert abs(e_gpu - ref) <= 1e-12 * abs(ref), (e_gpu, ref)


def test_positional_float_run_is_cpu_raw(capsys):
    """MG(256, 'float'):run() — the positional protocol's float follows cpu-raw.lua: both cycles bit-exact
    against the oracle's arith="double" (warm Vs, Jacobi 7+7, injection, cpu-raw.lua:142-258), and not equal
    to gpu.lua's float arithmetic."""
    mg = _mg()
    s = mg.MultigridHIPRaw(256, "float")
    assert s.arith == "double"
    assert all(lv["engine"] == "piece" for lv in s.ctx.levels)
    o = Oracle(dim=2, n=(256, 256, 1), coarse_init="warm", **RAW)
    o.init_point_charge()
    olds, errs_ref = [], []
    for _ in range(2):
        olds.append(o.get(0))
        errs_ref.append(o.step())
    errs = s.run()
    assert len(errs) == 2
    assert np.array_equal(s.psi, o.get(0))
    out = capsys.readouterr().out.splitlines()
    assert out[0].split() == ["#iter", "err"] and len(out) == 3
    for e, r in zip(errs, errs_ref):
        assert abs(e - r) <= 4 * 256 * 256 * 2.0 ** -53 * abs(r)
    g = mg.MultigridHIPRaw(256, "float", arith="real")
    g.quiet = True
    g.run()
    assert not np.array_equal(g.psi, s.psi)  # the two reference float semantics differ


GOLDEN_RAW = sorted(glob.glob(os.path.join(GOLDEN, "rawf2d_n*.npz")))


@pytest.mark.parametrize("path", GOLDEN_RAW, ids=lambda p: os.path.basename(p)[:-4])
def test_rawfloat_golden_fixtures(path):
    """10 outer iterations of MultigridCPURaw(n, 'float') against the committed fixtures (psi after 1, 2, 10)."""
    z = np.load(path, allow_pickle=False)
    cfg = json.loads(str(z["config"]))
    dim, n = cfg.pop("dim"), tuple(cfg.pop("n"))
    ctx = _ctx(dim=dim, n=n, **cfg)
    ctx.init_point_charge()
    assert np.array_equal(ctx.get_f(), z["f"])
    prev = ctx.get_psi()
    for it in range(1, 11):
        e = ctx.cycle()
        psi = ctx.get_psi()
        if it in (1, 2, 10):
            assert np.array_equal(psi, z[f"psi{it}"]), f"cycle {it}"
        _err_ok(e, psi, prev)
        assert abs(e - z["errs"][it - 1]) <= max(1e-12, 4 * psi.size * 2.0 ** -53) * abs(z["errs"][it - 1])
        prev = psi


RAW_CYCLES = [
    dict(dim=2, n=64, smoother="jacobi", coarse_init="fresh"),
    dict(dim=2, n=128, smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(dim=2, n=64, smoother="rbgs", nu1=2, nu2=2, cycle="F", prolong="linear", coarse_bc="consistent",
         restriction="full_weighting"),
    dict(dim=3, n=32, smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(dim=3, n=16, smoother="jacobi", prolong="pc", coarse_init="warm"),
    dict(dim=3, n=32, smoother="rbgs", nu1=2, nu2=2, cycle="F", prolong="linear", coarse_bc="consistent",
         restriction="full_weighting"),
]


@pytest.mark.parametrize("cfg", RAW_CYCLES, ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
def test_rawfloat_cycles_match_oracle(cfg):
    cfg = dict(cfg)
    dim, n = cfg.pop("dim"), cfg.pop("n")
    ctx = _ctx(dim=dim, n=_n3(dim, n), **RAW, **cfg)
    o = Oracle(dim=dim, n=_n3(dim, n), **RAW, **cfg)
    ctx.init_point_charge()
    o.init_point_charge()
    for it in range(3):
        old = o.get(0)
        e = ctx.cycle()
        o.step()
        new = o.get(0)
        assert np.array_equal(ctx.get_psi(), new), f"cycle {it + 1}"
        _err_ok(e, new, old)
        # the oracle sums sequentially: its rounding bound ~4 N eps
        assert abs(e - err_arr(new, old, arith="double")) <= max(1e-12, 4 * new.size * 2.0 ** -53) * e


@pytest.mark.parametrize("smoother", ["jacobi", "rbgs"])
@pytest.mark.parametrize("dim,n", [(2, 64), (3, 16)])
@pytest.mark.parametrize("level,bc", [(0, "zero"), (1, "consistent")])
def test_rawfloat_pieces(smoother, dim, n, level, bc):
    """Each twoGrid piece on a level: smoothing, residual + restriction, prolongation + correction, and the
    rs / errorBuf views (cpu-raw.lua:155-171, 96-100), bit for bit against the oracle's double arithmetic."""
    ctx = _ctx(dim=dim, n=_n3(dim, n), smoother=smoother, coarse_bc=bc, prolong="linear", **RAW)
    shp = ctx.shape(level)
    u, f = _rand(shp, 1), _rand(shp, 2)
    h = (2.0 ** level) / n
    cl = coarse_coef(bc, level)
    ctx.set_psi(u, level)
    ctx.set_f(f, level)
    ctx.smooth(level, 2)
    us = smooth_arr(dim, u, f, smoother, 2, h, cl, arith="double")
    assert np.array_equal(ctx.get_psi(level), us)
    assert np.array_equal(ctx.get_field(2, level), residual_arr(dim, us, f, h, cl, arith="double"))  # rs
    rn, fn = ctx.residual_norm(level)
    ref = residual_sumsq_arr(dim, us, f, h, cl, arith="double")
    assert abs(rn * rn - ref) <= 1e-12 * ref
    ctx.residual_restrict(level)
    R = restrict_arr(dim, residual_arr(dim, us, f, h, cl, arith="double"), arith="double")
    assert np.array_equal(ctx.get_f(level + 1), R)
    V = _rand(ctx.shape(level + 1), 3)
    ctx.set_psi(V, level + 1)
    ctx.prolong_correct(level)
    assert np.array_equal(ctx.get_psi(level), prolong_correct_arr(dim, us, V, "linear", coarse_coef(bc, level + 1),
                                                                  arith="double"))


def test_rawfloat_full_weighting_piece():
    ctx = _ctx(dim=3, n=(32, 32, 32), smoother="rbgs", coarse_bc="consistent", restriction="full_weighting", **RAW)
    u, f = _rand(ctx.shape(1), 4), _rand(ctx.shape(1), 5)
    ctx.set_psi(u, 1)
    ctx.set_f(f, 1)
    ctx.residual_restrict(1)
    h, cl = 2.0 / 32, coarse_coef("consistent", 1)
    r = residual_arr(3, u, f, h, cl, arith="double")
    R = restrict_fw_arr(3, r, coarse_coef("consistent", 2), arith="double")
    assert np.array_equal(ctx.get_f(2), R)
    assert not np.array_equal(R, restrict_fw_arr(3, r, coarse_coef("consistent", 2)))


def test_rawfloat_error_buffer_view():
    """errorBuf after an outer iteration = float((psi - psiOld)^2) evaluated in double (cpu-raw.lua:96-100)."""
    ctx = _ctx(dim=2, n=(64, 64, 1), coarse_init="warm", **RAW)
    ctx.init_point_charge()
    old = ctx.get_psi()
    ctx.cycle()
    new = ctx.get_psi()
    d = new.astype(np.float64) - old.astype(np.float64)
    assert np.array_equal(ctx.get_field(5), (d * d).astype(np.float32))
    assert np.array_equal(ctx.get_field(4), old)  # psiOld


@pytest.mark.parametrize("world", [2, 4])
def test_rawfloat_slab_loopback(world):
    """The slab decomposition (deep halos, agglomeration) under the double arithmetic: gathered psi equals
    the single domain bit for bit."""
    import threading

    mg = _mg()
    box, gather = (32, 32, 64), 512
    cfg = dict(smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent", **RAW)
    single = _ctx(dim=3, n=box, **cfg)
    single.init_point_charge()
    single.cycles(2)
    ref = single.get_psi()
    lb = mg.Loopback(world)
    out, errors = [None] * world, []

    def rank_main(r):
        try:
            ctx = mg.Context(mg.make_opts(dim=3, n=box, rank=r, world=world, gather_cells=gather, device=0,
                                          comm_id=b"\0" * 128, **cfg), loopback=lb)
            ctx.init_point_charge()
            ctx.cycles(2)
            out[r] = ctx.get_psi()
            ctx.close()
        except Exception as e:  # noqa: BLE001 - surfaced below
            errors.append((r, repr(e)))

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    lb.close()
    assert not errors, errors
    assert np.array_equal(np.concatenate(out, axis=0), ref)


def test_rawfloat_rejects_coarse_engine():
    mg = _mg()
    ctx = _ctx(dim=2, n=(64, 64, 1), **RAW)
    with pytest.raises(mg.MGPError) as ei:
        ctx.set_coarse_level(8)
    assert "per piece" in str(ei.value)
