"""CPU tests of the oracle itself: two independent restatements agree bit for bit, and both
are pinned by known-answer tests and the committed golden fixtures.

The reference cannot be executed here (Lua is absent), so parity with the reference is
"unpinned" beyond these known answers; see DESIGN.md §Oracle.
"""
import glob
import hashlib
import json
import os

import numpy as np
import pytest

import mgp_oracle_np as N
from oracle_lib import Oracle, coarse_coef, prolong_correct_arr, residual_arr, restrict_arr, restrict_fw_arr, smooth_arr

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _np_model(cfg):
    dt = np.float64 if cfg.get("real", "double") == "double" else np.float32
    codes = dict(smoother={"jacobi": 0, "rbgs": 1, "gs_lex": 2}, cycle={"V": 0, "F": 1}, prolong={"pc": 0, "linear": 1},
                 coarse_init={"fresh": 0, "warm": 1}, coarse_bc={"zero": 0, "consistent": 1})
    return N.Multigrid(cfg["dim"], cfg["n"], dt, cfg.get("nu1", 7), cfg.get("nu2", 7),
                       codes["smoother"][cfg.get("smoother", "jacobi")], codes["cycle"][cfg.get("cycle", "V")],
                       codes["prolong"][cfg.get("prolong", "pc")], codes["coarse_init"][cfg.get("coarse_init", "fresh")],
                       coarse_bc=codes["coarse_bc"][cfg.get("coarse_bc", "zero")],
                       restriction={"average": 0, "full_weighting": 1}[cfg.get("restriction", "average")],
                       arith=cfg.get("arith", "real"))


CROSS = [
    dict(dim=2, n=(16, 16, 1)),
    dict(dim=2, n=(16, 16, 1), coarse_init="warm"),
    dict(dim=2, n=(16, 16, 1), real="float"),
    dict(dim=2, n=(32, 16, 1), smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(dim=2, n=(16, 16, 1), smoother="rbgs", nu1=2, nu2=2, cycle="F", prolong="linear", coarse_bc="consistent", real="float"),
    dict(dim=2, n=(8, 8, 1), smoother="gs_lex", nu1=2, nu2=2),
    dict(dim=3, n=(8, 8, 8), smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(dim=3, n=(8, 8, 16), smoother="rbgs", nu1=2, nu2=2, cycle="F", prolong="linear", coarse_bc="consistent", real="float"),
    dict(dim=3, n=(8, 8, 8), smoother="jacobi", prolong="pc"),
    # the full-weighting restriction option (build-defined, north_star)
    dict(dim=2, n=(32, 16, 1), smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent",
         restriction="full_weighting"),
    dict(dim=2, n=(16, 16, 1), restriction="full_weighting", real="float"),
    dict(dim=3, n=(8, 8, 16), smoother="rbgs", nu1=2, nu2=2, cycle="F", prolong="linear", coarse_bc="consistent",
         restriction="full_weighting"),
    dict(dim=3, n=(8, 8, 8), smoother="rbgs", nu1=2, nu2=2, prolong="linear", real="float", restriction="full_weighting"),
    # cpu-raw.lua's real = 'float' (float buffers, double expressions, float errorBuf)
    dict(dim=2, n=(16, 16, 1), real="float", arith="double", coarse_init="warm"),
    dict(dim=2, n=(32, 32, 1), real="float", arith="double"),
    dict(dim=2, n=(16, 8, 1), real="float", arith="double", smoother="rbgs", nu1=2, nu2=2, prolong="linear",
         coarse_bc="consistent", cycle="F"),
    dict(dim=2, n=(8, 8, 1), real="float", arith="double", smoother="gs_lex", nu1=2, nu2=2),
    dict(dim=3, n=(8, 8, 16), real="float", arith="double", smoother="rbgs", nu1=2, nu2=2, prolong="linear",
         coarse_bc="consistent", restriction="full_weighting"),
    dict(dim=3, n=(8, 8, 8), real="float", arith="double", smoother="jacobi", prolong="pc"),
]


@pytest.mark.parametrize("cfg", CROSS, ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
def test_c_and_numpy_restatements_bit_identical(cfg):
    o = Oracle(**cfg)
    m = _np_model(cfg)
    o.init_point_charge()
    m.init_point_charge()
    for _ in range(3):
        ec, en = o.step(), m.step()
        assert np.array_equal(o.get(0).ravel(), m.psi.ravel())
        assert abs(ec - en) <= 1e-13 * abs(ec)


def test_first_jacobi_sweep_closed_form_2d():
    """SURVEY §8c KAT 2: from psi0 = -f one Jacobi sweep gives 2.5e5 h^2 at the charge,
    2.5e5 at its 4 neighbours and exactly 0 elsewhere (n = 8)."""
    n, h = 8, 1.0 / 8
    o = Oracle(dim=2, n=(n, n, 1))
    o.init_point_charge()
    u = smooth_arr(2, o.get(0), o.get(1), "jacobi", 1, h)
    c = n // 2
    assert u[c, c] == 2.5e5 * h * h == 3906.25
    for dj, di in ((0, 1), (0, -1), (1, 0), (-1, 0)):
        assert u[c + dj, c + di] == 2.5e5
    mask = np.ones_like(u, bool)
    mask[c, c] = False
    for dj, di in ((0, 1), (0, -1), (1, 0), (-1, 0)):
        mask[c + dj, c + di] = False
    assert np.all(u[mask] == 0)


def test_first_jacobi_sweep_closed_form_3d():
    n, h = 8, 1.0 / 8
    o = Oracle(dim=3, n=(n, n, n))
    o.init_point_charge()
    u = smooth_arr(3, o.get(0), o.get(1), "jacobi", 1, h)
    c = n // 2
    assert u[c, c, c] == pytest.approx(1e6 * h * h / 6, rel=1e-15)
    for d in ((1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)):
        assert u[c + d[0], c + d[1], c + d[2]] == pytest.approx(1e6 / 6, rel=1e-15)
    assert np.count_nonzero(u) == 7


@pytest.mark.parametrize("dim", [2, 3])
def test_one_cell_coarse_solve(dim):
    """SURVEY §8c KAT 1 / cpu.lua:76-93: u = f / (-2 dim / h^2) exactly on a 1-cell grid."""
    shape = (1,) * dim
    for h in (1.0, 0.5, 0.125):
        f = np.full(shape, -3.0)
        u = smooth_arr(dim, np.full(shape, 123.0), f, "jacobi", 1, h)
        assert u.ravel()[0] == -3.0 / (-2 * dim / (h * h))


def test_err_sequence_fresh_vs_warm_n8():
    """SURVEY §8c KAT 4: cycle 1 identical, cycle 2 splits by coarse-guess semantics."""
    f = Oracle(dim=2, n=(8, 8, 1), coarse_init="fresh")
    w = Oracle(dim=2, n=(8, 8, 1), coarse_init="warm")
    f.init_point_charge()
    w.init_point_charge()
    e1f, e1w = f.step(), w.step()
    assert e1f == e1w
    assert e1f == pytest.approx(122091.06275197188, rel=1e-14)
    assert f.step() == pytest.approx(6789.948050838726, rel=1e-14)
    assert w.step() == pytest.approx(6828.1698388918103, rel=1e-14)


def test_warm_start_diverges_n64():
    """SURVEY §8c KAT 5 (test-gpu-obj.lua:3 'diverging'): the persistent-Vs semantics grow at n >= 32."""
    w = Oracle(dim=2, n=(64, 64, 1), coarse_init="warm")
    f = Oracle(dim=2, n=(64, 64, 1), coarse_init="fresh")
    w.init_point_charge()
    f.init_point_charge()
    ew = [w.step() for _ in range(30)]
    ef = [f.step() for _ in range(30)]
    assert ew[-1] > ew[10]  # growing
    assert ef[-1] < ef[10]  # fresh keeps contracting


def _dst(o, dim, n):
    f = o.get(1)
    shp = f.shape if dim == 3 else (1,) + f.shape
    return N.dst_exact(f.reshape(shp).astype(np.float64), 1.0 / n[0], dim).reshape(f.shape)


def test_reference_path_converges_to_dst_solution():
    """SURVEY §8c KAT 3: cpu.lua's iteration (fresh V, Jacobi 7+7, PC) converges to A^-1 f."""
    from oracle_lib import lib
    import ctypes

    n = (32, 32, 1)
    o = Oracle(dim=2, n=n)
    o.init_point_charge()
    errs = np.zeros(3000)
    it = lib.mgo_solve(o.h, 3000, 1e-10, errs.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    assert errs[it - 1] < 1e-10
    ex = _dst(o, 2, n)
    assert np.max(np.abs(o.get(0) - ex)) < 1e-7 * np.max(np.abs(ex))


@pytest.mark.parametrize("cfg", [
    dict(dim=2, n=(64, 64, 1), smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(dim=2, n=(64, 64, 1), smoother="rbgs", nu1=2, nu2=2, cycle="F", prolong="linear", coarse_bc="consistent"),
    dict(dim=3, n=(16, 16, 16), smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(dim=3, n=(16, 16, 64), smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
], ids=["2dV", "2dF", "3dV", "3dV-box"])
def test_north_star_family_converges_to_dst(cfg):
    """Build-defined smoothers/cycles share the reference's fixed point A^-1 f (relative L2 <= 1e-10)."""
    o = Oracle(**cfg)
    o.init_point_charge()
    for _ in range(15):
        o.step()
    ex = _dst(o, cfg["dim"], cfg["n"])
    assert np.linalg.norm(o.get(0) - ex) <= 1e-10 * np.linalg.norm(ex)


def test_consistent_bc_level0_is_reference_operator():
    assert coarse_coef("consistent", 0) == 0.0
    assert coarse_coef("consistent", 1) == pytest.approx(1 / 3)
    assert coarse_coef("zero", 5) == 0.0
    rng = np.random.default_rng(0)
    u, f = rng.standard_normal((16, 16)), rng.standard_normal((16, 16))
    assert np.array_equal(residual_arr(2, u, f, 1 / 16, coarse_coef("consistent", 0)), residual_arr(2, u, f, 1 / 16))


def test_pieces_match_numpy():
    rng = np.random.default_rng(1)
    for dim, shp in ((2, (16, 32)), (3, (8, 16, 8))):
        u, f = rng.standard_normal(shp), rng.standard_normal(shp)
        s3 = shp if dim == 3 else (1,) + shp
        for cl in (0.0, 1 / 3):
            r = residual_arr(dim, u, f, 0.25, cl)
            assert np.array_equal(r.reshape(s3), N.residual(u.reshape(s3), f.reshape(s3), 0.25, dim, cl))
        R = restrict_arr(dim, r)
        assert np.array_equal(R.reshape(tuple(s // 2 for s in s3) if dim == 3 else (1,) + R.shape),
                              N.restrict(r.reshape(s3), dim))
        V = rng.standard_normal(R.shape)
        for kind in ("pc", "linear"):
            up = prolong_correct_arr(dim, u, V, kind, 1 / 3)
            Vs = V.reshape(tuple(s // 2 for s in s3) if dim == 3 else (1,) + V.shape)
            ref = u.reshape(s3) + N.prolong(Vs, s3, dim, {"pc": 0, "linear": 1}[kind], 1 / 3)
            assert np.array_equal(up.reshape(s3), ref)


GOLDEN_FILES = sorted(glob.glob(os.path.join(GOLDEN, "*.npz")))


def test_golden_manifest_hashes():
    with open(os.path.join(GOLDEN, "MANIFEST.json")) as fh:
        man = json.load(fh)
    assert len(man) == len(GOLDEN_FILES) > 0
    for p in GOLDEN_FILES:
        with open(p, "rb") as fh:
            assert hashlib.sha256(fh.read()).hexdigest() == man[os.path.basename(p)]["sha256"]


@pytest.mark.parametrize("path", GOLDEN_FILES, ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_reproduces_golden(path):
    z = np.load(path, allow_pickle=False)
    cfg = json.loads(str(z["config"]))
    cfg["n"] = tuple(cfg["n"])
    o = Oracle(**cfg)
    o.init_point_charge()
    assert np.array_equal(o.get(1), z["f"])
    errs = []
    for it in range(1, 11):
        errs.append(o.step())
        if it in (1, 2, 10):
            assert np.array_equal(o.get(0), z[f"psi{it}"])
    np.testing.assert_allclose(errs, z["errs"], rtol=1e-13, atol=0)


# ---- full-weighting restriction (build-defined option; north_star "full-weighting restriction") ----

@pytest.mark.parametrize("dim,shape", [(2, (16, 32)), (2, (2, 2)), (3, (8, 16, 4)), (3, (2, 2, 2)), (3, (16, 16, 16))])
@pytest.mark.parametrize("real", [np.float64, np.float32])
@pytest.mark.parametrize("clc", [0.0, 1 / 3, 7 / 9])
def test_full_weighting_c_equals_numpy(dim, shape, real, clc):
    r = np.random.default_rng(5).standard_normal(shape).astype(real)
    s3 = shape if dim == 3 else (1,) + shape
    R = restrict_fw_arr(dim, r, clc)
    Rn = N.restrict_fw(r.reshape(s3), dim, clc)
    assert np.array_equal(R.reshape(Rn.shape).view(np.uint8), np.ascontiguousarray(Rn).view(np.uint8))


@pytest.mark.parametrize("dim,shape", [(2, (16, 32)), (3, (8, 16, 4)), (3, (4, 4, 4))])
@pytest.mark.parametrize("clc", [0.0, 1 / 3, 7 / 9])
def test_full_weighting_is_adjoint_of_linear_prolongation(dim, shape, clc):
    """R = 2^-dim P^T: <R r, V> 2^dim == <r, P V> for the linear P with the same coarse coefficient."""
    rng = np.random.default_rng(6)
    r = rng.standard_normal(shape)
    V = rng.standard_normal(tuple(s // 2 for s in shape))
    PV = prolong_correct_arr(dim, np.zeros(shape), V, "linear", clc)
    lhs = float(np.sum(restrict_fw_arr(dim, r, clc) * V)) * 2 ** dim
    rhs = float(np.sum(r * PV))
    assert abs(lhs - rhs) <= 1e-12 * max(1.0, abs(rhs))


def test_full_weighting_known_answers():
    """Interior coarse cells of a constant field are that constant (weights (1,3,3,1)/8 per axis); a corner
    coarse cell with zero ghosts keeps 7/8 per axis (the fine cell outside contributes +0)."""
    for dim, shape in ((2, (16, 16)), (3, (8, 8, 8))):
        R = restrict_fw_arr(dim, np.ones(shape), 0.0)
        inner = R[(slice(1, -1),) * dim]
        assert np.all(inner == 1.0)
        assert R[(0,) * dim] == (7 / 8) ** dim
        # with the consistent boundary coefficient c, the face weight is 3 - c: (7 - c) / 8 per face axis
        c = 1 / 3
        Rc = restrict_fw_arr(dim, np.ones(shape), c)
        assert Rc[(0,) * dim] == pytest.approx(((7 - c) / 8) ** dim, rel=1e-15)


@pytest.mark.parametrize("cfg", [
    dict(dim=2, n=(64, 64, 1), smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(dim=2, n=(64, 64, 1), smoother="rbgs", nu1=2, nu2=2, cycle="F", prolong="linear", coarse_bc="zero"),
    dict(dim=3, n=(16, 16, 16), smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent"),
    dict(dim=3, n=(32, 32, 32), smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="zero"),
], ids=["2dV-consistent", "2dF-zero", "3dV-consistent", "3dV-zero"])
def test_full_weighting_converges_to_dst(cfg):
    """The full-weighting option shares the fixed point A^-1 f (DST-I exact solution)."""
    o = Oracle(restriction="full_weighting", threads=4, **cfg)
    o.init_point_charge()
    errs = [o.step() for _ in range(25)]
    ex = _dst(o, cfg["dim"], cfg["n"])
    assert np.linalg.norm(o.get(0) - ex) <= 1e-9 * np.linalg.norm(ex)
    assert errs[-1] < errs[5] * 1e-6


def test_full_weighting_rescues_the_zero_boundary_v_cycle():
    """2D 256^2 RB-GS 2+2 V-cycle with linear P and ghost-0 coarse levels: the 2x2 average diverges
    (SURVEY §7 [probe]), full weighting converges (update-RMS contraction ~0.81 per cycle)."""
    kw = dict(dim=2, n=(256, 256, 1), smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="zero", threads=4)
    a, f = Oracle(**kw), Oracle(restriction="full_weighting", **kw)
    a.init_point_charge()
    f.init_point_charge()
    ea = [a.step() for _ in range(14)]
    ef = [f.step() for _ in range(14)]
    assert ea[-1] > ea[-2]
    assert ef[-1] < 0.9 * ef[-2] and ef[-1] < 1e-2 * ef[0]


# ---- cpu-raw.lua's real = 'float' (arith="double"): float buffers, double expressions ----

def test_cpu_raw_float_differs_from_gpu_lua_float():
    """The two reference fp32 semantics disagree: gpu.lua rounds every operation to float (gpu.lua:32),
    cpu-raw.lua evaluates in LuaJIT doubles and rounds at each store (cpu-raw.lua:34-63).  Both stay within
    fp32 accuracy of the fp64 run."""
    kw = dict(dim=2, n=(64, 64, 1), coarse_init="warm")
    a, b, d = Oracle(real="float", **kw), Oracle(real="float", arith="double", **kw), Oracle(real="double", **kw)
    for o in (a, b, d):
        o.init_point_charge()
        o.step()
        o.step()
    pa, pb, pd = a.get(0).astype(np.float64), b.get(0).astype(np.float64), d.get(0)
    assert not np.array_equal(pa, pb)
    for p in (pa, pb):
        assert np.linalg.norm(p - pd) <= 1e-5 * np.linalg.norm(pd)


def test_cpu_raw_float_pieces_round_once():
    """Per piece, arith="double" equals the fp64 expression rounded once to float (cpu-raw.lua:34-85)."""
    from oracle_lib import err_arr
    rng = np.random.default_rng(11)
    u = rng.standard_normal((16, 16)).astype(np.float32)
    f = rng.standard_normal((16, 16)).astype(np.float32)
    h = 1 / 16
    assert np.array_equal(smooth_arr(2, u, f, "jacobi", 1, h, arith="double"),
                          smooth_arr(2, u.astype(np.float64), f.astype(np.float64), "jacobi", 1, h).astype(np.float32))
    r = residual_arr(2, u, f, h, arith="double")
    assert np.array_equal(r, residual_arr(2, u.astype(np.float64), f.astype(np.float64), h).astype(np.float32))
    assert np.array_equal(restrict_arr(2, r, arith="double"),
                          restrict_arr(2, r.astype(np.float64)).astype(np.float32))
    V = rng.standard_normal((8, 8)).astype(np.float32)
    assert np.array_equal(prolong_correct_arr(2, u, V, "pc", arith="double"), prolong_correct_arr(2, u, V, "pc"))
    # errorBuf is a float image: each square rounded to float before the double sum (cpu-raw.lua:249-253)
    d = u.astype(np.float64) - f.astype(np.float64)
    ref = np.sqrt(sum(float(np.float32(x)) for x in (d * d).ravel()) / d.size)
    assert err_arr(u, f, arith="double") == pytest.approx(ref, rel=1e-15)
    assert err_arr(u, f, arith="double") != err_arr(u, f)


def test_cpu_raw_float_first_sweep_closed_form():
    """SURVEY §8c KAT 2 holds for cpu-raw's float run too: the first Jacobi sweep values are exact floats."""
    n, h = 8, 1.0 / 8
    o = Oracle(dim=2, n=(n, n, 1), real="float", arith="double")
    o.init_point_charge()
    u = smooth_arr(2, o.get(0), o.get(1), "jacobi", 1, h, arith="double")
    c = n // 2
    assert u[c, c] == np.float32(3906.25) and u[c, c + 1] == np.float32(2.5e5)


def test_harness_cpu_column_runs_without_gpu(tmp_path):
    """The TSV harness (test/test.lua:8-63) with only the plugged-in CPU column needs no device."""
    import harness_columns
    from mgpoisson import harness

    harness.register_column("cpu-raw", harness_columns.CpuRaw)
    out = tmp_path / "cpu-vs-gpu.txt"
    rows = harness.bench(4, 5, tries=2, cols=("cpu-raw",), out=str(out), quiet=True)
    lines = out.read_text().splitlines()
    assert lines[0] == "#size\tcpu-raw" and [int(l.split("\t")[0]) for l in lines[1:]] == [16, 32]
    assert all(r[1] > 0 for r in rows)
    # the column is cpu-raw.lua's run(): 2 outer iterations from the warm-start semantics
    s = harness_columns.CpuRaw(8)
    s.quiet = True
    e = s.run()
    assert len(e) == 2 and e[0] == pytest.approx(122091.06275197188, rel=1e-14)
    assert e[1] == pytest.approx(6828.1698388918103, rel=1e-14)
