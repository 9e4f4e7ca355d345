"""GPU tests of the round-2 boundary additions and of the BASELINE configs 4/5 rank slabs.

* plane-range I/O and the device-side field fingerprint (mgp_get_planes / mgp_field_stats);
* the residual norm ||f - A u|| (north star "wavefront-level reductions for the residual norm")
  against the C oracle's calcResidual (cpu.lua:108-123);
* lazy coarse-guess zeroing with nu1 = 0 and mgp_two_grid leaving the solver's own state alone;
* one rank's slab of BASELINE configs[3] (2048 x 2048 x 256) and configs[4] (4096 x 4096 x 512 fp32
  F-cycle, 8.6e9 cells > 2^31): the temporally blocked phases against MGP_FUSED=0 bit for bit,
  compared through the 64-bit fingerprint (34 GB per field cannot come to the host).
"""
import numpy as np
import pytest

from oracle_lib import Oracle, coarse_coef, residual_arr

pytestmark = pytest.mark.gpu

REAL = {"double": np.float64, "float": np.float32}
M64 = (1 << 64) - 1


def _mg():
    import mgpoisson

    return mgpoisson


def _ctx(**kw):
    mg = _mg()
    return mg.Context(mg.make_opts(**kw))


def _rand(shape, dtype, seed):
    return np.random.default_rng(seed).uniform(-1.0, 1.0, size=shape).astype(dtype)


def _mix64(z):
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def fingerprint(arr, z0=0):
    """Host restatement of mgp_field_stats' hash: sum mod 2^64 of mix64(bits ^ mix64(global index))."""
    a = np.ascontiguousarray(arr)
    bits = a.view(np.uint32 if a.dtype == np.float32 else np.uint64).ravel().astype(object)
    nplane = a.shape[-1] * a.shape[-2] if a.ndim == 3 else a.size
    base = z0 * nplane
    h = 0
    for i, b in enumerate(bits):
        h = (h + _mix64(int(b) ^ _mix64(base + i))) & M64
    return h


@pytest.mark.parametrize("dim,box,real", [(3, (16, 8, 4), "float"), (2, (16, 16, 1), "double"), (3, (8, 4, 8), "double")])
def test_field_stats_match_host_restatement(dim, box, real):
    ctx = _ctx(dim=dim, n=box, real=real)
    u = _rand(ctx.shape(0), REAL[real], 3)
    ctx.set_psi(u)
    h, s, q, mx = ctx.field_stats()
    assert h == fingerprint(u)
    d = u.astype(np.float64)
    assert abs(s - d.sum()) <= 1e-12 * np.abs(d).sum()
    assert abs(q - (d * d).sum()) <= 1e-12 * (d * d).sum()
    assert mx == np.abs(d).max()
    u2 = u.copy()
    u2.ravel()[5] = np.nextafter(u2.ravel()[5], np.inf)  # one ulp in one cell changes the hash
    ctx.set_psi(u2)
    assert ctx.field_stats()[0] != h


@pytest.mark.parametrize("real", ["float", "double"])
def test_planes_io_roundtrip(real):
    ctx = _ctx(dim=3, n=(64, 32, 16), real=real, smoother="rbgs", nu1=2, nu2=2)
    u = _rand(ctx.shape(0), REAL[real], 4)
    ctx.set_psi(u)
    assert np.array_equal(ctx.get_planes(0, 3, 5), u[3:8])
    w = _rand((4, 32, 64), REAL[real], 5)
    ctx.set_planes(0, 9, w)
    u[9:13] = w
    assert np.array_equal(ctx.get_psi(), u)
    with pytest.raises(_mg().MGPError):
        ctx.get_planes(0, 14, 3)


@pytest.mark.parametrize("dim,n,level,bc", [(2, 64, 0, "zero"), (2, 128, 1, "consistent"), (3, 32, 0, "zero"),
                                            (3, 64, 1, "consistent"), (3, 8, 2, "consistent")])
@pytest.mark.parametrize("real", ["double", "float"])
def test_residual_norm_matches_oracle(dim, n, level, bc, real):
    """||f - A u||_2 and ||f||_2 on the device vs the oracle's residual array summed in fp64."""
    ctx = _ctx(dim=dim, n=(n, n, n if dim == 3 else 1), real=real, coarse_bc=bc)
    shp = ctx.shape(level)
    u = _rand(shp, REAL[real], 7)
    f = _rand(shp, REAL[real], 8)
    ctx.set_psi(u, level)
    ctx.set_f(f, level)
    r, fn = ctx.residual_norm(level)
    ref = residual_arr(dim, u, f, (2.0 ** level) / n, coarse_coef(bc, level)).astype(np.float64)
    assert abs(r - np.sqrt((ref * ref).sum())) <= 1e-12 * r
    assert abs(fn - np.sqrt((f.astype(np.float64) ** 2).sum())) <= 1e-12 * fn


def test_residual_norm_converges():
    """Relative residual ||r|| / ||f|| of the bench configuration drops by orders of magnitude."""
    ctx = _ctx(dim=3, n=(64, 64, 64), real="double", smoother="rbgs", nu1=2, nu2=2, prolong="linear",
               coarse_bc="consistent", cycle="F")
    ctx.init_point_charge()
    r0, f0 = ctx.residual_norm()
    ctx.cycles(12)
    r1, f1 = ctx.residual_norm()
    assert f0 == f1 == 1e6
    assert r1 / f1 < 1e-8 * (r0 / f0)


@pytest.mark.parametrize("kw", [
    dict(dim=2, n=(256, 256, 1), real="double", prolong="linear", coarse_bc="consistent"),
    dict(dim=3, n=(64, 64, 64), real="float", prolong="linear", coarse_bc="consistent"),
    dict(dim=3, n=(64, 64, 64), real="double", prolong="pc", cycle="F"),
], ids=["2d-256", "3d-64-f32", "3d-64-F-f64"])
def test_fresh_guess_with_nu1_zero_matches_oracle(kw):
    """RB-GS, fresh coarse guess and nu1 = 0 — the restriction reads a zero guess, not
    last cycle's; psi bit-identical to the oracle on every cycle."""
    kw = dict(smoother="rbgs", nu1=0, nu2=2, coarse_init="fresh", **kw)
    ctx = _ctx(**kw)
    o = Oracle(**kw)
    ctx.init_point_charge()
    o.init_point_charge()
    for it in range(3):
        ctx.cycle()
        o.step()
        assert np.array_equal(ctx.get_psi(), o.get(0)), f"cycle {it + 1}"


@pytest.mark.parametrize("real,smoother", [("double", "jacobi"), ("float", "rbgs")])
def test_two_grid_leaves_solver_state(real, smoother):
    """twoGrid(h, u, f, L) on caller buffers of the finest size must not replace the
    solver's psi and RHS (cpu-raw.lua:186 works on the buffers passed in)."""
    kw = dict(dim=2, n=(64, 64, 1), real=real, smoother=smoother, nu1=2, nu2=2)
    a, b = _ctx(**kw), _ctx(**kw)
    a.init_point_charge()
    b.init_point_charge()
    a.cycles(2)
    b.cycles(2)
    u = _rand((64, 64), REAL[real], 9)
    f = _rand((64, 64), REAL[real], 10)
    a.two_grid(1.0 / 64, u, f, 64)
    assert np.array_equal(a.get_f(), b.get_f())
    assert np.array_equal(a.get_psi(), b.get_psi())
    assert list(a.cycles(2)) == list(b.cycles(2))
    assert np.array_equal(a.get_psi(), b.get_psi())
    with pytest.raises(ValueError):
        a.two_grid(1.0 / 64, u, f[:10], 64)


def _slab_run(box, cycle, cycles, fused, monkeypatch):
    monkeypatch.setenv("MGP_FUSED", "1" if fused else "0")
    kw = dict(dim=3, n=box, real="float", smoother="rbgs", nu1=2, nu2=2, cycle=cycle, prolong="linear",
              coarse_bc="consistent")
    ctx = _ctx(**kw)
    try:
        ctx.init_point_charge()
        # the point charge sits where the init kernel (grid-stride past 2^32 slots) put it
        z = box[2] // 2
        pl = ctx.get_planes(1, z - 1, 3)
        assert pl[1, box[1] // 2, box[0] // 2] == -1e6 and np.count_nonzero(pl) == 1
        if fused:
            ctx.timing(True)
        errs = ctx.cycles(cycles)
        if fused:
            t = ctx.timing_read()
            ctx.timing(False)
            assert t["fused_pre"][1] >= cycles and t["fused_post"][1] >= cycles, t
        stats = ctx.field_stats()
        r, fnorm = ctx.residual_norm()
        mid = ctx.get_planes(0, z - 2, 4)
        return errs, stats, r / fnorm, mid
    finally:
        ctx.close()


@pytest.mark.slow
@pytest.mark.parametrize("box,cycle,cycles", [((2048, 2048, 256), "V", 2), ((4096, 4096, 512), "F", 2)],
                         ids=["config4-rank-slab", "config5-rank-slab"])
def test_baseline_rank_slab_fused_equals_unfused(box, cycle, cycles, monkeypatch):
    """One rank's slab of configs[3] / configs[4] on one GPU (world = 1: the slab's z faces are the box
    faces).  The temporally blocked path equals one launch per piece bit for bit (device fingerprint of
    psi, err sequence to summation order, the middle planes bit-exact), and the cycles converge."""
    a = _slab_run(box, cycle, cycles, True, monkeypatch)
    b = _slab_run(box, cycle, cycles, False, monkeypatch)
    assert a[1][0] == b[1][0], "psi fingerprints differ"
    assert np.array_equal(a[3], b[3])
    np.testing.assert_allclose(a[0], b[0], rtol=1e-12, atol=0)
    assert all(np.isfinite(a[0])) and a[0][1] < a[0][0]
    assert a[2] < 1.0


def test_loopback_w8_fused_config4_aspect(monkeypatch):
    """Loopback world 8 at config 4's per-rank aspect (8:8:1 slabs: 256 x 256 x 32 per rank), k_zs forced on
    the distributed levels: gathered psi == the single-domain run bit for bit."""
    import threading

    monkeypatch.setenv("MGP_FUSED", "1")
    monkeypatch.setenv("MGP_FUSED_MIN_CELLS", "65536")
    mg = _mg()
    box, world = (256, 256, 256), 8
    cfg = dict(real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent")
    lb = mg.Loopback(world)
    res, errors = [None] * world, []

    def rank_main(r):
        try:
            ctx = mg.Context(mg.make_opts(dim=3, n=box, rank=r, world=world, device=0, comm_id=b"\0" * 128, **cfg),
                             loopback=lb)
            assert ctx.levels[0]["nz_local"] == 32 and ctx.levels[1]["distributed"]
            ctx.init_point_charge()
            ctx.timing(True)
            errs = ctx.cycles(3)
            t = ctx.timing_read()
            ctx.timing(False)
            assert t["fused_pre"][1] == 3 and t["fused_post"][1] == 3 and t["half_sweep"][1] == 0, t
            res[r] = (ctx.field_stats(), errs, ctx.residual_norm())
            ctx.close()
        except Exception as e:  # noqa: BLE001
            errors.append((r, repr(e)))

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    lb.close()
    assert not errors, errors
    ref = _ctx(dim=3, n=box, **cfg)
    ref.init_point_charge()
    e_ref = ref.cycles(3)
    h_ref = ref.field_stats()[0]
    assert sum(res[r][0][0] for r in range(world)) & M64 == h_ref
    for r in range(world):
        np.testing.assert_allclose(res[r][1], e_ref, rtol=1e-12, atol=0)
        np.testing.assert_allclose(res[r][2], ref.residual_norm(), rtol=1e-12, atol=0)


@pytest.mark.parametrize("real", ["double", "float"])
def test_cpu_raw_fields(real):
    """cpu-raw.lua:148-171 state by name: rs/Rs/vs/Vs per level size, psiOld, errorBuf, tmpU."""
    from oracle_lib import prolong_correct_arr

    mg = _mg()
    r = mg.MultigridHIPRaw(32, real, nu1=2, nu2=2, coarse_init="fresh")
    r.quiet = True
    r.run(1)
    old = r.psi
    r.run(1)
    psi = r.psi
    ctx = r.ctx
    assert np.array_equal(r.psiOld, old)
    # cpu-raw.lua semantics (MultigridHIPRaw's default arith="double"): the difference and its square in double,
    # stored once in the real type
    d = psi.astype(np.float64) - old.astype(np.float64)
    assert np.array_equal(r.errorBuf, (d * d).astype(psi.dtype))
    assert r.tmpU.shape == psi.shape  # Jacobi target buffer
    assert sorted(r.rs.keys(), reverse=True) == [32, 16, 8, 4, 2, 1]
    for size in (32, 16, 8):
        lvl = [lv["nx"] for lv in ctx.levels].index(size)
        u, f = r.Vs[size], r.Rs[size]
        ref = residual_arr(2, u, f, (2.0 ** lvl) / 32, 0.0, arith="double")
        assert np.array_equal(r.rs[size], ref)
        V = r.Vs[size // 2]
        assert np.array_equal(r.vs[size], prolong_correct_arr(2, np.zeros_like(u), V, "pc", 0.0, arith="double"))
    with pytest.raises(TypeError):
        r.rs[8] = np.zeros((8, 8))


def test_cpu_lua_knobs_and_matrix_two_grid():
    """cpu.lua protocol: size is {n, n}, inPlaceIterativeSolver is writable (Jacobi <-> GaussSeidel,
    rebuilding the device context with psi / f kept), twoGrid(h, u, f) takes lua-matrix-style lists."""
    mg = _mg()
    s = mg.MultigridHIP(size=16)
    assert s.size == (16, 16)
    assert s.inPlaceIterativeSolver == mg.MultigridHIP.Jacobi
    s.step()
    psi = s.psi
    s.inPlaceIterativeSolver = mg.MultigridHIP.GaussSeidel
    assert s.inPlaceIterativeSolver == mg.MultigridHIP.GaussSeidel
    assert np.array_equal(s.psi, psi)
    o = Oracle(dim=2, n=(16, 16, 1), smoother="gs_lex")  # GaussSeidel = cpu.lua:24-37's lexicographic sweep
    o.set(0, psi)
    o.set(1, s.f)
    s.step()
    o.step()
    assert np.array_equal(s.psi, o.get(0))
    u = _rand((8, 8), np.float64, 1)
    f = _rand((8, 8), np.float64, 2)
    ua = u.copy()
    s.twoGrid(2.0 / 16, ua, f)
    ul = [list(map(float, u[:, i])) for i in range(8)]  # ul[i][j], x = i
    fl = [list(map(float, f[:, i])) for i in range(8)]
    s.twoGrid(2.0 / 16, ul, fl)
    assert np.array_equal(np.array(ul).T, ua)


@pytest.mark.parametrize("dim,n,real", [(2, 64, "double"), (3, 32, "double"), (2, 32, "float")])
def test_device_cg_second_oracle(dim, n, real):
    """SURVEY §8(f) row 3 (converge-multigrid-vs-krylov.lua:38-69): conjugate gradients on the device
    (x0 = -f, b = f, stop at rSq / bSq < eps) and the converged multigrid psi (north-star RB-GS 2+2
    F-cycles) solve the same discrete system: they agree to 1e-8 relative (fp64; 1e-4 in fp32)."""
    box = (n, n, n if dim == 3 else 1)
    ctx = _ctx(dim=dim, n=box, real=real, smoother="rbgs", nu1=2, nu2=2, cycle="F", prolong="linear",
               coarse_bc="consistent")
    ctx.init_point_charge()
    ctx.cycles(40)
    mg = ctx.get_psi().astype(np.float64)
    x, iters, err, hist = ctx.cg_solve(epsilon=1e-26 if real == "double" else 1e-12, maxiter=5000, history=True)
    assert 0 < iters < 5000 and len(hist) == iters
    assert hist[-1] == np.abs(x).max()
    rel = np.linalg.norm(x.astype(np.float64) - mg) / np.linalg.norm(mg)
    assert rel <= (1e-8 if real == "double" else 1e-4), rel
    # the solver's own state is untouched
    assert np.array_equal(ctx.get_psi(), mg.astype(ctx.dtype))


def test_device_cg_matches_reference_operator_on_cpu_lua_path():
    """The cpu.lua configuration (2D Jacobi 7+7 V, injection) converges to the same A^-1 f as CG."""
    ctx = _ctx(dim=2, n=(16, 16, 1), real="double")
    ctx.init_point_charge()
    for _ in range(400):
        if ctx.cycle() < 1e-12:
            break
    x, iters, err = ctx.cg_solve(epsilon=1e-28, maxiter=2000)
    mg = ctx.get_psi()
    assert np.abs(x - mg).max() <= 1e-8 * np.abs(mg).max()


@pytest.mark.parametrize("world", [2, 4])
def test_loopback_zpost_distributed_level(world, monkeypatch):
    """Engine 4 (zpost: PRE per piece, POST temporally blocked) on a distributed level: loopback slabs of a 256^3
    box with level 0 fused and level 1 (128 x 128 x 128 / world) zpost equal the single domain bit for bit, and
    the single domain equals one launch per piece on that level."""
    import threading

    monkeypatch.setenv("MGP_FUSED_MIN_CELLS", str(1 << 23 if world == 2 else 1 << 22))
    monkeypatch.setenv("MGP_ZPOST_MIN_CELLS", str(1 << 19))
    mg = _mg()
    box = (256, 256, 256)
    cfg = dict(real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent")
    lb = mg.Loopback(world)
    res, errors = [None] * world, []

    def rank_main(r):
        try:
            ctx = mg.Context(mg.make_opts(dim=3, n=box, rank=r, world=world, device=0, comm_id=b"\0" * 128, **cfg),
                             loopback=lb)
            eng = [lv["engine"] for lv in ctx.levels]
            assert eng[:2] == ["zs", "zpost"] and ctx.levels[1]["distributed"], eng
            ctx.init_point_charge()
            errs = ctx.cycles(3)
            res[r] = (ctx.field_stats(), errs)
            ctx.close()
        except Exception as e:  # noqa: BLE001
            errors.append((r, repr(e)))

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    lb.close()
    assert not errors, errors
    ref = _ctx(dim=3, n=box, **cfg)
    assert [lv["engine"] for lv in ref.levels][1] == "zpost"
    ref.init_point_charge()
    e_ref = ref.cycles(3)
    h_ref = ref.field_stats()[0]
    assert sum(res[r][0][0] for r in range(world)) & M64 == h_ref
    for r in range(world):
        np.testing.assert_allclose(res[r][1], e_ref, rtol=1e-12, atol=0)
    psi_ref = ref.get_psi()
    ref.close()
    monkeypatch.setenv("MGP_ZPOST_MIN_CELLS", str(1 << 40))
    pp = _ctx(dim=3, n=box, **cfg)
    assert [lv["engine"] for lv in pp.levels][1] == "piece"
    pp.init_point_charge()
    e_pp = pp.cycles(3)
    assert np.array_equal(pp.get_psi(), psi_ref)
    np.testing.assert_allclose(e_pp, e_ref, rtol=1e-12, atol=0)


@pytest.mark.parametrize("dim,box,real,cycle", [
    (3, (512, 512, 512), "float", "V"),
    (3, (512, 512, 512), "double", "V"),
    (2, (4096, 4096, 1), "float", "V"),
    (3, (256, 256, 256), "float", "F"),
], ids=["configs2-f32", "configs2-f64", "configs1-2d", "256cube-F"])
def test_run_to_run_determinism_full_size(dim, box, real, cycle, monkeypatch):
    """The bench workloads at full size, 40 cycles, three fresh contexts (graph replay twice, eager
    launches once): psi's device fingerprint and every err identical.  Every kernel of the path writes
    each cell once per phase and sums in fixed orders, so any difference is a race (a wave reading an
    LDS slot or a plane before its producer wrote it) — the class of bug round 3 found late."""
    kw = dict(dim=dim, n=box, real=real, smoother="rbgs", nu1=2, nu2=2, cycle=cycle, prolong="linear",
              coarse_bc="consistent")
    runs = []
    for graph in ("1", "1", "0"):
        monkeypatch.setenv("MGP_GRAPH", graph)
        ctx = _ctx(**kw)
        try:
            ctx.init_point_charge()
            errs = np.concatenate([ctx.cycles(20), ctx.cycles(20)])
            runs.append((ctx.field_stats()[0], errs))
        finally:
            ctx.close()
    assert runs[0][0] == runs[1][0] == runs[2][0], "psi fingerprints differ between runs"
    assert np.array_equal(runs[0][1], runs[1][1]) and np.array_equal(runs[0][1], runs[2][1])
    assert np.all(np.isfinite(runs[0][1])) and runs[0][1][-1] < runs[0][1][0]
