"""GPU: the RCCL transport executed on one GPU.

RCCL refuses two ranks on one device, and the test boxes have one GPU, so the multi-GPU tests run the slab code
path on the loopback transport (device copies instead of RCCL calls).  With MGP_TRANSPORT=rccl a world-1 context
takes that same slab path on a real one-rank RCCL communicator (include/mgpoisson.h, mgp_api.cpp env_rccl1):

  - mgp_create: ncclGetUniqueId -> ncclCommInitRank -> ncclCommSplit (the side stream's communicator);
  - a cycle: the grouped ncclSend/ncclRecv halo exchanges (peerless at world 1: empty groups, on both
    communicators), the agglomeration ncclAllGather (in place), the err ncclAllReduce; residual norm and metrics
    all-reduces;
  - mgp_group_create on one device: the non-blocking ncclCommInitRankConfig (a second grouped non-blocking init
    makes the side-stream communicators: a grouped ncclCommSplit of non-blocking communicators fails in RCCL 7.2)
    + polling, and after an injected rank failure group_abort's ncclCommAbort.

Bar: psi bit-identical to the plain world-1 context, err / norms to 1e-12, the executed call log equal to the
host-only plan, every logged call timed on its stream (so it ran on the RCCL transport: a world-1 context has
no other)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NS = dict(real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent")

CASES = [
    (3, (64, 64, 64), dict(NS, gather_cells=4096), None),
    (3, (128, 128, 128), dict(NS, cycle="F", gather_cells=4096), "65536"),  # k_zs slab levels + side communicator
    (3, (32, 32, 64), dict(real="double", smoother="jacobi", nu1=3, nu2=3, prolong="pc", coarse_init="warm",
                           gather_cells=512), None),
    (2, (256, 256), dict(NS), None),  # 2D: no slab levels, the err all-reduce only
]


def _mg():
    import mgpoisson

    return mgpoisson


@pytest.mark.parametrize("dim,box,cfg,fused", CASES, ids=["V-f32", "F-fused-f32", "jacobi-warm-f64", "2d"])
def test_rccl_world1_equals_plain_context(dim, box, cfg, fused, monkeypatch):
    mg = _mg()
    if fused:
        monkeypatch.setenv("MGP_FUSED", "1")
        monkeypatch.setenv("MGP_FUSED_MIN_CELLS", fused)
    opts = mg.make_opts(dim=dim, n=box, **cfg)
    ref = mg.Context(opts)
    ref.init_point_charge()
    e_ref = ref.cycles(3)
    psi_ref, rn_ref, met_ref = ref.get_psi(), ref.residual_norm(), ref.metrics()
    ref.close()

    monkeypatch.setenv("MGP_TRANSPORT", "rccl")
    ctx = mg.Context(mg.make_opts(dim=dim, n=box, **cfg))
    assert ctx.levels[0]["distributed"] == (dim == 3)
    if fused:
        assert ctx.levels[0]["engine"] == "zs"
    ctx.init_point_charge()
    ctx.comm_log(reset=True)
    ctx.timing(True)
    e = np.concatenate([ctx.cycles(2), [ctx.cycle()]])
    t = ctx.timing_read()
    ctx.timing(False)
    log = ctx.comm_log()
    assert np.array_equal(ctx.get_psi(), psi_ref)
    np.testing.assert_allclose(e, e_ref, rtol=1e-12, atol=0)
    np.testing.assert_allclose(ctx.residual_norm(), rn_ref, rtol=1e-12, atol=0)
    rel, cnt, frob = ctx.metrics()
    assert cnt == met_ref[1]
    np.testing.assert_allclose([rel, frob], [met_ref[0], met_ref[2]], rtol=1e-12, atol=0)

    ops = {r[0] for r in log}
    assert "allreduce" in ops
    if dim == 3:
        assert {"exchange", "allgather"} <= ops  # slab levels exchange (empty groups) and agglomerate
        assert any(lv["distributed"] for lv in ctx.levels) and not ctx.levels[-1]["distributed"]
    if fused:
        assert any(r[1] == 1 for r in log)  # the early POST exchange on the split communicator
    assert log == mg.plan_comm(ctx.opts, 3)
    assert t["collective"][1] == sum(1 for r in log if r[0] != "exchange")
    assert t["exchange"][1] == sum(1 for r in log if r[0] == "exchange")
    ctx.close()


def test_rccl_world1_group_nonblocking_init_and_abort(monkeypatch):
    import time

    mg = _mg()
    opts = mg.make_opts(dim=3, n=(64, 64, 64), gather_cells=4096, **NS)
    ref = mg.Context(opts)
    ref.init_point_charge()
    e_ref = ref.cycles(2)
    psi_ref = ref.get_psi()
    ref.close()

    monkeypatch.setenv("MGP_TRANSPORT", "rccl")
    g = mg.Group(opts, 1, devices=[0])  # two grouped non-blocking ncclCommInitRankConfig, polled
    assert g.ranks[0].levels[0]["distributed"]
    g.init_point_charge()
    np.testing.assert_allclose(g.cycles(2), e_ref, rtol=1e-12, atol=0)
    assert np.array_equal(g.get_psi(), psi_ref)
    monkeypatch.setenv("MGP_TEST_FAIL_RANK", "0")
    t0 = time.perf_counter()
    with pytest.raises(mg.MGPError, match="injected failure"):
        g.cycles(1)
    assert time.perf_counter() - t0 < 30
    monkeypatch.delenv("MGP_TEST_FAIL_RANK")
    with pytest.raises(mg.MGPError, match="aborted"):  # ncclCommAbort ran: the group is unusable
        g.cycle()
    g.close()


def test_group_argument_error_leaves_group_usable():
    """Only a failure that every rank hits alike before any peer call (a bad argument) keeps the group; any other
    failure aborts it (test_group_rank_failure_aborts_instead_of_hanging)."""
    mg = _mg()
    g = mg.Group(mg.make_opts(dim=3, n=(32, 32, 64), **NS), 2, devices=[0, 0])
    g.init_point_charge()
    with pytest.raises(mg.MGPError):
        g.residual_norm(level=99)
    g.cycles(1)
    g.close()


def _ndev():
    import torch

    return torch.cuda.device_count()


@pytest.mark.skipif("_ndev() < 2", reason="needs two GPUs (the test boxes have one; RCCL refuses two ranks per device)")
def test_group_on_two_devices_real_rccl(monkeypatch):
    """the group's RCCL path with distinct devices — non-blocking communicators, the side-stream
    communicator carrying the early POST exchange next to the compute stream's exchanges — equals the single domain
    and issues the planned call sequence on every rank; an injected rank failure returns instead of hanging."""
    import time

    mg = _mg()
    monkeypatch.setenv("MGP_FUSED_MIN_CELLS", "65536")
    opts = mg.make_opts(dim=3, n=(128, 128, 256), gather_cells=4096, **NS)
    ref = mg.Context(opts)
    ref.init_point_charge()
    e_ref = ref.cycles(3)
    psi_ref = ref.get_psi()
    ref.close()
    g = mg.Group(opts, 2, devices=[0, 1])
    g.init_point_charge()
    for r in g.ranks:
        r.comm_log(reset=True)
    np.testing.assert_allclose(g.cycles(3), e_ref, rtol=1e-12, atol=0)
    assert np.array_equal(g.get_psi(), psi_ref)
    logs = [r.comm_log() for r in g.ranks]
    assert logs[0] == logs[1] == mg.plan_comm(mg.make_opts(dim=3, n=(128, 128, 256), gather_cells=4096, rank=0,
                                                           world=2, comm_id=b"\0" * 128, **NS), 3)
    assert any(c[1] == 1 for c in logs[0])  # side-stream exchanges ran
    monkeypatch.setenv("MGP_TEST_FAIL_RANK", "1")
    t0 = time.perf_counter()
    with pytest.raises(mg.MGPError, match="injected failure"):
        g.cycles(2)
    assert time.perf_counter() - t0 < 60
    monkeypatch.delenv("MGP_TEST_FAIL_RANK")
    with pytest.raises(mg.MGPError, match="aborted"):
        g.cycle()
    g.close()


def test_comm_deadline_reports_the_stalled_exchange_and_aborts(monkeypatch):
    """a per-process RCCL context waits for its streams under a deadline (MGP_COMM_TIMEOUT_S,
    default 600 s).  An exchange held on the GPU (MGP_TEST_STALL=2: the context's second exchange first enqueues a
    kernel that holds the stream, as a peer that never arrives would) makes cycles() return within the deadline with
    MGP_ERR_RCCL naming the rank, the stalled call and its level, the communicators aborted (ncclCommAbort); the
    context then refuses further exchanges instead of hanging, and closes."""
    import time

    mg = _mg()
    monkeypatch.setenv("MGP_TRANSPORT", "rccl")
    monkeypatch.setenv("MGP_COMM_TIMEOUT_S", "3")
    monkeypatch.setenv("MGP_TEST_STALL", "2")
    ctx = mg.Context(mg.make_opts(dim=3, n=(64, 64, 64), gather_cells=4096, **NS))
    assert ctx.levels[0]["distributed"]
    ctx.init_point_charge()
    t0 = time.perf_counter()
    with pytest.raises(mg.MGPError, match=r"communication deadline: rank 0 of 1 waited .* stuck in call #1, a halo "
                                          r"exchange of level \d+ .*communicators aborted") as ei:
        ctx.cycles(2)
    dt = time.perf_counter() - t0
    assert 2.9 < dt < 30, dt
    assert ei.value.code == -3  # MGP_ERR_RCCL
    with pytest.raises(mg.MGPError, match="deadline"):
        ctx.cycle()
    ctx.close()


def test_comm_deadline_is_silent_on_a_healthy_run(monkeypatch):
    """The deadline's polling wait changes nothing on a healthy run: psi bit-identical to the blocking wait."""
    mg = _mg()
    opts = mg.make_opts(dim=3, n=(64, 64, 64), gather_cells=4096, **NS)
    monkeypatch.setenv("MGP_TRANSPORT", "rccl")
    out = []
    for t in ("0", "5"):
        monkeypatch.setenv("MGP_COMM_TIMEOUT_S", t)
        ctx = mg.Context(opts)
        ctx.init_point_charge()
        out.append((ctx.cycles(2), ctx.get_psi()))
        ctx.close()
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert np.array_equal(out[0][1], out[1][1])
