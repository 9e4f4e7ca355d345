"""GPU: the exchanges and collectives a rank executes equal the host-only plan, and are the same on every rank.

RCCL matches the calls of one communicator in issue order, so every rank of a slab decomposition must issue
the same sequence per communicator; the early POST halo exchange goes to the side stream's own communicator
(mgp_api.cpp early_exchange_post).  The executed log (mgp_comm_log) of a loopback decomposition (the multi-GPU
code path with device copies for the transfers) is compared with mgp_plan_comm (the same cycle logic run on
the host with every device call skipped — what bench.py --plan-only reports for the driver's N-GPU lines).
"""
import os
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _mg():
    import mgpoisson

    return mgpoisson


def _run(box, world, cfg, cycles, env=None):
    mg = _mg()
    lb = mg.Loopback(world)
    logs, timings, errors = [None] * world, [None] * world, []

    def rank_main(r):
        try:
            ctx = mg.Context(mg.make_opts(dim=3, n=box, rank=r, world=world, device=0, comm_id=b"\0" * 128, **cfg),
                             loopback=lb)
            ctx.init_point_charge()
            ctx.comm_log(reset=True)
            ctx.timing(True)
            ctx.cycles(cycles)
            timings[r] = ctx.timing_read()
            ctx.timing(False)
            logs[r] = ctx.comm_log()
            ctx.close()
        except Exception as e:  # noqa: BLE001 - surfaced below
            errors.append((r, repr(e)))

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    lb.close()
    assert not errors, errors
    return logs, timings


# side: level 0 runs temporally blocked (k_zs), so its early POST exchange rides the side communicator (the
# fp64 POST tile is 64 wide: a 32-wide box runs level 0 per piece, every exchange on the main one)
CASES = [
    ((64, 64, 256), 2, dict(cycle="V"), 4096, True),
    ((64, 64, 512), 8, dict(cycle="V"), 4096, True),
    ((64, 64, 256), 4, dict(cycle="F"), 4096, True),
    ((32, 32, 256), 8, dict(cycle="F", real="double"), 512, False),
    # full weighting: k_resfw on the 64-wide slab levels (u exchanged two planes deep), the two-pass form below
    ((64, 64, 256), 2, dict(cycle="V", restriction="full_weighting"), 4096, True),
]


@pytest.mark.parametrize("box,world,extra,gather,side", CASES, ids=["w2-V", "w8-V", "w4-F", "w8-F-f64", "w2-V-fw"])
def test_executed_comm_log_equals_plan(box, world, extra, gather, side, monkeypatch):
    monkeypatch.setenv("MGP_FUSED", "1")
    monkeypatch.setenv("MGP_FUSED_MIN_CELLS", "65536")
    mg = _mg()
    cfg = dict(real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear", coarse_bc="consistent",
               gather_cells=gather)
    cfg.update(extra)
    cycles = 3
    logs, timings = _run(box, world, cfg, cycles)
    assert all(l == logs[0] for l in logs)  # call-order equality across ranks
    plan = mg.plan_comm(mg.make_opts(dim=3, n=box, rank=0, world=world, comm_id=b"\0" * 128, **cfg), cycles)
    assert logs[0] == plan
    # the early POST exchange rides the side communicator (MGP_EARLY_X=0: no side stream, POST's halo goes out on
    # the compute stream before POST)
    assert any(r[1] == 1 for r in plan) == (side and os.environ.get("MGP_EARLY_X", "1") != "0")
    # every exchange and collective was timed on its stream
    n_ex = sum(1 for r in plan if r[0] == "exchange")
    n_co = sum(1 for r in plan if r[0] != "exchange")
    for t in timings:
        assert t["exchange"][1] == n_ex and t["collective"][1] == n_co
        assert t["exchange"][0] > 0 and t["collective"][0] > 0


def test_comm_log_single_gpu_is_empty():
    mg = _mg()
    ctx = mg.Context(mg.make_opts(dim=3, n=(32, 32, 32), real="float", smoother="rbgs", nu1=2, nu2=2,
                                  prolong="linear", coarse_bc="consistent"))
    ctx.init_point_charge()
    ctx.cycles(2)
    assert ctx.comm_log() == []
    assert mg.plan_comm(ctx.opts, 2) == []
    e = np.float64(ctx.cycle())
    assert np.isfinite(e)
