"""The driver's multi-GPU launch of bench.py, rehearsed on CPU (no GPU needed).

The driver runs `python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1
--master-port P bench.py --gpus N ...` for N = 2, 4, 8.  `--plan-only` takes that exact path — rank/world from
the environment, the gloo process group, the RCCL unique id made on rank 0 and broadcast to every rank, the
options each rank builds — up to the point where the context would be created, then gathers every rank's level
plan (mgp_plan: the same host logic mgp_create runs) and checks on rank 0 that the ranks agree on the
hierarchy and that the slabs of every distributed level tile the box in rank order.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(n, *args):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", str(n), "--plan-only", *args]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0 alone prints
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 4])
def test_weak_scaling_launch_plan(n):
    """Weak scaling (the default line): a 512^3 slab per rank of a 512 x 512 x 512 N box, k_zs on every slab."""
    d = _launch(n)
    assert d["n_gpus"] == n and d["global_box"] == [512, 512, 512 * n]
    assert d["rank_slabs_level0"] == [[512 * r, 512] for r in range(n)]
    assert d["engines"][0] == "zs" and d["distributed_levels"] >= 2
    assert d["comm_id_bytes"] == 128


def test_strong_scaling_launch_plan_config3():
    """BASELINE configs[3]: 2048^3 over 8 ranks, 256 planes each (the driver's 8-GPU node)."""
    d = _launch(8, "--box", "2048,2048,2048")
    assert d["global_box"] == [2048, 2048, 2048]
    assert d["rank_slabs_level0"] == [[256 * r, 256] for r in range(8)]
    assert d["engines"][0] == "zs"


def test_north_star_lines_planned_at_8_ranks():
    """At 8 ranks the default run adds BASELINE configs[3] (2048^3 V) and configs[4] (4096^3 F) to the line;
    --plan-only lists each workload's per-cycle RCCL calls and bytes per rank (mgp_plan_comm: the library's own
    cycle logic, run on the host with every device call skipped)."""
    d = _launch(8)
    assert set(d["north_star_lines"]) == {"configs[3]", "configs[4]"}
    weak = d["comm_per_cycle"]
    # weak scaling: level 0 (k_zs): u before PRE, u on the side stream after PRE; levels 1-4 (deep halos): f before
    # pre-smoothing, u before post-smoothing; the coarse V planes level 0's and level 1's POST (k_zs) read; one
    # all-gather, one all-reduce
    assert weak["allreduces"] == 1 and weak["allgathers"] == 1 and weak["side_stream_exchanges"] == 1
    assert weak["calls"] == len(weak["sequence"]) == 14
    c3, c4 = (d["north_star_lines"][k]["comm_per_cycle"] for k in ("configs[3]", "configs[4]"))
    assert d["north_star_lines"]["configs[4]"]["cycle"] == "F"
    assert c3["side_stream_exchanges"] == 2  # levels 0 and 1 run k_zs on 2048 x 2048 x 256 slabs
    assert c4["allgathers"] > 1 and c4["calls"] > c3["calls"]  # the F-cycle revisits the agglomerated levels
    assert c4["halo_MB_per_neighbour"] > c3["halo_MB_per_neighbour"] > weak["halo_MB_per_neighbour"]


@pytest.mark.parametrize("n", [1, 2])
def test_north_star_lines_planned_at_1_and_2_ranks(n):
    """the driver's 1- and 2-GPU runs carry the configs[3] whole-box line too (2048^3 fits one
    GPU: ~160 GB with u, f, t, psiOld and the hierarchy), so the 1/2/4/8 runs give the north star's strong-scaling
    curve; configs[4] (4096^3) does not fit fewer than 4 GPUs and is listed as skipped.  N = 1 adds the fp64 line."""
    d = _launch(n)
    ns = d["north_star_lines"]
    assert set(ns) == {"configs[3]", "configs[4]"}
    assert ns["configs[3]"]["fits"] and not ns["configs[4]"]["fits"]
    assert ns["configs[3]"]["global_box"] == [2048, 2048, 2048]
    assert d.get("fp64_line", False) == (n == 1)
    if n == 2:
        assert ns["configs[3]"]["comm_per_cycle"]["allreduces"] == 1


def test_plan_comm_is_identical_on_every_rank():
    """RCCL matches calls per communicator in issue order: every rank of a slab decomposition must issue the same
    sequence (a rank at the end of the stack exchanges with one neighbour, but calls in the same order)."""
    sys.path.insert(0, os.path.join(ROOT, "lua-multigrid-poisson_amd"))
    import mgpoisson as mg

    for box, cyc, w in [((512, 512, 4096), "V", 8), ((2048, 2048, 2048), "V", 8), ((4096, 4096, 4096), "F", 8),
                        ((256, 256, 512), "F", 2)]:
        logs = [mg.plan_comm(mg.make_opts(dim=3, n=box, real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear",
                                          coarse_bc="consistent", cycle=cyc, rank=r, world=w, comm_id=b"\0" * 128), 2)
                for r in range(w)]
        assert all(l == logs[0] for l in logs), (box, cyc, w)
        assert logs[0][-1] == ("allreduce", 0, 0, 1, 8)


def test_plan_comm_without_side_stream(monkeypatch):
    """MGP_EARLY_X=0: POST's halo goes out on the compute stream before POST, so the plan lists no side-stream
    exchange (the host-only plan has neither stream: only an existing side stream marks an exchange as its)."""
    sys.path.insert(0, os.path.join(ROOT, "lua-multigrid-poisson_amd"))
    import mgpoisson as mg

    kw = dict(dim=3, n=(512, 512, 1024), real="float", smoother="rbgs", nu1=2, nu2=2, prolong="linear",
              coarse_bc="consistent", rank=0, world=2, comm_id=b"\0" * 128)
    on = mg.plan_comm(mg.make_opts(**kw), 1)
    monkeypatch.setenv("MGP_EARLY_X", "0")
    off = mg.plan_comm(mg.make_opts(**kw), 1)
    assert any(r[1] == 1 for r in on) and not any(r[1] == 1 for r in off)
    assert len(off) == len(on)


def _traffic_file(tmp_path, name, bench_args, kernels, src):
    sys.path.insert(0, ROOT)
    import shlex

    import bench

    p = tmp_path / name
    p.write_text(json.dumps({"kernels": kernels, "source_hash": src,
                             "workload": bench.workload_key_from_argv(shlex.split(bench_args)), "bench_args": bench_args}))
    return str(p)


def test_pick_traffic_keys_on_workload_and_grid(tmp_path):
    """2048^3 and 4096^2 x 512 have the same cells (8,589,934,592), so the configs[4] slab's PMC
    file must not be taken for the 2048^3 box; a file of the right workload whose launch grid differs is refused too;
    the right file is taken only when every timed launch's symbol and grid are in it."""
    sys.path.insert(0, ROOT)
    import bench

    post = "k_zs<float, false, 1, true, true, true>"
    pre = "k_zs<float, true, 0, false, true, false>"
    ent = lambda g: {"grid": g, "launches": 2, "read_bytes": 1.0, "write_bytes": 1.0, "bytes_per_launch": 2.0}  # noqa: E731
    slab4 = _traffic_file(tmp_path, "slab4.json", "--box 4096,4096,512 --cycle F", {post: ent(100), pre: ent(50)}, "h")
    box_badgrid = _traffic_file(tmp_path, "box_g.json", "--box 2048,2048,2048", {post: ent(101), pre: ent(50)}, "h")
    box_oldsrc = _traffic_file(tmp_path, "box_s.json", "--box 2048,2048,2048", {post: ent(100), pre: ent(50)}, "old")
    box = _traffic_file(tmp_path, "box.json", "--box 2048,2048,2048", {post: ent(100), pre: ent(50)}, "h")
    a = bench.parse(["--box", "2048,2048,2048"])
    wkey = bench.workload_key(a, (2048, 2048, 2048), 1)
    launched = {"fused_post": (post, 100), "fused_pre": (pre, 50)}
    p, tr, why = bench.pick_traffic(",".join([slab4, box_badgrid, box_oldsrc]), wkey, launched, src_hash="h")
    assert p is None and tr is None
    rel = lambda p: os.path.relpath(p, ROOT)  # noqa: E731
    assert "workload" in why[rel(slab4)] and "grid 100" in why[rel(box_badgrid)] and "source" in why[rel(box_oldsrc)]
    p, tr, why = bench.pick_traffic(",".join([slab4, box_badgrid, box]), wkey, launched, src_hash="h")
    assert p == box and why is None
    # the slab itself is matched by its own file, and the weak-scaling key differs by world
    a4 = bench.parse(["--box", "4096,4096,512", "--cycle", "F"])
    assert bench.pick_traffic(slab4, bench.workload_key(a4, (4096, 4096, 512), 1), launched, src_hash="h")[0] == slab4
    d = bench.parse([])
    assert bench.workload_key(d, (512, 512, 1024), 2) != bench.workload_key(d, (512, 512, 512), 1)
