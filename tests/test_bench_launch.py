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
