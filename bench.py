#!/usr/bin/env python3
"""bench.py — V-cycles/s + finest-smoother HBM GB/s of the MI355X multigrid Poisson hot path.

Metric (BASELINE.json): "V-cycles/sec + finest-smoother achieved HBM GB/s, 3D Poisson".
Workload at N=1: BASELINE.json configs[2] — 3D Poisson 512^3, 7-point stencil, V-cycle with
2+2 red/black Gauss-Seidel smoothing, single MI355X (the largest configuration that fits one
GPU; 4096^3 needs >= 4 GPUs).  fp32, trilinear prolongation, 2x2x2-average
restriction, consistent coarse boundary, point-charge RHS (cpu.lua:182-193), and the
reference's per-cycle err = RMS update (cpu.lua:200-203) computed on the device every cycle.

Scaling: weak.  Each rank owns a 512^3 z-slab of a 512 x 512 x (512 N) box; the V-cycle is
domain-decomposed with RCCL halo exchange after every smoothing half-sweep and an all-gather
onto every rank once a level has <= 32768 cells.  value = (N slabs x K cycles) / max-rank
time, i.e. 512^3-cell V-cycles per second for the whole job (= plain V-cycles/s at N=1).

Launch: python bench.py [--gpus N --steps K --warmup W]  (N>1 under torch.distributed.run).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "lua-multigrid-poisson_amd"))

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--n", type=int, default=512, help="cells per axis of each rank's cube slab")
    p.add_argument("--real", default="float", choices=["float", "double"])
    p.add_argument("--cycle", default="V", choices=["V", "F"])
    p.add_argument("--nu", type=int, default=2)
    p.add_argument("--no-timing", action="store_true", help="skip the per-launch smoother events")
    p.add_argument("--cpu-cycles", type=int, default=2, help="oracle cycles timed for cpu_baseline (0 = skip)")
    p.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "r01_final_pmc_traffic.json"),
                   help="JSON with the PMC-measured HBM bytes per launch of the dominant kernel (tools/pmc_traffic.py); "
                        "used only when its kernel name matches")
    return p.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
    import torch
    import torch.distributed as dist

    import mgpoisson

    comm_id = None
    if world > 1:
        dist.init_process_group(backend="gloo")
        obj = [mgpoisson.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm_id = obj[0]

    n = a.n
    cfg = dict(dim=3, n=(n, n, n * world), real=a.real, smoother="rbgs", nu1=a.nu, nu2=a.nu, cycle=a.cycle,
               prolong="linear", coarse_bc="consistent", coarse_init="fresh", err_mode=1, device=local,
               rank=rank, world=world, comm_id=comm_id)
    ctx = mgpoisson.Context(mgpoisson.make_opts(**cfg))
    ctx.init_point_charge()
    rb = 4 if a.real == "float" else 8
    cells_rank = n * n * n

    def barrier_sync():
        ctx.sync()
        torch.cuda.synchronize(local)
        if world > 1:
            dist.barrier()

    # warmup (untimed; also captures the hipGraphs of the cycle)
    if a.warmup:
        ctx.cycles(a.warmup)
    barrier_sync()
    t0 = time.perf_counter()
    errs = ctx.cycles(a.steps)
    barrier_sync()
    dt = time.perf_counter() - t0

    # roofline window: the same K cycles again, launched eagerly with a HIP event pair around
    # every timed level-0 launch on the context's stream (graph replay cannot bracket single
    # launches); the kernels are identical, only the host launch path differs
    timed = {}
    if not a.no_timing:
        ctx.timing(True)
        ctx.cycles(a.steps)
        timed = ctx.timing_read()
        ctx.timing(False)
        barrier_sync()

    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    value = world * a.steps / dt
    line = {
        "metric": "V-cycles/sec + finest-smoother achieved HBM GB/s, 3D Poisson",
        "value": value,
        "unit": "V-cycles/s (512^3-cell slabs, whole job)" if a.cycle == "V" else "F-cycles/s (512^3-cell slabs, whole job)",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": 1e3 * dt / a.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if a.real == "float" else "f64",
        "data": "synthetic point-charge RHS (cpu.lua:182-193), psi0 = -f",
        "config": {
            "workload": f"BASELINE configs[2]: 3D Poisson {n}^3 per GPU, 7-point, RB-GS {a.nu}+{a.nu}, {a.cycle}-cycle, "
                        "trilinear P, 2x2x2-average R, per-cycle RMS-update err",
            "global_box": [n, n, n * world],
            "parallelism": f"slab-z x{world} (RCCL halo per half-sweep)" if world > 1 else "single GPU",
            "levels": len(ctx.levels),
        },
        "final_err": float(errs[-1]),
    }
    tname = "float" if a.real == "float" else "double"
    lin = 1
    kernels = {"half_sweep": f"k_half<{tname}, 3, 1, false>",
               "fused_pre": f"k_zs<{tname}, true, 0, false, true>",
               "fused_post": f"k_zs<{tname}, false, {lin}, true, true>"}
    # Algorithmic bytes per level-0 cell of one launch (reals): what the launch must move
    # to and from HBM.  half_sweep: read the other colour and f, write this colour of half the cells.
    # fused_pre (k_zs: 2 RB-GS sweeps + residual + restriction): read black u and f, write u and R/8.
    # fused_post (k_zs: prolongation + correction + 2 sweeps + err): read black u, V/8, f, psiOld; write u.
    algo_reals = {"half_sweep": 1.5, "fused_pre": 2.625, "fused_post": 3.625}
    per_kind = {k: v for k, v in timed.items() if v[1] > 0}
    cells = n * n * n
    if per_kind:
        # per kind: (ms, launches, algorithmic bytes, reference-path bytes as the library counts them:
        # SURVEY.md §8(d) per-sweep accounting, i.e. what one launch per half-sweep would move)
        kinds = {k: (ms, cnt, algo_reals[k] * rb * cells * cnt, by) for k, (ms, cnt, by) in per_kind.items()}
        line["level0_kernels"] = {
            k: {"kernel": kernels[k], "launches": cnt, "avg_us": 1e3 * ms / cnt,
                "algorithmic_bytes_per_launch": ab / cnt, "achieved_GBps": ab / (ms * 1e-3) / 1e9,
                "per_sweep_accounting_bytes_per_launch": by / cnt,
                "effective_GBps_per_sweep_accounting": by / (ms * 1e-3) / 1e9}
            for k, (ms, cnt, ab, by) in kinds.items()}
        dom = max(kinds, key=lambda k: kinds[k][0])  # the kernel with the most level-0 time
        ms, cnt, ab, by = kinds[dom]
        achieved = ab / (ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS, "traffic": None, "kernel": kernels[dom],
                "algorithmic_bytes_per_launch": ab / cnt, "avg_launch_us": 1e3 * ms / cnt,
                "window": f"{a.steps} cycles after the timed region, HIP events around each launch"}
        if a.traffic and os.path.exists(a.traffic):
            with open(a.traffic) as fh:
                tr = json.load(fh)
            ent = tr.get("kernels", {}).get(kernels[dom]) if "kernels" in tr else (
                tr if tr.get("kernel") == kernels[dom] else None)
            if ent:
                roof["traffic"] = ent.get("bytes_per_launch")
                roof["traffic_source"] = os.path.relpath(a.traffic, ROOT)
        line["roofline"] = roof

    if rank == 0 and world == 1 and a.cpu_cycles > 0:
        line["cpu_baseline"] = cpu_baseline(cfg, a.cpu_cycles)
    if rank == 0:
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(cfg, cycles):
    """The C oracle (the build's restatement of the reference CPU path) on this host, 1 thread."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import Oracle

    kw = {k: cfg[k] for k in ("dim", "n", "real", "smoother", "nu1", "nu2", "cycle", "prolong", "coarse_bc", "coarse_init")}
    o = Oracle(threads=1, **kw)
    o.init_point_charge()
    t0 = time.perf_counter()
    for _ in range(cycles):
        o.step()
    dt = time.perf_counter() - t0
    return {"value": cycles / dt, "unit": "V-cycles/s (512^3)" if cfg["cycle"] == "V" else "F-cycles/s (512^3)",
            "cores": 1, "kind": "port",
            "sample": f"{cycles} full cycles of the same 3D {cfg['n'][0]}^3 workload, oracle/mgp_oracle.c "
                      f"(gcc -O2, -ffp-contract=off), single thread like the reference, {dt:.1f} s"}


if __name__ == "__main__":
    main()
