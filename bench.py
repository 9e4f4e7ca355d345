#!/usr/bin/env python3
"""bench.py — V-cycles/s + finest-smoother HBM GB/s of the MI355X multigrid Poisson hot path.

Metric (BASELINE.json): "V-cycles/sec + finest-smoother achieved HBM GB/s, 3D Poisson".
Workload at N=1: BASELINE.json configs[2] — 3D Poisson 512^3, 7-point stencil, V-cycle with
2+2 red/black Gauss-Seidel smoothing, single MI355X (the largest configuration that fits one
GPU; 4096^3 needs >= 4 GPUs).  fp32, trilinear prolongation, 2x2x2-average
restriction, consistent coarse boundary, point-charge RHS (cpu.lua:182-193), and the
reference's per-cycle err = RMS update (cpu.lua:200-203) computed on the device every cycle.

Scaling (default): weak.  Each rank owns a 512^3 z-slab of a 512 x 512 x (512 N) box; the V-cycle
is domain-decomposed with RCCL halo exchange (per half-sweep, or once per temporally blocked phase)
and an all-gather onto every rank once a level has <= 32768 cells.  value = (N slabs x K cycles) /
max-rank time, i.e. 512^3-cell V-cycles per second for the whole job (= plain V-cycles/s at N=1).

--box NX,NY,NZ: strong scaling of one global box split into N z-slabs (BASELINE configs[3]:
--box 2048,2048,2048; configs[4]: --box 4096,4096,4096 --cycle F).  On one GPU, --box 2048,2048,256
and --box 4096,4096,512 run one rank's slab of those configs.  value = cycles/s of the whole box.
--dim 2 --n 4096: BASELINE configs[1] (2D 4096^2 RB-GS, cache-resident: flagged in the line).
--config0: BASELINE configs[0], the reference cpu.lua path (2D 256^2, fp64, Jacobi 7+7 V-cycle, injection,
ghost-0 coarse levels), with the CPU port timed over the same cycles (1 thread and OpenMP) beside the GPU.
--restriction full_weighting: the build's full-weighting option instead of the 2^d cell average.

At every N the default (weak) run adds the north-star workloads to the same JSON line (`north_star_lines`):
BASELINE configs[3] (2048^3 V-cycle) and configs[4] (4096^3 F-cycle) as one box split into N z-slabs (N = 1: the
whole box on one GPU), each run after the previous context is closed, with per-rank halo-exchange and collective
time from HIP events, so that the driver's 1/2/4/8-GPU runs give the north star's strong-scaling curve
(--no-north-star skips them; configs[4] is skipped where it does not fit the ranks' HBM: N < 4).  At N = 1 the
line also carries the fp64 512^3 workload (the reference's default precision, gpu.lua:32) as `fp64_line`.

Roofline fields: `roofline.frac` is the dominant level-0 kernel's algorithmic (compulsory) bytes over its
event-timed duration against 8 TB/s; `roofline.cycle_frac` the compulsory bytes of every level of one cycle
 over ms_per_step against 8 TB/s; `finest_smoother_GBps` BASELINE.md's definition
3 sizeof(real) cells_per_rank sweeps / summed finest-level smoothing kernel time.

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


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10, help="untimed cycles (graph capture, clocks)")
    p.add_argument("--n", type=int, default=512, help="cells per axis of each rank's cube slab (weak scaling)")
    p.add_argument("--box", default=None, help="NX,NY,NZ global box, strong scaling over the ranks (slab-z)")
    p.add_argument("--dim", type=int, default=3, choices=[2, 3])
    p.add_argument("--real", default="float", choices=["float", "double"])
    p.add_argument("--cycle", default="V", choices=["V", "F"])
    p.add_argument("--nu", type=int, default=2)
    p.add_argument("--smoother", default="rbgs", choices=["rbgs", "jacobi"])
    p.add_argument("--prolong", default="linear", choices=["linear", "pc"])
    p.add_argument("--coarse-bc", default="consistent", choices=["consistent", "zero"])
    p.add_argument("--restriction", default="average", choices=["average", "full_weighting"])
    p.add_argument("--config0", action="store_true",
                   help="BASELINE configs[0]: 2D 256^2 fp64 Jacobi 7+7 V-cycle, injection, ghost 0 (cpu.lua path)")
    p.add_argument("--copy-probe-mb", type=int, default=2048,
                   help="buffer size of the measured copy-bandwidth probe reported beside the roofline (0 = skip)")
    p.add_argument("--no-timing", action="store_true", help="skip the per-launch smoother events")
    p.add_argument("--plan-only", action="store_true",
                   help="no GPU: run the launch plumbing (process group, comm id broadcast, options) and print every "
                        "rank's level plan (mgp_plan, host logic) after checking that the ranks' slabs tile the box, "
                        "with each workload's per-cycle RCCL calls and bytes per rank (mgp_plan_comm)")
    p.add_argument("--no-north-star", action="store_true",
                   help="with N >= 4: skip the configs[3] / configs[4] lines after the weak-scaling line")
    p.add_argument("--ns-steps", type=int, default=5, help="timed cycles of each north-star line")
    p.add_argument("--ns-warmup", type=int, default=2, help="untimed cycles of each north-star line")
    p.add_argument("--cpu-reps", type=int, default=3, help="cpu_baseline: best of this many timed samples")
    p.add_argument("--cpu-cycles", type=int, default=4, help="oracle cycles timed for cpu_baseline (0 = skip)")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="threads of the OpenMP cpu_baseline (0 = OMP_NUM_THREADS or all host cores)")
    p.add_argument("--traffic", default=",".join(os.path.join(ROOT, "profiles", f"pmc_traffic_{w}.json") for w in
                                                 ("current", "slab3", "slab4", "box2048", "fw", "2d", "2d64", "f64")),
                   help="comma list of JSONs with the PMC-measured HBM bytes per launch (tools/pmc_traffic.py); the "
                        "first one measured on this build, this workload (box, world, options) and the timed launch's "
                        "kernel and grid is used (pick_traffic)")
    a = p.parse_args(argv)
    if a.config0:
        a.dim, a.n, a.real, a.smoother, a.nu, a.prolong, a.coarse_bc, a.cycle = 2, 256, "double", "jacobi", 7, "pc", "zero", "V"
    return a


NORTH_STAR = [("configs[3]", (2048, 2048, 2048), "V", "BASELINE configs[3]: 3D Poisson 2048^3"),
              ("configs[4]", (4096, 4096, 4096), "F", "BASELINE configs[4]: 3D Poisson 4096^3 fp32 F-cycle")]


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group(backend="gloo")

    box, strong = workload_box(a, world)
    cfg = make_cfg(a, box, rank, world, local, new_comm_id(dist, rank, world))
    if a.plan_only:
        plan_only(a, cfg, box, rank, world, dist)
        return
    line = run_workload(a, cfg, box, strong, rank, world, local, dist, a.steps, a.warmup, primary=True)
    if want_north_star(a, world) and world == 1:
        fa = argparse.Namespace(**vars(a))
        fa.real = "double"
        sub = run_workload(fa, make_cfg(fa, box, rank, world, local, None), box, strong, rank, world, local, dist,
                           a.ns_steps * 4, a.ns_warmup)
        line["fp64_line"] = {k: sub.get(k) for k in ("value", "unit", "ms_per_step", "steps", "warmup", "dtype", "config",
                                                     "final_err", "relative_residual", "roofline", "finest_smoother_GBps",
                                                     "finest_level_hbm_GBps")}
    if want_north_star(a, world):
        extra = {}
        for name, nbox, cyc, _ in NORTH_STAR:
            if nbox[2] % world or nbox[2] // world < 2:
                continue
            ns = argparse.Namespace(**vars(a))
            ns.cycle, ns.box = cyc, ",".join(map(str, nbox))
            ncfg = make_cfg(ns, nbox, rank, world, local, new_comm_id(dist, rank, world))
            fit = fits_hbm(ncfg, world, local)
            if fit is None:
                extra[name] = {"skipped": f"does not fit {world} x HBM (u, f, t and the hierarchy)"}
                continue
            with env_override(fit):
                sub = run_workload(ns, ncfg, nbox, True, rank, world, local, dist, a.ns_steps, a.ns_warmup)
            if rank == 0:
                extra[name] = {k: sub.get(k) for k in ("value", "unit", "ms_per_step", "steps", "warmup", "config",
                                                       "final_err", "relative_residual", "hbm_used_GB_rank0",
                                                       "roofline", "comm_per_rank", "finest_smoother_GBps",
                                                       "finest_level_hbm_GBps")}
                if fit:
                    extra[name]["env"] = fit
        if rank == 0:
            line["north_star_lines"] = extra
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def want_north_star(a, world):
    return not a.box and a.dim == 3 and not a.config0 and not a.no_north_star


def new_comm_id(dist, rank, world):
    """A fresh RCCL unique id from rank 0 for every context (an id serves one communicator)."""
    if world == 1:
        return None
    import mgpoisson

    obj = [mgpoisson.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def workload_box(a, world):
    n = a.n
    if a.box:
        box = tuple(int(x) for x in a.box.split(","))
        if len(box) != 3:
            raise SystemExit("--box takes NX,NY,NZ")
        return box, True
    if a.dim == 2:
        if world != 1:
            raise SystemExit("2D runs are single-GPU (the slab decomposition is 3D)")
        return (n, n, 1), False
    return (n, n, n * world), False


def workload_key(a, box, world):
    """What a PMC traffic file must have been measured on to describe this run's launches: the global box, the
    ranks it is split over and every option that changes the kernels or their grids (pick_traffic)."""
    return {"box": list(box), "world": world, "dim": a.dim if not a.box else 3, "real": a.real, "cycle": a.cycle,
            "smoother": a.smoother, "nu": a.nu, "prolong": a.prolong, "coarse_bc": a.coarse_bc,
            "restriction": a.restriction}


def workload_key_from_argv(argv, world=1):
    """workload_key of `bench.py <argv>` run with `world` ranks (tools/pmc_traffic.py tags its JSON with it)."""
    a = parse(list(argv))
    box, _ = workload_box(a, world)
    return workload_key(a, box, world)


def make_cfg(a, box, rank, world, local, comm_id):
    return dict(dim=a.dim if not a.box else 3, n=box, real=a.real, smoother=a.smoother, nu1=a.nu, nu2=a.nu,
                cycle=a.cycle, prolong=a.prolong, coarse_bc=a.coarse_bc, coarse_init="fresh", err_mode=1, device=local,
                rank=rank, world=world, comm_id=comm_id, restriction=a.restriction)


def fits_hbm(cfg, world, local, total=None):
    """{} if the context fits this GPU's HBM as built, {"MGP_KEEP_PSI_OLD": "0"} if it fits only without the
    psiOld-keeping output buffer (u, f, t and the hierarchy), None if not even then (total: HBM bytes per GPU,
    default the device's)."""
    rb = 4 if cfg["real"] == "float" else 8
    cells = cfg["n"][0] * cfg["n"][1] * cfg["n"][2] / world
    if total is None:
        import torch

        total = torch.cuda.get_device_properties(local).total_memory
    est = lambda arrays: cells * rb * arrays * 8 / 7 + (2 << 30)  # noqa: E731
    if est(4) < 0.92 * total:
        return {}
    if est(3) < 0.92 * total:
        return {"MGP_KEEP_PSI_OLD": "0"}
    return None


class env_override:
    def __init__(self, env):
        self.env, self.old = env or {}, {}

    def __enter__(self):
        for k, v in self.env.items():
            self.old[k] = os.environ.get(k)
            os.environ[k] = v

    def __exit__(self, *exc):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def run_workload(a, cfg, box, strong, rank, world, local, dist, steps, warmup, primary=False):
    """One workload: K timed cycles (hipGraph replay on one GPU), then the same K again with event timing; returns
    the bench line (meaningful on rank 0)."""
    import torch

    import mgpoisson

    n = a.n
    ctx = mgpoisson.Context(mgpoisson.make_opts(**cfg))
    ctx.init_point_charge()
    rb = 4 if a.real == "float" else 8
    lv0 = ctx.levels[0]
    cells_rank = lv0["nx"] * lv0["ny"] * (lv0["nz_local"] if cfg["dim"] == 3 else 1)
    free_b, total_b = torch.cuda.mem_get_info(local)

    def barrier_sync():
        ctx.sync()
        torch.cuda.synchronize(local)
        if world > 1:
            dist.barrier()

    # the copy-bandwidth probe (the line's measured copy peak) runs before the warmup cycles: it is the run's first
    # sustained GPU load, so the clocks have ramped when the warmup starts (MGP_BENCH_PROBE_LATE=1: after the timing)
    copy_peak = None
    probe_first = os.environ.get("MGP_BENCH_PROBE_LATE", "0") == "0"
    if primary and a.copy_probe_mb > 0 and local == 0 and rank == 0 and probe_first:
        copy_peak = mgpoisson.copy_bandwidth(local, a.copy_probe_mb << 20, 10)
    # warmup (untimed; also captures the hipGraphs of the cycle)
    if warmup:
        ctx.cycles(warmup)
    barrier_sync()
    t0 = time.perf_counter()
    errs = ctx.cycles(steps)
    barrier_sync()
    dt = time.perf_counter() - t0

    # roofline window: the same K cycles again, launched eagerly with a HIP event pair around
    # every timed level-0 launch and every exchange / collective on the stream it runs on (graph replay cannot
    # bracket single launches); the kernels are identical, only the host launch path differs
    timed, launched = {}, {}
    if not a.no_timing:
        ctx.timing(True)
        ctx.cycles(steps)
        timed = ctx.timing_read()
        launched = ctx.timing_kernels()  # (before mgp_timing(c, 0), which resets the record)
        ctx.timing(False)
        barrier_sync()

    if primary and a.copy_probe_mb > 0 and local == 0 and rank == 0 and not probe_first:
        copy_peak = mgpoisson.copy_bandwidth(local, a.copy_probe_mb << 20, 10)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    comm = {k: timed.get(k, (0.0, 0, 0.0)) for k in ("exchange", "collective")}
    comm_all = [comm]
    if world > 1:
        comm_all = [None] * world
        dist.all_gather_object(comm_all, comm)

    value = (1 if strong else world) * steps / dt
    kind = "V" if a.cycle == "V" else "F"
    gcells = box[0] * box[1] * box[2]
    sm = "RB-GS" if a.smoother == "rbgs" else "Jacobi"
    pr = ("trilinear P" if cfg["dim"] == 3 else "bilinear P") if a.prolong == "linear" else "injection P"
    rs = (f"{'2x2x2' if cfg['dim'] == 3 else '2x2'}-average R" if a.restriction == "average"
          else "full-weighting R (adjoint of the linear P)")
    bc = "consistent coarse boundary" if a.coarse_bc == "consistent" else "ghost-0 coarse boundary"
    algo = f"{sm} {a.nu}+{a.nu}, {kind}-cycle, {pr}, {rs}, {bc}, per-cycle RMS-update err"
    if strong:
        named = {nb: label for _, nb, _, label in NORTH_STAR}
        slab = {(2048, 2048, 256): "one rank's slab of BASELINE configs[3] (2048^3 / 8 ranks)",
                (4096, 4096, 512): "one rank's slab of BASELINE configs[4] (4096^3 / 8 ranks)"}
        wl = named.get(box) or (slab.get(box) if world == 1 else None) or f"3D Poisson {box[0]}x{box[1]}x{box[2]}"
        workload = f"{wl}, 7-point, {algo}"
        unit = f"{kind}-cycles/s ({box[0]}x{box[1]}x{box[2]} box, whole job)"
    elif cfg["dim"] == 2:
        uf_mb = 2 * n * n * rb / 1e6
        tag = ("BASELINE configs[0] (the cpu.lua reference path)" if a.config0
               else "BASELINE configs[1]" if n == 4096 else "2D")
        workload = (f"{tag}: 2D Poisson {n}^2, 5-point, {algo}; u+f = {uf_mb:.0f} MB "
                    + ("fit the 256 MB Infinity Cache (MALL-resident: GB/s can exceed HBM)" if uf_mb < 256
                       else "exceed the 256 MB Infinity Cache"))
        unit = f"{kind}-cycles/s ({n}^2)"
    else:
        tag = "BASELINE configs[2]: " if n == 512 else ""
        workload = f"{tag}3D Poisson {n}^3 per GPU, 7-point, {algo}"
        unit = f"{kind}-cycles/s ({n}^3-cell slabs, whole job)"
    rnorm, fnorm = ctx.residual_norm()
    ms_step = 1e3 * dt / steps
    line = {
        "metric": "V-cycles/sec + finest-smoother achieved HBM GB/s, 3D Poisson",
        "value": value,
        "unit": unit,
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f32" if a.real == "float" else "f64",
        "data": "synthetic point-charge RHS (cpu.lua:182-193), psi0 = -f",
        "config": {
            "workload": workload,
            "global_box": list(box),
            "rank_slab": [lv0["nx"], lv0["ny"], lv0["nz_local"]],
            "parallelism": (f"slab-z x{world} (RCCL halo exchange)" if world > 1 else "single GPU"),
            "levels": len(ctx.levels),
        },
        "final_err": float(errs[-1]),
        "relative_residual": rnorm / fnorm,
        "hbm_used_GB_rank0": (total_b - free_b) / 1e9,
    }
    if world > 1:
        # per rank and cycle: halo exchanges (grouped send/recv, either stream) and the all-gather / err all-reduce,
        # HIP-event time on the stream they run on (includes waiting for the neighbour), and what the rank sends
        line["comm_per_rank"] = [
            {"exchange_ms_per_cycle": r["exchange"][0] / steps, "exchanges_per_cycle": r["exchange"][1] / steps,
             "exchange_MB_sent_per_cycle": r["exchange"][2] / steps / 1e6,
             "collective_ms_per_cycle": r["collective"][0] / steps,
             "collectives_per_cycle": r["collective"][1] / steps} for r in comm_all]
    tname = "float" if a.real == "float" else "double"
    lin = 1 if a.prolong == "linear" else 0
    fw = a.restriction == "full_weighting"
    kz = "k_zs" if cfg["dim"] == 3 else "k_ys"  # the temporally blocked phases: planes / rows streamed
    # PRE's LINEAR: 0 the average restriction inside, 1 smoothing only (the full weighting after it), 2 the full weighting
    # inside (fp32 3D one-rank levels: mgp_kernels.hip fused_fwf_supported)
    pre_lin = (2 if (tname == "float" and cfg["dim"] == 3 and world == 1) else 1) if fw else 0
    kernels = {"half_sweep": f"k_half<{tname}, {cfg['dim']}, 1, false>",
               "fused_pre": f"{kz}<{tname}, true, {pre_lin}, false, true>",
               "fused_post": f"{kz}<{tname}, false, {lin}, true, true>"}
    coarse = 0.5 ** cfg["dim"]
    # SURVEY.md §8(d) per-sweep accounting (what one launch per half-sweep would move) of the fused phases
    per_sweep = {"half_sweep": 1.5, "fused_pre": 3.0 * a.nu + 2.0 + coarse, "fused_post": 3.0 * a.nu + 2.0 + coarse + 2.0}
    per_kind = {k: v for k, v in timed.items() if k in kernels and v[1] > 0}
    # the fused kinds' kernels as the library launched them (symbol and grid: mgp_timing_kernel), not re-derived
    for k, (nm, _) in launched.items():
        if k in kernels:
            kernels[k] = nm
    cells = cells_rank
    if per_kind:
        # per kind: (ms, launches, algorithmic bytes as the library counts them: include/mgpoisson.h
        # MGP_TIMING_*, DESIGN.md §4 — read black u and f, write black u and R / 2^dim for PRE; read black u,
        # V / 2^dim, f, psiOld, write u for POST)
        kinds = {k: (ms, cnt, by) for k, (ms, cnt, by) in per_kind.items()}
        line["level0_kernels"] = {
            k: {"kernel": kernels[k], "launches": cnt, "avg_us": 1e3 * ms / cnt,
                "algorithmic_bytes_per_launch": by / cnt, "achieved_GBps": by / (ms * 1e-3) / 1e9,
                "per_sweep_accounting_bytes_per_launch": per_sweep[k] * rb * cells,
                "effective_GBps_per_sweep_accounting": per_sweep[k] * rb * cells * cnt / (ms * 1e-3) / 1e9}
            for k, (ms, cnt, by) in kinds.items()}
        dom = max(kinds, key=lambda k: kinds[k][0])  # the kernel with the most level-0 time
        ms, cnt, by = kinds[dom]
        achieved = by / (ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS, "traffic": None, "kernel": kernels[dom],
                "algorithmic_bytes_per_launch": by / cnt, "avg_launch_us": 1e3 * ms / cnt,
                "window": f"{steps} cycles after the timed region, HIP events around each launch"}
        cyc_bytes = cycle_compulsory_bytes(ctx.levels, cfg, a, rb)
        roof["cycle_compulsory_bytes"] = cyc_bytes
        roof["cycle_frac"] = cyc_bytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBPS
        roof["cycle_frac_definition"] = ("compulsory bytes of every level of one cycle (fused / tiled levels: their "
                                         "phases' algorithmic bytes; per-piece levels: SURVEY §8(d) W; F-cycle: level "
                                         "l visited l+1 times) / ms_per_step / 8 TB/s")
        # PMC traffic is measured by a separate rocprofv3 pass (tools/gpu_round.sh), never in this run; it
        # is used only when it was measured on this exact kernel source and workload
        if copy_peak:
            roof["measured_copy_peak"] = copy_peak
            roof["frac_of_measured_copy_peak"] = achieved / copy_peak
            roof["copy_probe"] = (f"mgp_copy_bandwidth: 16-byte streaming copy of {a.copy_probe_mb} MiB, best of 10, "
                                  "read + write bytes (BASELINE.md: measured copy-kernel peak)")
        roof["traffic_measured_this_run"] = False
        if dom in launched:
            roof["grid"] = launched[dom][1]
        wkey = workload_key(a, box, world)
        want = {k: launched[k] for k in kinds if k in launched}
        tpath, tr, why = pick_traffic(a.traffic, wkey, want)
        roof["traffic_source"] = os.path.relpath(tpath, ROOT) if tpath else None
        roof["traffic_source_matches_build"] = tpath is not None
        if not tpath:
            roof["traffic_rejected"] = why  # per candidate file: why it does not describe this run's launches
        else:
            tk = tr["kernels"]
            ent = tk[launched[dom][0]] if dom in launched else None
            if ent:
                roof["traffic"] = ent["bytes_per_launch"]
                roof["traffic_ratio"] = ent["bytes_per_launch"] / (by / cnt)
            # the measured counterpart of BASELINE's "finest-smoother achieved HBM GB/s": the PMC bytes of the
            # level-0 smoothing phases (PRE + POST) over their event-timed duration
            fin = [(tk[launched[k][0]]["bytes_per_launch"], kinds[k]) for k in ("fused_pre", "fused_post")
                   if k in kinds and k in launched]
            if len(fin) == 2:
                byt = sum(b * c for b, (_, c, _) in fin)
                sec = sum(ms_ for _, (ms_, _, _) in fin) * 1e-3
                line["finest_level_hbm_GBps"] = {
                    "value": byt / sec / 1e9, "pmc_bytes_per_cycle": byt / steps, "kernel_us_per_cycle": 1e6 * sec / steps,
                    "source": roof["traffic_source"],
                    "definition": "PMC-measured HBM bytes (FETCH_SIZE x2 + WRITE_SIZE, tools/pmc_traffic.py) of the "
                                  "finest level's PRE and POST launches over their HIP-event time: bytes actually "
                                  "moved, bounded by 8 TB/s (finest_smoother_GBps is the per-sweep-equivalent figure)"}
        line["roofline"] = roof
        # finest-smoother GB/s = 3 sizeof(real) cells_per_rank sweeps / summed smoother kernel time
        # (the level-0 smoothing launches; a fused phase is counted with its nu sweeps)
        sweeps = sum(cnt * (1 if k == "half_sweep" else a.nu) / (2 if k == "half_sweep" else 1)
                     for k, (ms_, cnt, _) in kinds.items())
        tsum = sum(ms_ for ms_, _, _ in kinds.values()) * 1e-3
        line["finest_smoother_GBps"] = {
            "value": 3 * rb * cells * sweeps / tsum / 1e9, "sweeps_timed": sweeps, "kernel_s": tsum,
            "definition": "BASELINE.md: 3 sizeof(real) cells_per_rank sweeps / summed finest-level smoothing kernel "
                          "time; the temporally blocked phases do nu sweeps per launch from one read of the level, so "
                          "this per-sweep figure is bounded by 8 TB/s x (sweeps per compulsory pass), not 8 TB/s"}

    if primary and rank == 0 and world == 1 and a.cpu_cycles > 0:
        thr = a.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
        # configs[0] is small: the CPU port runs the same cycles the GPU timed, in full
        c_omp, c_one = (steps, steps) if a.config0 else (a.cpu_cycles, max(1, a.cpu_cycles // 2))
        line["cpu_baseline"] = cpu_baseline(cfg, c_omp, thr, gcells, a.cpu_reps)
        line["cpu_baseline_1thread"] = cpu_baseline(cfg, c_one, 1, gcells, a.cpu_reps)
    ctx.close()
    return line


def pick_traffic(paths, wkey, launched, src_hash=None):
    """(path, json, rejected) of the first traffic JSON of the comma list that describes this run's launches: measured
    on this build (source hash), on this workload (workload_key: box, ranks and options — not merely the same cell
    count, which 2048^3 and 4096^2 x 512 share) and holding every timed kernel `launched` = {kind: (symbol, grid)}
    with the same grid.  Else (None, None, {path: reason}): the line then carries traffic null."""
    src_hash = src_hash or source_hash()
    rejected = {}
    for p in (paths or "").split(","):
        if not p or not os.path.exists(p):
            continue
        try:
            with open(p) as fh:
                tr = json.load(fh)
        except (OSError, ValueError) as e:
            rejected[os.path.relpath(p, ROOT)] = f"unreadable: {e}"
            continue
        tk = tr.get("kernels", {})
        key = os.path.relpath(p, ROOT)
        if tr.get("source_hash") != src_hash:
            rejected[key] = f"measured on source {tr.get('source_hash')}, this build is {src_hash}"
        elif tr.get("workload") != wkey:
            rejected[key] = f"measured on workload {tr.get('workload')}"
        elif not launched:
            rejected[key] = "no timed launch to match"
        else:
            bad = [f"{nm} grid {g}" for nm, g in launched.values() if tk.get(nm, {}).get("grid") != g]
            if bad:
                rejected[key] = "no measured launch of " + ", ".join(bad)
            else:
                return p, tr, None
    return None, None, rejected


def cycle_compulsory_bytes(levels, cfg, a, rb):
    """Compulsory HBM bytes of one cycle: per level the cells x reals a level must move — fused
    (k_zs / k_ys) and tiled (k_blk, tail) levels their phases' algorithmic reals (PRE 2 + 2^-d, POST 2.5 + 2^-d,
    + 1 psiOld with the err on level 0), per-piece levels SURVEY §8(d)'s W = (nu1 + nu2) 3 + 2 (2 + 2^-d)
    (+ 1 psiOld on level 0); F-cycle: level l is visited l + 1 times."""
    d = cfg["dim"]
    coarse = 0.5 ** d
    total = 0.0
    for l, lv in enumerate(levels):
        cells = lv["nx"] * lv["ny"] * (lv["nz_local"] if d == 3 else 1)
        last = l == len(levels) - 1
        if last:
            reals = 2.0  # coarse solve: read f, write u
        elif lv["engine"] == "piece":
            reals = 3.0 * 2 * a.nu + 2 * (2 + coarse)
        elif lv["engine"] == "zpost":  # PRE per piece (nu sweeps + residual / restriction), POST temporally blocked
            reals = 3.0 * a.nu + (2 + coarse) + (2.5 + coarse)
        else:
            reals = (2 + coarse) + (2.5 + coarse)
        if l == 0:
            reals += 1.0  # psiOld of the err
        visits = (l + 1) if a.cycle == "F" else 1
        total += visits * reals * rb * cells
    return total


def plan_only(a, cfg, box, rank, world, dist):
    """--plan-only: every rank computes its level plan exactly as mgp_create would (mgp_plan: slab, ghost
    depth rules, engines), the plans are gathered over the process group, and rank 0 checks that the ranks
    agree on the hierarchy and that the distributed levels' slabs tile the box in rank order, then prints one
    JSON line.  Exercises the N > 1 launch path of this script without a GPU (tests/test_bench_launch.py)."""
    import mgpoisson

    mine = mgpoisson.plan(mgpoisson.make_opts(**cfg))
    plans = [mine]
    if world > 1:
        plans = [None] * world
        dist.all_gather_object(plans, mine)
    if rank == 0:
        nl = len(plans[0])
        assert all(len(p) == nl for p in plans), "ranks disagree on the number of levels"
        for l in range(nl):
            rows = [p[l] for p in plans]
            for key in ("nx", "ny", "nz_global", "distributed", "engine"):
                assert len({r[key] for r in rows}) == 1, f"level {l}: ranks disagree on {key}"
            if rows[0]["distributed"]:
                z = 0
                for r in rows:
                    assert r["z0"] == z, f"level {l}: slab of rank {rows.index(r)} starts at {r['z0']}, expected {z}"
                    z += r["nz_local"]
                assert z == rows[0]["nz_global"], f"level {l}: slabs cover {z} of {rows[0]['nz_global']} planes"
            else:
                assert all(r["z0"] == 0 and r["nz_local"] == r["nz_global"] for r in rows), f"level {l}: replicated"
        out = {"plan_only": True, "n_gpus": world, "global_box": list(box), "levels": nl,
               "distributed_levels": sum(1 for r in plans[0] if r["distributed"]),
               "engines": [r["engine"] for r in plans[0]],
               "rank_slabs_level0": [[r[0]["z0"], r[0]["nz_local"]] for r in plans],
               "comm_id_bytes": len(cfg["comm_id"] or b""),
               "comm_per_cycle": comm_schedule(cfg)}
        if want_north_star(a, world):
            out["north_star_lines"] = {}
            for name, nbox, cyc, _ in NORTH_STAR:
                if nbox[2] % world or nbox[2] // world < 2:
                    continue
                ns = argparse.Namespace(**vars(a))
                ns.cycle, ns.box = cyc, ",".join(map(str, nbox))
                ncfg = make_cfg(ns, nbox, 0, world, 0, cfg["comm_id"])
                fit = fits_hbm(ncfg, world, 0, total=288e9)  # MI355X: 288 GB of HBM3E per GPU
                out["north_star_lines"][name] = {"global_box": list(nbox), "cycle": cyc, "fits": fit is not None,
                                                 "comm_per_cycle": comm_schedule(ncfg)}
            if world == 1:
                out["fp64_line"] = True
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def comm_schedule(cfg):
    """Rank 0's RCCL calls of one steady cycle (the second: the first also exchanges f once), from the library's
    host-only dry run of the cycle (mgp_plan_comm): calls per kind and bytes this rank sends."""
    import mgpoisson

    if cfg["world"] == 1:
        return {"calls": 0}
    one = len(mgpoisson.plan_comm(mgpoisson.make_opts(**cfg), 1))
    log = mgpoisson.plan_comm(mgpoisson.make_opts(**cfg), 2)[one:]
    nb = 1  # rank 0 has one neighbour; interior ranks send the same to each of their two
    out = {"calls": len(log), "halo_exchanges": sum(1 for r in log if r[0] == "exchange"),
           "side_stream_exchanges": sum(1 for r in log if r[0] == "exchange" and r[1]),
           "allgathers": sum(1 for r in log if r[0] == "allgather"),
           "allreduces": sum(1 for r in log if r[0] == "allreduce"),
           "halo_MB_per_neighbour": sum(r[4] for r in log if r[0] == "exchange") * nb / 1e6,
           "allgather_MB": sum(r[4] for r in log if r[0] == "allgather") / 1e6,
           "sequence": [list(r) for r in log]}
    return out


def source_hash():
    """sha256 (16 hex) of the library's kernel and ABI sources: tags PMC traffic to the build it measured."""
    import hashlib

    import glob

    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "lua-multigrid-poisson_amd", "csrc")
    for f in sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.cpp")) +
                    glob.glob(os.path.join(csrc, "*.h"))):
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def cpu_baseline(cfg, cycles, threads, gcells, reps=3):
    """The C oracle (the build's restatement of the reference CPU path) on this host, best of `reps` samples of
    `cycles` cycles each (best of 3).

    Bounded sample: the workload itself when it has <= 512^3 cells, else a 512^3 (3D) box of the same
    algorithm, scaled to the workload by cells (labelled extrapolated)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import Oracle

    kw = {k: cfg[k] for k in ("dim", "n", "real", "smoother", "nu1", "nu2", "cycle", "prolong", "coarse_bc", "coarse_init",
                              "restriction")}
    scale = 1.0
    if gcells > 512 ** 3:
        kw["n"] = (512, 512, 512)
        scale = 512 ** 3 / gcells
    o = Oracle(threads=threads, **kw)
    o.init_point_charge()
    samples = []
    for _ in range(max(1, reps)):
        t0 = time.perf_counter()
        for _ in range(cycles):
            o.step()
        samples.append(time.perf_counter() - t0)
    dt = min(samples)
    n = kw["n"]
    kind = "V" if cfg["cycle"] == "V" else "F"
    sample = (f"best of {len(samples)} samples of {cycles} full {kind}-cycles of {n[0]}x{n[1]}x"
              f"{n[2] if cfg['dim'] == 3 else 1} with the same algorithm, oracle/mgp_oracle.c (gcc -O2, "
              f"-ffp-contract=off), {threads} thread(s), {dt:.1f} s each (all: "
              + ", ".join(f"{s:.1f}" for s in samples) + " s)")
    if scale != 1.0:
        sample += "; EXTRAPOLATED to the workload's cells (x %.3g)" % scale
    return {"value": scale * cycles / dt, "unit": f"{kind}-cycles/s (same workload)", "cores": threads,
            "kind": "port", "sample": sample}


if __name__ == "__main__":
    main()
