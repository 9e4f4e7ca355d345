"""Sustained-load soak of one bench workload on one GPU (evidence for DESIGN.md §7, round 6).

Runs the workload bench.py would run with the same arguments for --seconds of wall time, in hipGraph-replayed batches of
--batch cycles, re-initialising the point charge every --reinit batches (so the convergence path is exercised again),
and records per batch: ms per cycle, the err range, and whether every err is finite.  Reports the first / last / min /
max batch time (clock or thermal drift under sustained load) and writes one JSON summary.

usage: python3 tools/soak.py [--seconds 120] [--batch 200] [--reinit 10] [--out gpurun_out/soak.json] [bench args...]
"""
import json
import math
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import bench  # noqa: E402


def main():
    argv = sys.argv[1:]
    opts = {"--seconds": 120.0, "--batch": 200, "--reinit": 10, "--out": "gpurun_out/soak.json"}
    rest = []
    i = 0
    while i < len(argv):
        if argv[i] in opts:
            opts[argv[i]] = type(opts[argv[i]])(argv[i + 1])
            i += 2
        else:
            rest.append(argv[i])
            i += 1
    a = bench.parse(rest)
    box, _ = bench.workload_box(a, 1)
    cfg = bench.make_cfg(a, box, 0, 1, 0, None)
    import numpy as np
    import torch

    import mgpoisson

    ctx = mgpoisson.Context(mgpoisson.make_opts(**cfg))
    ctx.init_point_charge()
    ctx.cycles(10)  # warmup + graph capture
    ctx.sync()
    torch.cuda.synchronize(0)
    batches = []
    t_end = time.perf_counter() + opts["--seconds"]
    nb = 0
    while time.perf_counter() < t_end:
        if nb and nb % opts["--reinit"] == 0:
            ctx.init_point_charge()
        ctx.sync()
        t0 = time.perf_counter()
        errs = np.asarray(ctx.cycles(opts["--batch"]))
        ctx.sync()
        dt = time.perf_counter() - t0
        fin = bool(np.all(np.isfinite(errs)))
        batches.append({"ms_per_cycle": 1e3 * dt / opts["--batch"], "err_first": float(errs[0]),
                        "err_last": float(errs[-1]), "finite": fin})
        print(f"batch {nb}: {1e3 * dt / opts['--batch']:.4f} ms/cycle, err {errs[0]:.3e} -> {errs[-1]:.3e}"
              f"{'' if fin else ' NON-FINITE'}", flush=True)
        nb += 1
        if not fin:
            break
    ms = [b["ms_per_cycle"] for b in batches]
    out = {"workload": " ".join(rest) or "default", "seconds": opts["--seconds"], "batch_cycles": opts["--batch"],
           "batches": len(batches), "cycles": len(batches) * opts["--batch"],
           "all_finite": all(b["finite"] for b in batches),
           "ms_per_cycle": {"first": ms[0], "last": ms[-1], "min": min(ms), "max": max(ms),
                            "mean": sum(ms) / len(ms),
                            "stdev": math.sqrt(sum((x - sum(ms) / len(ms)) ** 2 for x in ms) / len(ms))},
           "per_batch": batches}
    os.makedirs(os.path.dirname(opts["--out"]) or ".", exist_ok=True)
    with open(opts["--out"], "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "per_batch"}), flush=True)
    return 0 if out["all_finite"] else 1


if __name__ == "__main__":
    sys.exit(main())
