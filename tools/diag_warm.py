#!/usr/bin/env python3
"""Per-cycle wall time of the bench workload from a fresh context (where the warm-up goes).

Runs the bench's 512^3 fp32 RB-GS 2+2 V-cycle one cycle per mgp_cycles(1) call (synchronised, so
each time includes ~20 us of host overhead) and prints the times of the first K cycles, then K
cycles in one call.  Used to see how many replays the clocks / graph caches need to settle.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lua-multigrid-poisson_amd"))
import mgpoisson  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    cfg = dict(dim=3, n=(n, n, n), real="float", smoother="rbgs", nu1=2, nu2=2, cycle="V", prolong="linear",
               coarse_bc="consistent", coarse_init="fresh", err_mode=1, device=0)
    t0 = time.perf_counter()
    ctx = mgpoisson.Context(mgpoisson.make_opts(**cfg))
    ctx.init_point_charge()
    print(f"create+init {1e3 * (time.perf_counter() - t0):.1f} ms")
    ts = []
    for _ in range(k):
        t = time.perf_counter()
        ctx.cycles(1)
        ts.append(1e3 * (time.perf_counter() - t))
    print("per-cycle ms:", " ".join(f"{x:.3f}" for x in ts))
    for rep in range(3):
        t = time.perf_counter()
        ctx.cycles(20)
        print(f"20 cycles in one call, rep {rep}: {1e3 * (time.perf_counter() - t) / 20:.4f} ms/cycle")
    ctx.close()


if __name__ == "__main__":
    main()
