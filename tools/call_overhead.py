"""Fixed cost of one mgp_cycles(k) call (graph launches, the err counter reset, the stream sync, the err read-back):
times ctx.cycles(k) for several k after a warm-up and fits t = a + b k (a: per call, b: per cycle).

usage: python3 tools/call_overhead.py [bench args...]  (default workload: bench.py's)"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import bench  # noqa: E402


def main():
    a = bench.parse(sys.argv[1:])
    box, _ = bench.workload_box(a, 1)
    cfg = bench.make_cfg(a, box, 0, 1, 0, None)
    import mgpoisson

    ctx = mgpoisson.Context(mgpoisson.make_opts(**cfg))
    ctx.init_point_charge()
    ctx.cycles(200)
    ctx.sync()
    ks = [1, 2, 5, 10, 20, 50, 100, 200, 500]
    rows = []
    for rep in range(3):
        for k in ks:
            ctx.sync()
            t0 = time.perf_counter()
            ctx.cycles(k)
            dt = time.perf_counter() - t0
            rows.append((k, dt))
            print(f"k={k:4d} rep {rep}: {1e3 * dt:.4f} ms  ({1e3 * dt / k:.4f} ms/cycle)", flush=True)
    n = len(rows)
    mk = sum(k for k, _ in rows) / n
    mt = sum(t for _, t in rows) / n
    b = sum((k - mk) * (t - mt) for k, t in rows) / sum((k - mk) ** 2 for k, _ in rows)
    a0 = mt - b * mk
    out = {"workload": " ".join(sys.argv[1:]) or "default", "per_call_ms": 1e3 * a0, "per_cycle_ms": 1e3 * b,
           "min_by_k_ms": {k: 1e3 * min(t for kk, t in rows if kk == k) for k in ks}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
