#!/usr/bin/env python3
"""Print ms_per_step / value / level-0 kernel averages of the last bench JSON line in gpurun_out/<name>.log.
usage: tools/show_lines.py name [name ...]"""
import json
import os
import sys

for n in sys.argv[1:]:
    p = os.path.join("gpurun_out", n + ".log")
    if not os.path.exists(p):
        print(f"{n:10s} (no log)")
        continue
    lines = [json.loads(l) for l in open(p) if l.startswith("{")]
    if not lines:
        print(f"{n:10s} (no JSON line)")
        continue
    d = lines[-1]
    k = {kk: round(v["avg_us"], 1) for kk, v in d.get("level0_kernels", {}).items()}
    print(f"{n:10s} {d['ms_per_step']:.4f} ms  {d['value']:9.2f}  {k}")
