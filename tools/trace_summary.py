#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_trace.csv: time per (kernel, grid) and per-cycle wall/busy."""
import collections
import csv
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
rows = list(csv.DictReader(open(path)))


def name(r):
    m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
    return m.group(1) if m else r["Kernel_Name"][:40]


d = collections.defaultdict(list)
for r in rows:
    d[(name(r), int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = sum(sum(v) for v in d.values())
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(f"{k[0][:46]:46s} {k[1]:>10d} {len(v):>5d} {sum(v)/len(v):9.1f} us {100*sum(v)/tot:5.1f}%")
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# Cycles start at the finest level's PRE phase (the temporally blocked k_zs / k_ys PRE); without it, at the
# finest-level plain half-sweep that follows a coarse-tail launch.  (Round 2 delimited by k_sum_n, which
# k_resnorm's reduction launches too: its "per cycle" line mixed cycles and norm evaluations.)
delim = sys.argv[3] if len(sys.argv) > 3 else r"k_(zs|ys)<\w+, true"
starts = [i for i, r in enumerate(rows) if re.search(delim, r["Kernel_Name"])]
if len(starts) > 6:
    a, b = starts[-6], starts[-1]
    seg = rows[a:b]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    print(f"per cycle (last 5, delimited by /{delim}/): wall {(t1-t0)/5e6:.3f} ms, busy {busy/5e6:.3f} ms, "
          f"launches {len(seg)/5:.0f}")
