#!/usr/bin/env python3
"""One cycle of a rocprofv3 kernel trace, kernel by kernel (cycles delimited by the err sum k_sum_n).
usage: cycle_breakdown.py run_kernel_trace.csv [cycle index from the end, default 3] [kernel=grid]
With kernel=grid (e.g. "k_zs<float, true, 0=114688"), the index counts only the cycles holding a launch of that kernel
with that grid size (a trace of bench.py's default run also holds its fp64 and north-star lines)."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
back = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ends = [i for i, r in enumerate(rows) if "k_sum_n" in r["Kernel_Name"]]
pairs = list(zip(ends[:-1], ends[1:]))
if len(sys.argv) > 3:
    kname, grid = sys.argv[3].rsplit("=", 1)
    pairs = [(a, b) for a, b in pairs
             if any(kname in r["Kernel_Name"] and r["Grid_Size_X"] == grid for r in rows[a + 1:b + 1])]
a, b = pairs[-back]
busy = 0
for r in rows[a + 1:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    n = re.search(r"(k_\w+(<[^>]*>)?|__amd\w+)", r["Kernel_Name"]).group(1)
    print(f"{n[:44]:44s} grid {int(r['Grid_Size_X']):>9d} {(e - s) / 1e3:8.1f} us")
print(f"busy {busy / 1e3:.1f} us, period {(int(rows[b]['End_Timestamp']) - int(rows[a]['End_Timestamp'])) / 1e3:.1f} us")
