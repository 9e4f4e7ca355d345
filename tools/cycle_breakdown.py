#!/usr/bin/env python3
"""One cycle of a rocprofv3 kernel trace, kernel by kernel (cycles delimited by the err sum k_sum_n).
usage: cycle_breakdown.py run_kernel_trace.csv [cycle index from the end, default 3]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
back = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ends = [i for i, r in enumerate(rows) if "k_sum_n" in r["Kernel_Name"]]
a, b = ends[-back - 1], ends[-back]
busy = 0
for r in rows[a + 1:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    n = re.search(r"(k_\w+(<[^>]*>)?|__amd\w+)", r["Kernel_Name"]).group(1)
    print(f"{n[:44]:44s} grid {int(r['Grid_Size_X']):>9d} {(e - s) / 1e3:8.1f} us")
print(f"busy {busy / 1e3:.1f} us, period {(int(rows[b]['End_Timestamp']) - int(rows[a]['End_Timestamp'])) / 1e3:.1f} us")
