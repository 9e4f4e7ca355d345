#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration by load width on gfx950.

MI355X_MICROARCH.md documents the correction for 16-byte-per-lane streaming loads (FETCH_SIZE reports half of
the bytes).  k_zs POST (fp32) reads with 8-byte lanes and scalar coarse loads, so its factor is measured here:
copies of a known byte count with 16-, 8- and 4-byte lanes (mgp_copy_bandwidth with MGP_COPY_CALIB=1: kernels
k_copy16<0..2>, k_copy_w<8>, k_copy_w<4>), one rocprofv3 --pmc pass per counter.

  MGP_COPY_CALIB=1 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d OUT/p1 -o run -- \\
      python3 tools/fetch_calib.py run
  (same with WRITE_SIZE into OUT/p2)
  python3 tools/fetch_calib.py report OUT [out.json]
"""
import collections
import csv
import glob
import json
import os
import re
import sys

NBYTES = 1 << 30
REPS = 3


def run():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lua-multigrid-poisson_amd"))
    import mgpoisson

    assert os.environ.get("MGP_COPY_CALIB") == "1"
    print("copy GB/s", mgpoisson.copy_bandwidth(0, NBYTES, REPS))


def report(root, out=None):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(root, "p*", "*counter_collection.csv")):
        for r in csv.DictReader(open(path)):
            m = re.search(r"(k_copy\w*<\d+>)", r["Kernel_Name"])
            if m:
                vals[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for name, cs in sorted(vals.items()):
        row = {"bytes_read": NBYTES, "bytes_written": NBYTES}
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            if c in cs:
                v = sorted(cs[c])[len(cs[c]) // 2] * 1024  # median launch, KiB -> B
                row[c + "_bytes"] = v
                row[c + "_factor"] = NBYTES / v if v else None
        res[name] = row
        print(f"{name:16s} " + "  ".join(f"{k} {v:.3f}" for k, v in row.items() if k.endswith("factor") and v))
    if out:
        json.dump({"copy_bytes": NBYTES, "kernels": res,
                   "method": "median launch of each copy kernel; factor = known bytes / counter bytes"},
                  open(out, "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        report(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
