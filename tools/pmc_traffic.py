#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 --pmc passes (tools/pmc.sh output).

FETCH_SIZE and WRITE_SIZE are in KiB.  MI355X_MICROARCH.md (HBM / rocprofv3 section): on gfx950
FETCH_SIZE reports exactly half of the bytes of wide coalesced streaming reads, so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane streaming stores.  Output: per kernel (name, grid) the mean
bytes per launch, and for the finest smoother half-sweep a JSON file bench.py --traffic reads.

usage: tools/pmc_traffic.py gpurun_out/pmc [out.json]
"""
import collections
import csv
import glob
import json
import os
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
out = sys.argv[2] if len(sys.argv) > 2 else None

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for path in glob.glob(os.path.join(root, "p*", "*counter_collection.csv")):
    for r in csv.DictReader(open(path)):
        m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:40]
        vals[(name, int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))

rows = []
for (name, grid), cs in vals.items():
    if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
        continue
    fetch = 2.0 * 1024 * sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"])
    write = 1024 * sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"])
    rows.append((name, grid, fetch, write, len(cs["FETCH_SIZE"])))
rows.sort(key=lambda r: -(r[2] + r[3]))
for name, grid, fetch, write, n in rows[:20]:
    print(f"{name[:46]:46s} {grid:>10d} x{n:<4d} read {fetch/1e6:9.2f} MB  write {write/1e6:9.2f} MB")

fine = [r for r in rows if re.match(r"k_half<float, 3, 1, false>", r[0])]
if fine and out:
    name, grid, fetch, write, n = max(fine, key=lambda r: r[1])
    json.dump({"kernel": name, "grid": grid, "launches": n, "read_bytes": fetch, "write_bytes": write,
               "bytes_per_launch": fetch + write,
               "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, KiB -> B, FETCH_SIZE x2 "
                         "(gfx950 wide-load correction, MI355X_MICROARCH.md)"}, open(out, "w"), indent=1)
    print("wrote", out)
