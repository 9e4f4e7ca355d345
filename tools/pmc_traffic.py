#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 --pmc passes (tools/pmc.sh output).

FETCH_SIZE and WRITE_SIZE are in KiB.  MI355X_MICROARCH.md (HBM / rocprofv3 section): on gfx950
FETCH_SIZE reports exactly half of the bytes of wide coalesced streaming reads, so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane streaming stores.  Output: per kernel (name, grid) the mean
bytes per launch; with an output path, a JSON file bench.py --traffic reads:
{"kernels": {name: {grid, launches, read_bytes, write_bytes, bytes_per_launch}}, "method": ...}
holding, per kernel name, the launch grid with the most bytes (the finest level's launches).

usage: tools/pmc_traffic.py gpurun_out/pmc [out.json ["bench args of the measured run"]]
The JSON carries the source hash of the library it measured (bench.py source_hash()) and the workload key of
the bench arguments the passes ran (bench.workload_key: box, ranks, options); bench.py uses the traffic only
when both match its own run and every timed launch's kernel and grid is in the file (bench.pick_traffic).
"""
import collections
import csv
import glob
import json
import os
import re
import shlex
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
out = sys.argv[2] if len(sys.argv) > 2 else None
bench_args = sys.argv[3] if len(sys.argv) > 3 else ""
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import source_hash, workload_key_from_argv  # noqa: E402

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

if out:
    kernels = {}
    for name, grid, fetch, write, n in rows:  # sorted by bytes: the first row per name is the largest
        if name not in kernels:
            kernels[name] = {"grid": grid, "launches": n, "read_bytes": fetch, "write_bytes": write,
                             "bytes_per_launch": fetch + write}
    json.dump({"kernels": kernels, "source_hash": source_hash(),
               "workload": workload_key_from_argv(shlex.split(bench_args)), "bench_args": bench_args,
               "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over bench.py, KiB -> B, "
                         "FETCH_SIZE x2 (gfx950 wide-load correction, MI355X_MICROARCH.md); per kernel the "
                         "launch grid with the most bytes"}, open(out, "w"), indent=1)
    print("wrote", out)
