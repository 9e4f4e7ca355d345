#!/usr/bin/env python3
"""Per-kernel mean of every PMC counter collected by rocprofv3 --pmc passes.

usage: tools/pmc_summary.py <dir with p*/ pass subdirs> [kernel-regex] [out.json]

Prints, for each (kernel, grid) matching the regex (default: k_zs), the mean value per dispatch
of every counter found in any pass, plus derived ratios when their inputs are present:
  wait_frac      SQ_WAIT_ANY / SQ_WAVE_CYCLES        (waves parked on s_waitcnt / barrier)
  inst_stall     SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES   (issue stalls)
  active_frac    SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  lds_conflict   SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  eff_clock_GHz  GRBM_GUI_ACTIVE / 8 / kernel duration (needs the pass's kernel trace)
"""
import collections
import csv
import glob
import json
import os
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"k_zs")
out = sys.argv[3] if len(sys.argv) > 3 else None


def kname(s):
    m = re.search(r"(k_\w+(<[^>]*>)?)", s)
    return m.group(1) if m else s[:40]


vals = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(path)):
        name = kname(r["Kernel_Name"])
        if not pat.search(name):
            continue
        key = (name, int(r["Grid_Size"]))
        vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for extra in ("VGPR_Count", "SGPR_Count", "LDS_Block_Size", "Scratch_Size", "Workgroup_Size"):
            if extra in r and r[extra] != "":
                vals[key]["@" + extra] = [float(r[extra])]

res = {}
for key, cs in sorted(vals.items()):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    d = {}
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        for c, lab in (("SQ_WAIT_ANY", "wait_frac"), ("SQ_WAIT_INST_ANY", "inst_stall"),
                       ("SQ_ACTIVE_INST_ANY", "active_frac"), ("SQ_ACTIVE_INST_VALU", "valu_frac"),
                       ("SQ_ACTIVE_INST_LDS", "lds_frac"), ("SQ_WAIT_INST_LDS", "lds_issue_stall")):
            if c in m:
                d[lab] = m[c] / wc
    if m.get("SQ_LDS_IDX_ACTIVE"):
        d["lds_conflict"] = m.get("SQ_LDS_BANK_CONFLICT", 0.0) / m["SQ_LDS_IDX_ACTIVE"]
    res[f"{key[0]} grid={key[1]}"] = {"mean": m, "derived": d}
    print(f"== {key[0]}  grid={key[1]}")
    for c in sorted(m):
        print(f"   {c:28s} {m[c]:16.4g}")
    for c in sorted(d):
        print(f"   {c:28s} {d[c]:16.4f}")
if out:
    json.dump(res, open(out, "w"), indent=1)
