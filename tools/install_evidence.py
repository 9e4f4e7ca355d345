#!/usr/bin/env python3
"""Copy the end-of-round evidence in gpurun_out/ (tools/r06_final.sh) into profiles/
under a round prefix and print the bench lines.

usage: tools/install_evidence.py [prefix]   (default r03)

Files: <p>_pytest_gpu.txt, <p>_pmc_traffic.json (+ pmc_traffic_current.json, read by bench.py when its source
hash matches the build), <p>_pmc_traffic_summary.txt, <p>_kernel_stats.csv / <p>_trace_summary.txt /
<p>_cycle_breakdown.txt (rocprofv3 --kernel-trace --stats of the default bench command), <p>_2d_* (the same for
BASELINE configs[1]), <p>_bench.json (default bench line with PMC traffic) and one <p>_bench_*.json per config line.
"""
import json
import os
import shutil
import subprocess
import sys

P = "profiles/"
G = "gpurun_out/"
pre = sys.argv[1] if len(sys.argv) > 1 else "r03"


def last(p):
    return [l for l in open(p) if l.startswith("{")][-1]


def tool(args, out):
    with open(P + out, "w") as fh:
        subprocess.run([sys.executable] + args, stdout=fh, check=True)


shutil.copy(G + "pmc_traffic.json", P + f"{pre}_pmc_traffic.json")
shutil.copy(G + "pmc_traffic.json", P + "pmc_traffic_current.json")
shutil.copy(G + "pmc_traffic.txt", P + f"{pre}_pmc_traffic_summary.txt")
shutil.copy(G + "prof/run_kernel_stats.csv", P + f"{pre}_kernel_stats.csv")
# PMC traffic of the other workloads (tools/r06_final.sh), each tagged with its workload key; read by bench.py's
# --traffic default
for w in ("slab4", "slab3", "box2048", "fw", "2d", "2d64", "f64"):
    if os.path.exists(G + f"pmc_traffic_{w}.json"):
        shutil.copy(G + f"pmc_traffic_{w}.json", P + f"pmc_traffic_{w}.json")
        shutil.copy(G + f"pmc_traffic_{w}.txt", P + f"{pre}_pmc_traffic_{w}_summary.txt")
if os.path.exists(G + "fetch_calib.json"):
    shutil.copy(G + "fetch_calib.json", P + f"{pre}_fetch_calib.json")
if os.path.exists(G + "pytest_gpu.log") and os.path.exists(G + "smoke.log"):
    tail = [l for l in open(G + "pytest_gpu.log").read().splitlines() if l.strip()][-1:]
    smoke = [l for l in open(G + "smoke.log").read().splitlines() if l.startswith("smoke")]
    open(P + f"{pre}_pytest_gpu.txt", "w").write("\n".join(tail + smoke) + "\n")
if os.path.isdir(G + "sq"):  # SQ / TCC counter passes (tools/r04_final.sh)
    tool(["tools/pmc_summary.py", G + "sq", "k_zs|k_tail_c|k_fresh"], f"{pre}_sq_counters_summary.txt")
tool(["tools/trace_summary.py", G + "prof/run_kernel_trace.csv"], f"{pre}_trace_summary.txt")
tool(["tools/cycle_breakdown.py", G + "prof/run_kernel_trace.csv", "3", "k_zs<float, true, 0, false, true, false>=114688"],
     f"{pre}_cycle_breakdown.txt")
if os.path.exists(G + "prof2d/run_kernel_stats.csv"):
    shutil.copy(G + "prof2d/run_kernel_stats.csv", P + f"{pre}_2d_kernel_stats.csv")
    tool(["tools/trace_summary.py", G + "prof2d/run_kernel_trace.csv"], f"{pre}_2d_trace_summary.txt")
    tool(["tools/cycle_breakdown.py", G + "prof2d/run_kernel_trace.csv", "8"], f"{pre}_2d_cycle_breakdown.txt")

for w in ("fw", "f64"):  # one workload per trace: the full-weighting and fp64 512^3 lines
    if os.path.exists(G + f"prof{w}/run_kernel_stats.csv"):
        shutil.copy(G + f"prof{w}/run_kernel_stats.csv", P + f"{pre}_{w}_kernel_stats.csv")
        tool(["tools/cycle_breakdown.py", G + f"prof{w}/run_kernel_trace.csv", "8"], f"{pre}_{w}_cycle_breakdown.txt")

open(P + f"{pre}_bench.json", "w").write(last(G + "bench.log"))
files = [f"{pre}_bench.json"]
i = 1
while os.path.exists(G + f"bench_{i}.log"):
    d = json.loads(last(G + f"bench_{i}.log"))
    c = d["config"]
    box = "x".join(str(v) for v in c["global_box"] if v > 1)
    tag = f"{pre}_bench_{i}_{d['dtype']}_{box}" + ("_F" if d["unit"].startswith("F") else "")
    if "configs[0]" in c["workload"]:
        tag += "_config0"
    if "full-weighting" in c["workload"]:
        tag += "_fw"
    if d["steps"] == 20 and d["warmup"] == 5:
        tag += "_driver20x5"
    open(P + tag + ".json", "w").write(json.dumps(d) + "\n")
    files.append(tag + ".json")
    i += 1
for f in files:
    d = json.loads(open(P + f).read())
    r, c = d.get("roofline", {}), d.get("cpu_baseline", {})
    print(f, round(d["value"], 1), round(d["ms_per_step"], 4), r.get("kernel", "")[:32], round(r.get("achieved", 0)),
          round(r.get("frac", 0), 3), r.get("traffic"), round(c.get("value", 0), 3))
d = json.loads(open(P + f"{pre}_bench.json").read())
for k, v in d.get("level0_kernels", {}).items():
    print(k, round(v["avg_us"], 1), round(v["achieved_GBps"]))
