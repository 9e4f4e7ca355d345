#!/usr/bin/env python3
"""Copy the end-of-round evidence (tools/r02_final_all.sh output in gpurun_out/) into profiles/ and print
the bench lines.  usage: tools/install_evidence.py <gpurun log of that call>"""
import json
import shutil
import subprocess
import sys

P = "profiles/"
G = "gpurun_out/"
shutil.copy(G + "pmc_traffic.json", P + "r02_pmc_traffic.json")
shutil.copy(G + "pmc_traffic.json", P + "pmc_traffic_current.json")
shutil.copy(G + "pmc_traffic.txt", P + "r02_pmc_traffic_summary.txt")
shutil.copy(G + "prof/run_kernel_stats.csv", P + "r02_kernel_stats.csv")


def last(p):
    return [l for l in open(p) if l.startswith("{")][-1]


open(P + "r02_bench.json", "w").write(last(G + "bench.log"))
names = {1: "r02_bench_default20.json", 2: "r02_bench_4096x4096.json", 3: "r02_bench_f64_4096x4096.json",
         4: "r02_bench_f64_512x512x512.json", 5: "r02_bench_2048x2048x256.json", 6: "r02_bench_4096x4096x512_F.json"}
for i, n in names.items():
    open(P + n, "w").write(last(G + f"bench_{i}.log"))
log = open(sys.argv[1]).read().splitlines()
start = [i for i, l in enumerate(log) if l.startswith("== ") and "grid=" in l][0]
end = [i for i, l in enumerate(log) if l.startswith("[gpurun] status")][0]
open(P + "r02_sq_counters_summary.txt", "w").write("\n".join(l for l in log[start:end] if not l.startswith("smoke")) + "\n")
with open(P + "r02_trace_summary.txt", "w") as fh:
    subprocess.run([sys.executable, "tools/trace_summary.py", G + "prof/run_kernel_trace.csv"], stdout=fh, check=True)
with open(P + "r02_cycle_breakdown.txt", "w") as fh:
    subprocess.run([sys.executable, "tools/cycle_breakdown.py", G + "prof/run_kernel_trace.csv", "8"], stdout=fh, check=True)
for f in ["r02_bench.json"] + list(names.values()):
    d = json.loads(open(P + f).read())
    r, c = d["roofline"], d["cpu_baseline"]
    print(f, round(d["value"], 1), round(d["ms_per_step"], 3), r["kernel"][:30], round(r["achieved"]), round(r["frac"], 3),
          r.get("traffic"), round(c["value"], 3))
d = json.loads(open(P + "r02_bench.json").read())
for k, v in d["level0_kernels"].items():
    print(k, round(v["avg_us"], 1), round(v["achieved_GBps"]))
