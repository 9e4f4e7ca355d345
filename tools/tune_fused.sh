#!/bin/bash
# Sweep the fused RB-GS kernel's tuning knobs on the GPU box (bench.py, no CPU baseline).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for ty in ${TYS:-8 16}; do for nh in ${NHS:-2 4}; do for kc in ${KCS:-16 32 64}; do
  out=$(MGP_TY=$ty MGP_NH=$nh MGP_KC=$kc timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-cycles 0 2>/dev/null | grep '^{')
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop rc=$rc"; exit $rc; fi
  echo "TY=$ty NH=$nh KC=$kc $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print("cyc/s %.1f ms %.3f smoother GB/s %.0f launch_us %.1f" % (d["value"], d["ms_per_step"], d.get("finest_smoother_GBps",0), d.get("finest_smoother_launch_us",0)))')"
done; done; done
