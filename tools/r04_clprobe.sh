#!/bin/bash
# Round 4 probe: the cl != 0 fused PRE's step cost.  Kernel traces of the configs[3] rank slab under the
# default library and two timing variants (var/pfd1: cl = 0 PRE with one plane of prefetch; var/asclz: cl != 0
# PRE running the cl = 0 code, wrong at the faces; build them with tools/build_variants.sh and drop ./var from
# .gpurunignore first).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/clprobe
export TMPDIR=/tmp
for v in base pfd1 asclz; do
  lib=""
  [ $v != base ] && lib="var/$v/libmgpoisson.so"
  MGP_LIBRARY=${lib:-lua-multigrid-poisson_amd/mgpoisson/libmgpoisson.so} timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/clprobe/$v -o run --output-format csv -- python3 bench.py --box 2048,2048,256 --steps 8 --warmup 2 --cpu-cycles 0 --no-north-star > gpurun_out/clprobe/$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/clprobe/$v.log; exit $rc; }
  python3 tools/cycle_breakdown.py gpurun_out/clprobe/$v/run_kernel_trace.csv 2 | grep -E "k_zs|busy"
done
