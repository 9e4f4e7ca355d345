#!/bin/bash
# Round 4 probe: SQ counters of the cl != 0 fused PRE (default library) against the same launch running the
# cl = 0 code (var/asclz, timing only) on the configs[3] rank slab.  One counter pass per library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/clpmc
export TMPDIR=/tmp
for v in base asclz; do
  lib=lua-multigrid-poisson_amd/mgpoisson/libmgpoisson.so
  [ $v != base ] && lib="var/$v/libmgpoisson.so"
  MGP_LIBRARY=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES --kernel-trace --output-format csv -d gpurun_out/clpmc/$v -o run -- python3 bench.py --box 2048,2048,256 --steps 3 --warmup 1 --cpu-cycles 0 --no-timing --no-north-star > gpurun_out/clpmc/$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/clpmc/$v.log; exit $rc; }
done
