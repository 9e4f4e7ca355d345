#!/bin/bash
# PMC passes over the bench workload with the temporally blocked phases on (one counter group per run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmczs
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  echo "== pass $i: $grp"
  MGP_FUSED=${MGP_FUSED:-1} timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmczs/p$i -o run -- python bench.py --steps 2 --warmup 1 --cpu-cycles 0 --no-timing > gpurun_out/pmczs/p$i.log 2>&1
  rc=$?; echo "rc=$rc"
  case $rc in 0) ;; *) tail -5 gpurun_out/pmczs/p$i.log; exit $rc;; esac
done <<LIST
FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_MISC
LIST
echo done
