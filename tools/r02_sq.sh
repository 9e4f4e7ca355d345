#!/bin/bash
# SQ / LDS counter passes over the bench workload (k_zs PRE / POST are the level-0 kernels):
# one counter group per rocprofv3 run, kernel trace only, each pass under its own time limit.
# Output: gpurun_out/sq/p<i>/..., summary in gpurun_out/sq/summary.txt (tools/pmc_summary.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SQ_OUT:-sq}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || echo "counter list rc=$?"
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
      python3 bench.py --steps 2 --warmup 1 --cpu-cycles 0 --no-timing ${BENCH_ARGS:-} > $OUT/p$i.log 2>&1
  rc=$?; echo "rc=$rc"
  case $rc in 0) ;; *) tail -5 $OUT/p$i.log; exit $rc;; esac
done <<LIST
${SQ_GROUPS:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES}
LIST
python3 tools/pmc_summary.py $OUT 'k_zs|k_half|k_tail' $OUT/summary.json > $OUT/summary.txt
cat $OUT/summary.txt
