#!/bin/bash
# PMC passes for the bench workload (one counter group per rocprofv3 run; kernel-trace only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PMCDIR=${PMCDIR:-gpurun_out/pmc}
mkdir -p $PMCDIR
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $PMCDIR/p$i -o run -- python bench.py --steps ${PMC_STEPS:-3} --warmup 1 --cpu-cycles 0 --no-timing --no-north-star --copy-probe-mb 0 ${BENCH_ARGS:-} > $PMCDIR/p$i.log 2>&1
  rc=$?; echo "rc=$rc"
  case $rc in 0) ;; *) tail -5 $PMCDIR/p$i.log; exit $rc;; esac
done <<LIST
${PMC_GROUPS:-FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE}
LIST
echo done
