#!/bin/bash
# SQ / TCC counter passes (one rocprofv3 --pmc run per group) of one bench workload: SQDIR (default gpurun_out/sq_w),
# BENCH_ARGS the workload's bench.py arguments.  tools/pmc_summary.py SQDIR '<kernel regex>' summarises them.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=${SQDIR:-gpurun_out/sq_w}
rm -rf $D && mkdir -p $D
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $D/p$i -o run -- python3 bench.py ${BENCH_ARGS:-} --steps 3 --warmup 1 --cpu-cycles 0 --no-timing --no-north-star --copy-probe-mb 0 > $D/p$i.log 2>&1
  rc=$?; echo "sq pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $D/p$i.log; exit $rc; }
done <<LIST
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
LIST
