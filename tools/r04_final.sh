#!/bin/bash
# Round 4 evidence on the GPU box: PMC traffic + the default bench line carrying it + the rocprofv3
# kernel-trace/stats of the same command (tools/gpu_round.sh), SQ and TCC counter passes of the same workload,
# the driver's 20/5 line, the BASELINE config lines, the 2D kernel trace.  Stops at the first failure;
# everything lands in gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=50 bash tools/gpu_round.sh || exit $?
rm -rf gpurun_out/sq && mkdir -p gpurun_out/sq
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/sq/p$i -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-cycles 0 --no-timing --no-north-star > gpurun_out/sq/p$i.log 2>&1
  rc=$?; echo "sq pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/sq/p$i.log; exit $rc; }
done <<LIST
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
LIST
SKIP_ALL=1 TAILN=2 BENCHES="python3 bench.py --steps 20 --warmup 5
python3 bench.py --dim 2 --n 4096 --steps 50
python3 bench.py --dim 2 --n 4096 --real double --steps 50
python3 bench.py --real double --steps 30
python3 bench.py --config0 --steps 20
python3 bench.py --restriction full_weighting --steps 30
python3 bench.py --box 2048,2048,256 --steps 10 --warmup 2
python3 bench.py --box 4096,4096,512 --cycle F --steps 5 --warmup 1" bash tools/r03_check.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2d -o run --output-format csv -- python3 bench.py --dim 2 --n 4096 --steps 50 --cpu-cycles 0 > gpurun_out/prof2d.log 2>&1
rc=$?; tail -n 2 gpurun_out/prof2d.log; exit $rc
