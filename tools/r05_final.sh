#!/bin/bash
# Round 5 evidence on the GPU box, one call (stops at the first failure; everything lands in gpurun_out/, then
# tools/install_evidence.py r05 copies it into profiles/):
#   1. the whole GPU suite and smoke();
#   2. PMC FETCH_SIZE / WRITE_SIZE of the default 512^3 line, the bench line carrying that traffic, and the
#      rocprofv3 kernel trace + stats of the same command (tools/gpu_round.sh);
#   3. PMC traffic of the configs[4] rank slab (4096 x 4096 x 512, F-cycle) and the configs[3] rank slab
#      (2048 x 2048 x 256), one pass per counter group;
#   4. SQ / TCC counter passes of the default workload;
#   5. the driver's 20/5 line and the BASELINE config lines, each with the traffic JSON of its workload;
#   6. rocprofv3 kernel traces of configs[1] (2D 4096^2) and of the full-weighting 512^3 line.
# PART=1 runs 1, 2 and 4, PART=2 runs 3, 5 and 6 (two gpurun calls, each inside its time limit); default both.
set -u
PART=${PART:-12}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [[ $PART == *1* ]]; then
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -n 3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; tail -n 3 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
STEPS=50 bash tools/gpu_round.sh || exit $?
fi
slab() {  # name, cells per rank, bench args
  PMCDIR=gpurun_out/pmc_$1 PMC_STEPS=1 BENCH_ARGS="$3" PMC_GROUPS="FETCH_SIZE
WRITE_SIZE" bash tools/pmc.sh || exit $?
  python3 tools/pmc_traffic.py gpurun_out/pmc_$1 gpurun_out/pmc_traffic_$1.json $2 > gpurun_out/pmc_traffic_$1.txt || exit 1
  head -n 6 gpurun_out/pmc_traffic_$1.txt
}
if [[ $PART == *2* ]]; then
slab slab4 8589934592 "--box 4096,4096,512 --cycle F"
slab slab3 1073741824 "--box 2048,2048,256"
fi
if [[ $PART == *1* ]]; then
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
fi
[[ $PART == *2* ]] || exit 0
TR="--traffic gpurun_out/pmc_traffic.json,gpurun_out/pmc_traffic_slab4.json,gpurun_out/pmc_traffic_slab3.json"
SKIP_ALL=1 TAILN=2 BENCHES="python3 bench.py --steps 20 --warmup 5 $TR
python3 bench.py --dim 2 --n 4096 --steps 50 $TR
python3 bench.py --dim 2 --n 4096 --real double --steps 50 $TR
python3 bench.py --real double --steps 30 $TR
python3 bench.py --config0 --steps 20 $TR
python3 bench.py --restriction full_weighting --steps 30 $TR
python3 bench.py --box 2048,2048,256 --steps 10 --warmup 2 $TR
python3 bench.py --box 4096,4096,512 --cycle F --steps 5 --warmup 1 $TR" bash tools/bench_lines.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2d -o run --output-format csv -- python3 bench.py --dim 2 --n 4096 --steps 50 --cpu-cycles 0 > gpurun_out/prof2d.log 2>&1
rc=$?; tail -n 2 gpurun_out/prof2d.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/proffw -o run --output-format csv -- python3 bench.py --restriction full_weighting --steps 20 --cpu-cycles 0 --no-north-star > gpurun_out/proffw.log 2>&1
rc=$?; tail -n 2 gpurun_out/proffw.log; exit $rc
