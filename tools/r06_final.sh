#!/bin/bash
# Round 6 evidence on the GPU box (stops at the first failure; everything lands in gpurun_out/, then
# tools/install_evidence.py r06 copies it into profiles/).
#   PART 1: the whole GPU suite and smoke(); PMC FETCH_SIZE / WRITE_SIZE of the default 512^3 line, its bench line
#           and the rocprofv3 kernel trace + stats of that line alone (tools/gpu_round.sh); SQ counter passes.
#   PART 2: PMC traffic of every other measured workload, each tagged with its workload key (bench.workload_key:
#           box, ranks, options), so that a bench line only ever carries the traffic of its own launches; then the
#           driver's 20/5 line (with the configs[3] 2048^3 box and the fp64 line) and the BASELINE config lines, each
#           with every traffic JSON, and one rocprofv3 kernel trace per further workload (2D, full weighting, fp64).
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
rm -rf gpurun_out/sq && mkdir -p gpurun_out/sq
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/sq/p$i -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-cycles 0 --no-timing --no-north-star --copy-probe-mb 0 > gpurun_out/sq/p$i.log 2>&1
  rc=$?; echo "sq pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/sq/p$i.log; exit $rc; }
done <<LIST
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
LIST
fi
[[ $PART == *2* ]] || exit 0
pmc() {  # name, bench args of the workload
  PMCDIR=gpurun_out/pmc_$1 PMC_STEPS=1 BENCH_ARGS="$2" PMC_GROUPS="FETCH_SIZE
WRITE_SIZE" bash tools/pmc.sh > gpurun_out/pmc_$1.log 2>&1 || { tail -5 gpurun_out/pmc_$1.log; exit 1; }
  python3 tools/pmc_traffic.py gpurun_out/pmc_$1 gpurun_out/pmc_traffic_$1.json "$2" > gpurun_out/pmc_traffic_$1.txt || exit 1
  echo "pmc $1: $(head -n 2 gpurun_out/pmc_traffic_$1.txt | tail -n 1)"
}
pmc slab3 "--box 2048,2048,256"
pmc slab4 "--box 4096,4096,512 --cycle F"
pmc box2048 "--box 2048,2048,2048"
pmc fw "--restriction full_weighting"
pmc 2d "--dim 2 --n 4096"
pmc 2d64 "--dim 2 --n 4096 --real double"
pmc f64 "--real double"
TR="--traffic gpurun_out/pmc_traffic.json,gpurun_out/pmc_traffic_slab3.json,gpurun_out/pmc_traffic_slab4.json,gpurun_out/pmc_traffic_box2048.json,gpurun_out/pmc_traffic_fw.json,gpurun_out/pmc_traffic_2d.json,gpurun_out/pmc_traffic_2d64.json,gpurun_out/pmc_traffic_f64.json"
SKIP_ALL=1 TAILN=2 BENCHES="python3 bench.py --steps 20 --warmup 5 $TR
python3 bench.py --dim 2 --n 4096 --steps 50 $TR
python3 bench.py --dim 2 --n 4096 --real double --steps 50 $TR
python3 bench.py --real double --steps 30 --no-north-star $TR
python3 bench.py --config0 --steps 20 $TR
python3 bench.py --restriction full_weighting --steps 30 --no-north-star $TR
python3 bench.py --box 2048,2048,256 --steps 10 --warmup 2 $TR
python3 bench.py --box 4096,4096,512 --cycle F --steps 5 --warmup 1 $TR" bash tools/bench_lines.sh || exit $?
prof() {  # name, bench args: the kernel trace of that workload alone
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof$1 -o run --output-format csv -- python3 bench.py $2 --cpu-cycles 0 --no-north-star --copy-probe-mb 0 > gpurun_out/prof$1.log 2>&1
  rc=$?; tail -n 1 gpurun_out/prof$1.log; [ $rc -eq 0 ] || exit $rc
}
prof 2d "--dim 2 --n 4096 --steps 50"
prof fw "--restriction full_weighting --steps 20"
prof f64 "--real double --steps 20"
echo "r06 part 2 done"
