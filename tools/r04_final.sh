#!/bin/bash
# Round 4 evidence on the GPU box: PMC traffic + the default bench line carrying it + the rocprofv3
# kernel-trace/stats of the same command (tools/gpu_round.sh), the driver's 20/5 line, the BASELINE config
# lines, the 2D kernel trace.  Stops at the first failure; everything lands in gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=50 bash tools/gpu_round.sh || exit $?
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
