#!/bin/bash
# Round 4 extra evidence: PMC traffic of the 2D configs[1] line, and the run-to-run spread of the default and
# 2D lines on one box (five / three back-to-back bench runs).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc2d_t gpurun_out/spread
export TMPDIR=/tmp
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc2d_t/p$i -o run -- python3 bench.py --dim 2 --n 4096 --steps 3 --warmup 1 --cpu-cycles 0 --no-timing --no-north-star > gpurun_out/pmc2d_t/p$i.log 2>&1
  rc=$?; echo "pmc2d $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc2d_t/p$i.log; exit $rc; }
done
python3 tools/pmc_traffic.py gpurun_out/pmc2d_t gpurun_out/pmc2d_traffic.json 16777216 > gpurun_out/pmc2d_traffic.txt || exit 1
head -8 gpurun_out/pmc2d_traffic.txt
for k in 1 2 3 4 5; do
  timeout -k 10 120 python3 bench.py --steps 50 --warmup 3 --cpu-cycles 0 --no-north-star > gpurun_out/spread/d$k.log 2>&1 || exit $?
done
for k in 1 2 3; do
  timeout -k 10 120 python3 bench.py --dim 2 --n 4096 --steps 50 --cpu-cycles 0 --no-north-star > gpurun_out/spread/y$k.log 2>&1 || exit $?
done
echo done
