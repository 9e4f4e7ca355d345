#!/bin/bash
# Round evidence on the GPU box: PMC FETCH_SIZE / WRITE_SIZE passes -> per-kernel HBM traffic JSON,
# then the bench (reading that JSON for roofline.traffic) and a rocprofv3 kernel-trace summary of
# the same command, the default 512^3 line only (--no-north-star: the kernel stats hold one workload).  Everything lands in gpurun_out/ (copy what is judged into profiles/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PMC_GROUPS="FETCH_SIZE
WRITE_SIZE" bash tools/pmc.sh || exit $?
python3 tools/pmc_traffic.py gpurun_out/pmc gpurun_out/pmc_traffic.json "" > gpurun_out/pmc_traffic.txt || exit 1
cat gpurun_out/pmc_traffic.txt
echo "== bench"
timeout -k 10 300 python bench.py --steps ${STEPS:-50} --warmup 3 --no-north-star --traffic gpurun_out/pmc_traffic.json > gpurun_out/bench.log 2>&1
rc=$?; tail -n 3 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
echo "== prof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps ${STEPS:-50} --warmup 3 --no-north-star --cpu-cycles 0 --traffic gpurun_out/pmc_traffic.json > gpurun_out/prof.log 2>&1
rc=$?; tail -n 2 gpurun_out/prof.log; exit $rc
