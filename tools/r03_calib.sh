#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration by lane width (tools/fetch_calib.py), then the PMC traffic passes
# of the bench workload (tools/pmc.sh + tools/pmc_traffic.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/calib
export TMPDIR=/tmp MGP_COPY_CALIB=1
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/calib/p$i -o run -- python3 tools/fetch_calib.py run > gpurun_out/calib/p$i.log 2>&1
  rc=$?; echo "calib $c rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/calib/p$i.log; exit $rc; }
done
unset MGP_COPY_CALIB
python3 tools/fetch_calib.py report gpurun_out/calib gpurun_out/fetch_calib.json || exit 1
[ -n "${NO_PMC:-}" ] && exit 0
PMC_GROUPS="FETCH_SIZE
WRITE_SIZE" bash tools/pmc.sh || exit $?
python3 tools/pmc_traffic.py gpurun_out/pmc gpurun_out/pmc_traffic.json > gpurun_out/pmc_traffic.txt || exit 1
cat gpurun_out/pmc_traffic.txt
