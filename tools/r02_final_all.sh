#!/bin/bash
# GPU tests, then the end-of-round evidence (tools/r02_final.sh); stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/r02_final.sh
