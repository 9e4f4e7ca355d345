#!/bin/bash
# GPU box: the fused-phase parity tests (k_zs vs the launch-per-piece path and the oracle, loopback
# slabs, the full-size 512^3 test), then the in-tree and var/* library benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    -k "${TESTK:-fused or 512 or loopback or slab}" > gpurun_out/pytest_zs.log 2>&1
rc=$?; tail -n 5 gpurun_out/pytest_zs.log; [ $rc -eq 0 ] || exit $rc
bash tools/run_variants.sh
