#!/bin/bash
# Round 5: the GPU suite (or the files / -k expression in $TESTS), each step under its own limit; output in gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${LIMIT:-900} python3 -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout ${PER:-400} --timeout-method thread ${KEXPR:+-k "$KEXPR"} > gpurun_out/${LOG:-pytest_gpu}.log 2>&1
rc=$?; tail -n 5 gpurun_out/${LOG:-pytest_gpu}.log; exit $rc
