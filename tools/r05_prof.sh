#!/bin/bash
# Round 5: rocprofv3 kernel trace + stats of one bench command ($ARGS), summary under gpurun_out/$NAME.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/$NAME
timeout -k 10 ${LIMIT:-300} rocprofv3 --kernel-trace --stats -d gpurun_out/$NAME -o run --output-format csv -- python3 bench.py $ARGS --cpu-cycles 0 --no-north-star > gpurun_out/$NAME.log 2>&1
rc=$?; tail -c 400 gpurun_out/$NAME.log; exit $rc
