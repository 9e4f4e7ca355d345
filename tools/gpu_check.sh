#!/bin/bash
# GPU box: the GPU test suite, then the default bench line and (optionally) extra bench lines.
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 ${TEST_LIMIT:-600} python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -n 15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
i=0
while read -r args; do
  [ -z "$args" ] && continue
  i=$((i+1))
  echo "== bench $i: $args"
  timeout -k 10 300 python3 bench.py $args > gpurun_out/bench_$i.log 2>&1
  rc=$?; tail -n 1 gpurun_out/bench_$i.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
done <<LIST
${BENCHES:---steps 20 --warmup 3}
LIST
