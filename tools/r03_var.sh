#!/bin/bash
# GPU A/B of library variants (var/<name>/libmgpoisson.so, tools/build_variants.sh): the GPU suite against
# the variant named by TEST_VAR (skipped when empty), then REPS rounds of tools/run_variants.sh.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${TEST_VAR:-}" ]; then
  MGP_LIBRARY=$PWD/var/$TEST_VAR/libmgpoisson.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread ${TEST_K:+-k "$TEST_K"} > gpurun_out/var_tests.log 2>&1
  rc=$?; tail -n 3 gpurun_out/var_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 ${REPS:-2}); do
  echo "== round $r"
  bash tools/run_variants.sh || exit $?
done
