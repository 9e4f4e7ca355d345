#!/bin/bash
# Round 3 GPU call: r03_check.sh (selected tests, bench lines), then library variants (tools/run_variants.sh)
# with their parity tests (VAR_TESTS, run against every var/<name>/libmgpoisson.so); VAR_ARGS: one
# bench.py flag set per line for the variant comparison.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r03_check.sh || exit $?
for lib in $(ls var/*/libmgpoisson.so 2>/dev/null); do
  name=$(basename $(dirname $lib))
  if [ -n "${VAR_TESTS:-}" ]; then
    echo "== var tests $name $(date +%T)"
    MGP_LIBRARY=$PWD/$lib timeout -k 10 600 python3 -u -m pytest $VAR_TESTS -x -q --timeout 300 --timeout-method thread ${VAR_K:+-k "$VAR_K"} > gpurun_out/var_tests_$name.log 2>&1
    rc=$?; tail -n 2 gpurun_out/var_tests_$name.log; [ $rc -eq 0 ] || { echo "var $name tests rc=$rc"; exit $rc; }
  fi
done
while read -r args; do
  [ -z "$args" ] && continue
  echo "== variants: $args"
  STEPS=50 BENCH_ARGS="$args" bash tools/run_variants.sh || exit $?
done <<LIST
${VAR_ARGS:-}
LIST
echo "combo done"
