#!/bin/bash
# Bench lines on the GPU box (BENCHES, one per line; optional FIRST tests and the whole GPU suite before them).
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n ${TAILN:-4} "gpurun_out/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
if [ -n "${FIRST:-}" ]; then
  step tests_first 600 python3 -u -m pytest $FIRST -x -v --timeout 300 --timeout-method thread ${FIRST_K:+-k "$FIRST_K"}
fi
if [ -z "${SKIP_ALL:-}" ]; then
  step tests_all 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${DESELECT:+--deselect $DESELECT}
fi
i=0
while read -r args; do
  [ -z "$args" ] && continue
  i=$((i+1))
  step bench_$i 300 env $args
done <<LIST
${BENCHES:-}
LIST
echo "all done"
