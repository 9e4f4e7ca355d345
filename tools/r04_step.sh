#!/bin/bash
# Round 4 GPU-call helper: run each step under its own limit, stop at the first failure.
# usage: tools/r04_step.sh name:seconds:command [name:seconds:command ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; to=${rest%%:*}; cmd=${rest#*:}
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc"; tail -n ${TAILN:-4} "gpurun_out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
done
echo "all done"
