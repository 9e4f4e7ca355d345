#!/bin/bash
# One GPU call of A/B experiments: library variants (tools/run_variants.sh) and environment variants
# (tools/ab.sh) given as AB1 / AB2 ("VARIANTS;ARGS"), each step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "${SKIP_VAR:-}" ]; then
  for r in $(seq 1 ${REPS:-2}); do
    echo "== variants round $r"
    timeout -k 10 600 bash tools/run_variants.sh || exit $?
  done
fi
for spec in "${AB1:-}" "${AB2:-}" "${AB3:-}"; do
  [ -z "$spec" ] && continue
  echo "== ab: $spec"
  VARIANTS="${spec%%;*}" ARGS="${spec#*;}" R=${ABR:-3} S=${ABS:-100} timeout -k 10 600 bash tools/ab.sh || exit $?
done
