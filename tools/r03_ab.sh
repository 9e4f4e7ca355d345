#!/bin/bash
# Round 3 GPU call: env A/B runs (tools/ab.sh, one VARIANTS/ARGS pair per line of AB: "ARGS::V1|V2|..."),
# then library variants (tools/run_variants.sh, VAR_ARGS lines) with their parity tests (VAR_TESTS / VAR_K).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
while read -r line; do
  [ -z "$line" ] && continue
  args=${line%%::*}; vars=${line#*::}
  echo "== ab: [$args] $vars"
  VARIANTS="$vars" R=${R:-3} S=${S:-60} ARGS="$args" timeout -k 10 600 bash tools/ab.sh || exit $?
done <<LIST
${AB:-}
LIST
VAR_TESTS=${VAR_TESTS:-} SKIP_ALL=1 bash tools/r03_combo.sh
