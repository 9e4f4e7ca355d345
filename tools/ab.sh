#!/bin/bash
# Interleaved A/B of bench lines.  $AB = lines "label|ENV=.. ENV2=..|bench args"; $REPS rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for r in $(seq 1 ${REPS:-2}); do
  while IFS='|' read -r label envs args; do
    [ -z "$label" ] && continue
    out=gpurun_out/ab/${label}_$r.json
    env $envs timeout -k 10 ${LIMIT:-300} python3 bench.py $args --cpu-cycles 0 --no-north-star --copy-probe-mb 0 > $out 2> gpurun_out/ab/${label}_$r.err
    rc=$?
    python3 - "$out" "$label" <<'PY'
import json, sys
try:
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    k = d.get("level0_kernels", {})
    print(f"{sys.argv[2]:24s} {d['ms_per_step']:.4f} ms  {d['value']:.1f}/s  " + "  ".join(f"{n} {v['avg_us']:.1f}us" for n, v in k.items()), flush=True)
except Exception as e:
    print(sys.argv[2], "FAILED", e, flush=True)
PY
    [ $rc -eq 0 ] || exit $rc
  done <<< "$AB"
done
