#!/bin/bash
# On the GPU box: bench the in-tree library under several environment settings (one per line of
# ENVS, "name VAR=val VAR=val ..."), print cycles/s and the level-0 kernel averages.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/env
while read -r name rest; do
  [ -z "$name" ] && continue
  env $rest timeout -k 10 120 python3 bench.py --steps ${STEPS:-30} --warmup 3 --cpu-cycles 0 ${BENCH_ARGS:-} > gpurun_out/env/$name.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -3 gpurun_out/env/$name.log; exit $rc; fi
  python3 - "$name" gpurun_out/env/$name.log <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[2]) if l.startswith("{")][-1]
k = d.get("level0_kernels", {})
print(f"{sys.argv[1]:14s} {d['value']:8.1f}/s {d['ms_per_step']:.3f} ms  " +
      "  ".join(f"{n} {v['avg_us']:.1f}us" for n, v in k.items()))
PY
done <<LIST
${ENVS}
LIST
