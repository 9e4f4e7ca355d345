#!/bin/bash
# Interleaved A/B timing of library variants (env settings) on the GPU box: R rounds of each variant,
# bench --steps S (graph-replayed cycles, no per-launch events), median ms per cycle per variant.
#   VARIANTS="MGP_BLK=0|MGP_BLK=1" R=3 S=100 ARGS="--real double" bash tools/ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS='|' read -r -a V <<< "${VARIANTS:-MGP_BLK=1}"
: > gpurun_out/ab.txt
for r in $(seq 1 ${R:-3}); do
  for v in "${V[@]}"; do
    env $v timeout -k 10 120 python3 bench.py --steps ${S:-100} --warmup 5 --cpu-cycles 0 --no-timing ${ARGS:-} > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    ms=$(python3 -c 'import json; print(json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])["ms_per_step"])')
    echo "$v|$ms" >> gpurun_out/ab.txt
  done
done
python3 - <<'PY'
import collections, statistics
d = collections.defaultdict(list)
for line in open("gpurun_out/ab.txt"):
    v, ms = line.rstrip("\n").rsplit("|", 1)
    d[v].append(float(ms))
for v, xs in d.items():
    print(f"{v:40s} median {statistics.median(xs):.4f} ms  min {min(xs):.4f}  n {len(xs)}")
PY
