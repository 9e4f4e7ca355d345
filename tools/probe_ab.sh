#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/pab
for r in 1 2 3; do
  for mode in late first; do
    if [ $mode = late ]; then E="MGP_BENCH_PROBE_LATE=1"; else E="MGP_BENCH_PROBE_LATE=0"; fi
    env $E timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-cycles 0 --no-north-star > gpurun_out/pab/${mode}_$r.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/pab/${mode}_$r.json').read().strip().splitlines()[-1]); print('$mode', d['ms_per_step'], d['value'])"
  done
done
