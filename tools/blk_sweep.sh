#!/bin/bash
# k_blk tuning on the GPU box: bench lines over MGP_BLK / MGP_BLK_CELLS, then a rocprofv3 stats run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "MGP_BLK=0" "MGP_BLK_CELLS=32768" "MGP_BLK_CELLS=262144" "MGP_BLK_CELLS=2097152" ${EXTRA:-}; do
  env $v timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --cpu-cycles 0 > gpurun_out/bs.log 2>&1 || { tail -5 gpurun_out/bs.log; exit 1; }
  echo "$v $(python3 -c 'import json,sys; d=json.loads(open("gpurun_out/bs.log").read().strip().splitlines()[-1]); print(round(d["ms_per_step"],4))')"
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_blk -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --cpu-cycles 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_blk.log 2>&1
