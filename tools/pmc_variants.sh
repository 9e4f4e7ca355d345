#!/bin/bash
# On the GPU box: FETCH_SIZE / WRITE_SIZE passes (one counter group per rocprofv3 run) of the bench
# under the in-tree library and each var/<name> library; per-kernel traffic summary per library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pv
for lib in lua-multigrid-poisson_amd/mgpoisson/libmgpoisson.so $(ls var/*/libmgpoisson.so 2>/dev/null); do
  name=$(basename $(dirname $lib)); [ "$name" = mgpoisson ] && name=base
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    MGP_LIBRARY=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pv/$name/p$i -o run -- \
        python3 bench.py --steps 3 --warmup 1 --cpu-cycles 0 --no-timing > gpurun_out/pv/$name.p$i.log 2>&1 || { echo "$name pass $i failed"; exit 1; }
  done
  echo "== $name"
  python3 tools/pmc_traffic.py gpurun_out/pv/$name gpurun_out/pv/$name.json | grep k_zs || true
done
