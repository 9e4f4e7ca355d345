#!/bin/bash
# On the GPU box: kernel-trace the bench under the in-tree library and each var/<name> library;
# print the per-kernel averages (KPAT filters the kernel names).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tv
for lib in lua-multigrid-poisson_amd/mgpoisson/libmgpoisson.so $(ls var/*/libmgpoisson.so 2>/dev/null); do
  name=$(basename $(dirname $lib)); [ "$name" = mgpoisson ] && name=base
  MGP_LIBRARY=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tv/$name -o run --output-format csv -- \
      python3 bench.py --steps 10 --warmup 2 --cpu-cycles 0 --no-timing ${BENCH_ARGS:-} > gpurun_out/tv/$name.log 2>&1 || { echo "$name failed"; tail -3 gpurun_out/tv/$name.log; exit 1; }
  echo "== $name"
  python3 tools/trace_summary.py gpurun_out/tv/$name/run_kernel_trace.csv 40 | grep -E "${KPAT:-.}" || true
done
