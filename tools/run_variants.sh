#!/bin/bash
# On the GPU box: bench each var/<name>/libmgpoisson.so (plus the in-tree library as "base") and
# print cycles/s and the level-0 kernel averages.  BENCH_ARGS adds bench.py flags.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/var
for lib in lua-multigrid-poisson_amd/mgpoisson/libmgpoisson.so $(ls var/*/libmgpoisson.so 2>/dev/null); do
  name=$(basename $(dirname $lib)); [ "$name" = mgpoisson ] && name=base
  MGP_LIBRARY=$PWD/$lib timeout -k 10 120 python3 bench.py --steps ${STEPS:-30} --warmup 3 --cpu-cycles 0 ${BENCH_ARGS:-} > gpurun_out/var/$name.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -3 gpurun_out/var/$name.log; exit $rc; fi
  python3 - "$name" gpurun_out/var/$name.log <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[2]) if l.startswith("{")][-1]
k = d.get("level0_kernels", {})
print(f"{sys.argv[1]:14s} {d['value']:8.1f}/s {d['ms_per_step']:.3f} ms  " +
      "  ".join(f"{n} {v['avg_us']:.1f}us {v['achieved_GBps']:.0f}GB/s" for n, v in k.items()))
PY
done
