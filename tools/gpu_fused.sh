#!/bin/bash
# GPU-box A/B of the temporally blocked phases (k_zs): parity tests, bench with/without, kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n ${TAILN:-6} "gpurun_out/$name.log"
  case $rc in 0|1|5) return 0;; *) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
}
step fused_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "fused or full_size or smoke"
step bench_unfused 300 env MGP_FUSED=0 python bench.py --steps 20 --warmup 3 --cpu-cycles 0
step bench_fused 300 env MGP_FUSED=1 python bench.py --steps 20 --warmup 3 --cpu-cycles 0
step prof_fused 300 env MGP_FUSED=1 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fused -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --cpu-cycles 0 --no-timing
echo "all done"
