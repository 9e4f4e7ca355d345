#!/bin/bash
# Quick GPU check of the fused path: parity tests (-k FILTER) + one fused bench (+ optional trace).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n ${TAILN:-4} "gpurun_out/$name.log"
  case $rc in 0|1|5) return 0;; *) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
}
step tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${FILTER:-fused}"
step bench_fused 300 env MGP_FUSED=1 ${BENCH_ENV:-} python bench.py --steps 20 --warmup 3 --cpu-cycles 0
if [ -n "${TRACE:-}" ]; then
  step trace 300 env MGP_FUSED=1 ${BENCH_ENV:-} rocprofv3 --kernel-trace --stats -d gpurun_out/trace -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --cpu-cycles 0 --no-timing
fi
echo "all done"
