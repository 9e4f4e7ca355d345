#!/bin/bash
# GPU-box check: parity tests, smoke, a short bench, and a rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; a fault/abort/timeout stops the script immediately.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"; date +%T
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 15 "gpurun_out/$name.log"
  case $rc in 0|1|5) return 0;; *) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
}
STEPS=${STEPS:-tests smoke bench prof}
for s in $STEPS; do
  case $s in
    tests) step pytest_gpu 900 python -m pytest tests -m gpu -q -x ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 400 python bench.py --steps 50 --warmup 3 ;;
    prof)  step prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --cpu-cycles 0 ;;
  esac
done
echo "all done"
