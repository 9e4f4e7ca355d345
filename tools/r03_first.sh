#!/bin/bash
# Round 3, first GPU call: luajit probe, the GPU test suite, the driver's bench line, warm-up diagnostic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n ${TAILN:-3} "gpurun_out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || { echo "stopping after $name (rc=$rc)"; exit $rc; }
}
{ echo "which:"; which luajit luajit-2.1 lua lua5.1 lua5.3 lua5.4 2>&1; ls /usr/bin | grep -i lua; ls /usr/lib/x86_64-linux-gnu 2>/dev/null | grep -i lua; echo "nproc $(nproc)"; } > gpurun_out/luajit_probe.log 2>&1
cat gpurun_out/luajit_probe.log
step pytest_gpu 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step bench_driver 300 python3 bench.py --steps 20 --warmup 5
step diag_warm 300 python3 tools/diag_warm.py 512 40
echo "all done"
