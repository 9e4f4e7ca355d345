#!/bin/bash
# GPU box: the round's bench lines for BASELINE configs 1-5 (one bench.py run each, own time limit).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SKIP_TESTS=1 BENCHES="--steps 20 --warmup 3
--dim 2 --n 4096 --steps 20 --warmup 3
--dim 2 --n 4096 --real double --steps 20 --warmup 3
--real double --steps 20 --warmup 3
--box 2048,2048,256 --steps 10 --warmup 2
--box 4096,4096,512 --cycle F --steps 5 --warmup 1" bash tools/gpu_check.sh
