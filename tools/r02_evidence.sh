#!/bin/bash
# Round-2 evidence in one GPU call: GPU tests, PMC traffic + bench + rocprofv3 stats, SQ counter passes.
# Each step is time-limited by its own script; the chain stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_check.sh && bash tools/gpu_round.sh && bash tools/r02_sq.sh
