#!/bin/bash
# End-of-round evidence on the GPU box (one call): PMC traffic passes + the default bench line carrying
# that traffic + the rocprofv3 kernel-trace/stats of the same command (tools/gpu_round.sh), the bench
# lines of BASELINE configs 1-5 (tools/r02_lines.sh), then the SQ counter passes (tools/r02_sq.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
STEPS=50 bash tools/gpu_round.sh && bash tools/r02_lines.sh && bash tools/r02_sq.sh
