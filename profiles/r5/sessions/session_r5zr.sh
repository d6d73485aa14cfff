#!/bin/bash
# r5zr: the packet traversal's node step branch-free (scalar selects for the next node / push / pop,
# the stack top read before the node loads; fewer scalar instructions and one branch per step) vs
# head -- full GPU suite, then the driver line, 400 frames and C5 (3 runs each, same box)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash tools/gpu_check.sh tests || exit 1
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1
AB_EXTRA="--config C5 --steps 20 --warmup 3" bash tools/ab_head.sh r5zr "frame_parity or packet" || exit 1
