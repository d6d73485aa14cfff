#!/bin/bash
# r5zv: the packet step branch-free (scalar selects for next node / push / pop; the push condition
# is "some lane hits each child", as in the branchy step) vs head (r5zu) -- full GPU suite, then the
# driver line, 400 frames and C5 (3 runs each)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash tools/gpu_check.sh tests || exit 1
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1
grep -q " failed" gpurun_out/gpu_tests.log && exit 1
AB_EXTRA="--config C5 --steps 20 --warmup 3" bash tools/ab_head.sh r5zv "frame_parity or packet" || exit 1
