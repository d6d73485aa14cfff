#!/bin/bash
# r5zf: shade_eval defined as its two parts (no separate shade_hit copy; subtree / path kernels
# now run the same code as k_shade) -- full GPU suite, smoke, driver line / 400 frames / path vs HEAD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash tools/gpu_check.sh tests smoke || exit 1
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1; tail -1 gpurun_out/smoke.log
bash tools/ab_matrix.sh r5zf "base ablib/head/libpgrt.so" "--steps 20 --warmup 5" "--steps 400" "--mode path --steps 20 --warmup 3" || exit 1
