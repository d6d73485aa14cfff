#!/bin/bash
# r5zq: a step budget on the bounce levels' one-lane closest-hit launches (k_trace: a ray still
# traversing after B steps stops and is finished by k_trace8g<RESUME>, 8 lanes per ray): B = 160
# (base), 96, 256, 0 (no budget, same source) and the head build -- full GPU suite on base, then
# the driver line and 400 frames, 3 runs per cell
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash tools/gpu_check.sh tests || exit 1
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1
bash tools/ab_matrix.sh r5zq "base ablib/b96/libpgrt.so ablib/b256/libpgrt.so ablib/b0/libpgrt.so ablib/head/libpgrt.so" "--steps 20 --warmup 5" "--steps 400" || exit 1
timeout -k 10 300 python3 tools/frame_timeline.py --out gpurun_out/timeline_r5zq.json > gpurun_out/timeline_r5zq.txt 2>&1 || { tail -5 gpurun_out/timeline_r5zq.txt; exit 1; }
grep -E "t1[0-9][0-9] s0 (trace|trace_resume) " gpurun_out/timeline_r5zq.txt | head -12
