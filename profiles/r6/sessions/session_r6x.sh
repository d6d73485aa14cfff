#!/bin/bash
# r6x: ShadowFinal's completion code in its own k_trace instance (the deep levels' one-lane kernel back
# to 74 VGPRs, no SGPR spills): the GPU suite, then C5 (10^6 random triangles, 1 spp, one light) with
# ShadowFinal (tree) vs level 0 only (sfl0) vs off (nosf), and the driver line, same box, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh tests || exit 1
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1
grep -E "FAILED" gpurun_out/gpu_tests.log | head -5
RUNS=2 ARGS="--config C5 --steps 10 --warmup 2" bash tools/ab_multi.sh r6x base ablib/sfl0/libpgrt.so ablib/nosf/libpgrt.so || exit 1
RUNS=3 bash tools/ab_multi.sh r6xk20 base ablib/nosf/libpgrt.so || exit 1
