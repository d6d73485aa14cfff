#!/bin/bash
# r6s: level-0 opaque pixels of 1-spp batches with one light completed by the shadow trace
# (ShadowFinal, in tree) against the finish doing them (ablib/nosf = PGRT_SHADOW_FINAL=0): the GPU
# suite first, then the driver line, the 600-frame default line and one synchronous-frame timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh tests smoke || exit 1
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1
grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head -5
RUNS=3 bash tools/ab_multi.sh r6s base ablib/nosf/libpgrt.so || exit 1
RUNS=2 ARGS="--steps 600" bash tools/ab_multi.sh r6s600 base ablib/nosf/libpgrt.so || exit 1
timeout -k 10 300 python3 tools/frame_timeline.py --out gpurun_out/timeline_r6s.json > gpurun_out/timeline_r6s.txt 2>&1 || { tail -5 gpurun_out/timeline_r6s.txt; exit 1; }
