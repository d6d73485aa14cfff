#!/bin/bash
# r6m: frames per call on the driver line (20 frames: 8+8+4 default vs one call of 20, 10+10, 16+4) and on
# the 400-frame line (8 vs 16 / 32 per call), same box, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
RUNS=3 bash tools/ab_multi.sh r6m base "f20=--frames-per-call 20" "f10=--frames-per-call 10" "f16=--frames-per-call 16" || exit 1
RUNS=2 ARGS="--steps 400" bash tools/ab_multi.sh r6m400 base "f16=--frames-per-call 16" "f32=--frames-per-call 32" || exit 1
