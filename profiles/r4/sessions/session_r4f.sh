#!/bin/bash
# r4f: GPU tests + smoke on the fixed-stamps build, the C2 profile passes (frame traffic),
# timeline with wave percentiles, the driver's bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh tests smoke || exit 1
bash tools/profile.sh r4f C2 || exit 1
timeout -k 10 300 python3 tools/frame_timeline.py --out gpurun_out/timeline_r4f.json > gpurun_out/timeline_r4f.txt 2>&1 || { tail -5 gpurun_out/timeline_r4f.txt; exit 1; }
bash tools/gpu_check.sh bench_driver
