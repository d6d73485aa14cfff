#!/bin/bash
# r6fin3 (part a): after ShadowFinal got its own k_trace instance -- the C2 and C5 roofline profiles again (their closest-hit
# launches changed: the shadow trace completes opaque pixels / nodes), the device timelines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in C2 C5; do
  bash tools/profile.sh r6fin3 $c || exit 1
done
timeout -k 10 300 python3 tools/frame_timeline.py --out gpurun_out/timeline_r6fin3.json > gpurun_out/timeline_r6fin3.txt 2>&1 || { tail -5 gpurun_out/timeline_r6fin3.txt; exit 1; }
