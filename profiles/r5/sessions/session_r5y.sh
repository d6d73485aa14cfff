#!/bin/bash
# r5y: the synchronous frame's schedule knobs at the r5 head (two-part shades): subtree start level,
# packet levels, one-frame packet budget, 8-lane threshold -- host ms of one synchronous C2 frame
# (frame_timeline, timeline off; 2 runs each, same box)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for rep in 1 2; do
  for c in "" "--cfg subtree_level=2" "--cfg subtree_level=4" "--cfg packet_levels=1" "--cfg packet_levels=2" "--cfg packet_budget=32" "--cfg packet_budget=128" "--cfg group_max=800000" "--cfg group_max=100000" ""; do
    timeout -k 10 200 python3 tools/frame_timeline.py --reps 25 $c > gpurun_out/tl_r5y.txt 2>&1 || { tail -5 gpurun_out/tl_r5y.txt; exit 1; }
    echo "[$c] $(head -1 gpurun_out/tl_r5y.txt | grep -o '"host_ms_median_timeline_off": [0-9.]*') $(head -1 gpurun_out/tl_r5y.txt | grep -o '"device_span_ms_median": [0-9.]*')"
  done
done
