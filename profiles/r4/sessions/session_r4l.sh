#!/bin/bash
# r4l: deep tiles first (pgrt_config.tile_order) -- parity, then the synchronous frame's device
# timeline and the driver's 20-frame region, tile_order 0 (default) vs -1 (round-robin), same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4l.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r4l.log
[ $rc -eq 0 ] || exit $rc
tl() {  # name [args]
  local n=$1; shift
  timeout -k 10 300 python3 tools/frame_timeline.py --reps 15 --out gpurun_out/timeline_r4l_$n.json "$@" > gpurun_out/timeline_r4l_$n.txt 2>&1 || { tail -5 gpurun_out/timeline_r4l_$n.txt; exit 1; }
  echo "$n $(head -1 gpurun_out/timeline_r4l_$n.txt | grep -o '"host_ms_median_timeline_off.*')  r20 $(grep '^r20' gpurun_out/timeline_r4l_$n.txt | grep -o '"host_ms_per_frame_off_median": [0-9.]*')"
}
for r in 1 2 3; do
  tl deep$r
  tl rr$r --cfg tile_order=-1
done
tl deep_sub3 --cfg subtree_level=3
tl deep_sub2 --cfg subtree_level=2
tl co1 --cfg call_order=1
tl co1b --cfg call_order=1
