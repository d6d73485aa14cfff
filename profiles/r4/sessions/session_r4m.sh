#!/bin/bash
# r4m: deep tiles first + high-priority slot-0 stream + subtree from level 3 for one-frame batches
# (defaults) -- parity, then the synchronous frame and the driver's region against the variants
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4m.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r4m.log
[ $rc -eq 0 ] || exit $rc
tl() {  # name [args]
  local n=$1; shift
  timeout -k 10 300 python3 tools/frame_timeline.py --reps 15 --out gpurun_out/timeline_r4m_$n.json "$@" > gpurun_out/timeline_r4m_$n.txt 2>&1 || { tail -5 gpurun_out/timeline_r4m_$n.txt; exit 1; }
  echo "$n $(head -1 gpurun_out/timeline_r4m_$n.txt | grep -o '"host_ms_median_timeline_off.*')  r20 $(grep '^r20' gpurun_out/timeline_r4m_$n.txt | grep -o '"host_ms_per_frame_off_median": [0-9.]*')"
}
for r in 1 2; do
  tl def$r
  tl nosub$r --cfg subtree_level=-1
  tl rr$r --cfg tile_order=-1
  tl rrnosub$r --cfg tile_order=-1 --cfg subtree_level=-1
  tl sub2_$r --cfg subtree_level=2
  tl sub4_$r --cfg subtree_level=4
done
