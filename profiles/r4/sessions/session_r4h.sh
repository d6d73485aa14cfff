#!/bin/bash
# r4h: the synchronous frame's chain under speed-only configs: subtree levels, packet levels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tl() {  # name [args]
  local n=$1; shift
  timeout -k 10 300 python3 tools/frame_timeline.py --reps 15 --out gpurun_out/timeline_r4h_$n.json "$@" > gpurun_out/timeline_r4h_$n.txt 2>&1 || { tail -5 gpurun_out/timeline_r4h_$n.txt; exit 1; }
  echo "$n $(head -1 gpurun_out/timeline_r4h_$n.txt | grep -o '"host_ms_median_timeline_off.*')  r20 $(grep '^r20' gpurun_out/timeline_r4h_$n.txt | grep -o '"host_ms_per_frame_off_median": [0-9.]*')"
}
tl base
tl sub3 --cfg subtree_level=3
tl sub4 --cfg subtree_level=4
tl sub5 --cfg subtree_level=5
tl pkt1 --cfg packet_levels=1
tl pkt2 --cfg packet_levels=2
tl base2
