#!/bin/bash
# r4o: the synchronous frame's chain under speed-only configs at the new defaults (deep tiles
# first, priority slot 0, subtree from level 3): packet levels, packet budget, group_max
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tl() {  # name [args]
  local n=$1; shift
  timeout -k 10 300 python3 tools/frame_timeline.py --reps 15 --out gpurun_out/timeline_r4o_$n.json "$@" > gpurun_out/timeline_r4o_$n.txt 2>&1 || { tail -5 gpurun_out/timeline_r4o_$n.txt; exit 1; }
  echo "$n $(head -1 gpurun_out/timeline_r4o_$n.txt | grep -o '"host_ms_median_timeline_off.*')  r20 $(grep '^r20' gpurun_out/timeline_r4o_$n.txt | grep -o '"host_ms_per_frame_off_median": [0-9.]*')"
}
for r in 1 2; do
  tl def$r
  tl pkt1_$r --cfg packet_levels=1
  tl pkt2_$r --cfg packet_levels=2
  tl b32_$r --cfg packet_budget=32
  tl b128_$r --cfg packet_budget=128
  tl gm100k_$r --cfg group_max=100000
  tl gm1m_$r --cfg group_max=1000000
  tl pkt1gm1m_$r --cfg packet_levels=1 --cfg group_max=1000000
done
