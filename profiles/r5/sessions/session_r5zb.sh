#!/bin/bash
# r5zb: synchronous frame after the level-2 subtree default: subtree from level 1, level 0 only on
# packets, the 8-lane threshold -- host ms (median of 25, timeline off), 4 interleaved runs each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for rep in 1 2 3 4; do
  for c in "" "--cfg subtree_level=1" "--cfg packet_levels=1" "--cfg packet_levels=1 --cfg group_max=800000" "--cfg packet_budget=128" "--cfg tile_order=-1"; do
    timeout -k 10 200 python3 tools/frame_timeline.py --reps 25 $c > gpurun_out/tl_r5zb.txt 2>&1 || { tail -5 gpurun_out/tl_r5zb.txt; exit 1; }
    echo "[$c] $(head -1 gpurun_out/tl_r5zb.txt | grep -o '"host_ms_median_timeline_off": [0-9.]*') $(head -1 gpurun_out/tl_r5zb.txt | grep -o '"device_span_ms_median": [0-9.]*')"
  done
done
timeout -k 10 200 python3 tools/frame_timeline.py --reps 25 --out gpurun_out/tl_r5zb.json > gpurun_out/tl_r5zb.txt 2>&1 && sed -n 1,40p gpurun_out/tl_r5zb.txt | cut -c1-150
