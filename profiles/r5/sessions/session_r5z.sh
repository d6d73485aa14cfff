#!/bin/bash
# r5z: synchronous frame -- level 0 only on packets (bounce levels 8 lanes per ray) and / or the
# subtree from level 2; 4 interleaved runs each, same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for rep in 1 2 3 4; do
  for c in "" "--cfg packet_levels=1" "--cfg subtree_level=2" "--cfg packet_levels=1 --cfg subtree_level=2" "--cfg packet_levels=1 --cfg subtree_level=2 --cfg group_max=800000"; do
    timeout -k 10 200 python3 tools/frame_timeline.py --reps 25 $c > gpurun_out/tl_r5z.txt 2>&1 || { tail -5 gpurun_out/tl_r5z.txt; exit 1; }
    echo "[$c] $(head -1 gpurun_out/tl_r5z.txt | grep -o '"host_ms_median_timeline_off": [0-9.]*') $(head -1 gpurun_out/tl_r5z.txt | grep -o '"device_span_ms_median": [0-9.]*')"
  done
done
