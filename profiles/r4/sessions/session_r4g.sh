#!/bin/bash
# r4g: the L2 policy of the streaming data (cache_ops.hpp) on vs off, and early split clipping, on
# the driver's line and the synchronous frame's device timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_pair.sh r4g base ablib/nocache/libpgrt.so 3 || exit 1
bash tools/ab_pair.sh r4g_split base base 2 --steps 20 --warmup 5 --cfg split_beta=0.3 || exit 1
tl() {  # name [args]
  local n=$1; shift
  timeout -k 10 300 python3 tools/frame_timeline.py --reps 15 --out gpurun_out/timeline_r4g_$n.json "$@" > gpurun_out/timeline_r4g_$n.txt 2>&1 || { tail -5 gpurun_out/timeline_r4g_$n.txt; exit 1; }
  echo "$n $(head -1 gpurun_out/timeline_r4g_$n.txt | cut -c1-400)"
}
tl base
PGRT_LIB=ablib/nocache/libpgrt.so tl nocache
tl split03 --cfg split_beta=0.3
tl split10 --cfg split_beta=1.0
