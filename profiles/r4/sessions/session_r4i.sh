#!/bin/bash
# r4i: work donation between the 8-lane groups of a wave (trace8_donate): parity, then same-box
# A/B against PGRT_DONATE=0 on the driver's line and the synchronous frame's timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4i.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r4i.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab_pair.sh r4i base ablib/nodonate/libpgrt.so 3 || exit 1
tl() {  # name [args]
  local n=$1; shift
  timeout -k 10 300 python3 tools/frame_timeline.py --reps 15 --out gpurun_out/timeline_r4i_$n.json "$@" > gpurun_out/timeline_r4i_$n.txt 2>&1 || { tail -5 gpurun_out/timeline_r4i_$n.txt; exit 1; }
  echo "$n $(head -1 gpurun_out/timeline_r4i_$n.txt | grep -o '"host_ms_median_timeline_off.*')  r20 $(grep '^r20' gpurun_out/timeline_r4i_$n.txt | grep -o '"host_ms_per_frame_off_median": [0-9.]*')"
}
tl base
PGRT_LIB=ablib/nodonate/libpgrt.so tl nodonate
tl pkt1 --cfg packet_levels=1
