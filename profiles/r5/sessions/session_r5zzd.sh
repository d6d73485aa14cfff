#!/bin/bash
# r5zzd: the synchronous frame's deep-tile slot traces its level 0 per ray (raygen + the 8 / 4-lane
# or one-lane kernel) instead of as 8x8 packets vs head: full GPU suite, driver line, 400 frames, C5,
# synchronous frame timeline (3 runs each; the deep slot's level-0 launches printed)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash tools/gpu_check.sh tests || exit 1
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1
grep -q " failed" gpurun_out/gpu_tests.log && exit 1
AB_EXTRA="--config C5 --steps 20 --warmup 3" bash tools/ab_head.sh r5zzd "frame_parity or packet or subtree" || exit 1
for rep in 1 2 3; do
  for lib in head new; do
    if [ $lib = head ]; then export PGRT_LIB=ablib/head/libpgrt.so; else unset PGRT_LIB; fi
    timeout -k 10 300 python3 tools/frame_timeline.py --out gpurun_out/timeline_r5zzd_${lib}_$rep.json > gpurun_out/timeline_r5zzd_${lib}_$rep.txt 2>&1 || { tail -5 gpurun_out/timeline_r5zzd_${lib}_$rep.txt; exit 1; }
    echo "$lib $(head -1 gpurun_out/timeline_r5zzd_${lib}_$rep.txt | cut -c1-260)"
    grep -E "s0 (trace|trace_pkt|trace8g|raygen|shade) +L0|s0 subtree" gpurun_out/timeline_r5zzd_${lib}_$rep.txt | head -4
  done
done
unset PGRT_LIB
