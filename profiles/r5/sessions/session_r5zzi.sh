#!/bin/bash
# r5zzi: the packet traversal's triangle records loaded at full width (3 scalar loads per triangle
# instead of 7 narrowed ones; more SGPRs live) vs head: full GPU suite, driver line, 400 frames, C5,
# synchronous frame timeline (3 runs each)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash tools/gpu_check.sh tests || exit 1
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1
grep -q " failed" gpurun_out/gpu_tests.log && exit 1
AB_EXTRA="--config C5 --steps 20 --warmup 3" bash tools/ab_head.sh r5zzi "frame_parity or packet or subtree" || exit 1
for rep in 1 2 3; do
  for lib in head new; do
    if [ $lib = head ]; then export PGRT_LIB=ablib/head/libpgrt.so; else unset PGRT_LIB; fi
    timeout -k 10 300 python3 tools/frame_timeline.py --out gpurun_out/timeline_r5zzi_${lib}_$rep.json > gpurun_out/timeline_r5zzi_${lib}_$rep.txt 2>&1 || { tail -5 gpurun_out/timeline_r5zzi_${lib}_$rep.txt; exit 1; }
    echo "$lib $(head -1 gpurun_out/timeline_r5zzi_${lib}_$rep.txt | cut -c1-260)"
    grep -E "combine +L1|finish" gpurun_out/timeline_r5zzi_${lib}_$rep.txt | head -4
  done
done
unset PGRT_LIB
