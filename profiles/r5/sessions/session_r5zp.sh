#!/bin/bash
# r5zp: synchronous frames' subtree launch with two 4-lane groups per ray tree, split at the tree's
# first two-child dielectric node (new) vs one 8-lane group per tree (head) -- full GPU suite, then
# the synchronous C2 frame timeline of each, 3 interleaved runs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash tools/gpu_check.sh tests || exit 1
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1
for rep in 1 2 3; do
  for lib in head new; do
    if [ $lib = head ]; then export PGRT_LIB=ablib/head/libpgrt.so; else unset PGRT_LIB; fi
    timeout -k 10 300 python3 tools/frame_timeline.py --out gpurun_out/timeline_r5zp_${lib}_$rep.json > gpurun_out/timeline_r5zp_${lib}_$rep.txt 2>&1 || { tail -5 gpurun_out/timeline_r5zp_${lib}_$rep.txt; exit 1; }
    echo "$lib $(head -1 gpurun_out/timeline_r5zp_${lib}_$rep.txt)"
    grep -E "subtree" gpurun_out/timeline_r5zp_${lib}_$rep.txt | head -2
  done
done
unset PGRT_LIB
