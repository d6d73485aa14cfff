#!/bin/bash
# r5zo: k_finish_pending with compacted pending pixels (8 masks per wave, one pending pixel per lane
# and round) vs one wave per mask (head) -- full GPU suite, driver / 400-frame lines (3 runs each,
# same box), synchronous frame timeline of each, and a steady kernel trace of the new build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash tools/gpu_check.sh tests || exit 1
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1
AB_EXTRA="--config C5 --steps 20 --warmup 3" bash tools/ab_head.sh r5zo "frame_parity" || exit 1
for lib in head new; do
  if [ $lib = head ]; then export PGRT_LIB=ablib/head/libpgrt.so; else unset PGRT_LIB; fi
  timeout -k 10 300 python3 tools/frame_timeline.py --out gpurun_out/timeline_r5zo_$lib.json > gpurun_out/timeline_r5zo_$lib.txt 2>&1 || { tail -5 gpurun_out/timeline_r5zo_$lib.txt; exit 1; }
  echo "$lib $(head -1 gpurun_out/timeline_r5zo_$lib.txt)"
  grep -E "finish" gpurun_out/timeline_r5zo_$lib.txt | head -4
done
unset PGRT_LIB
