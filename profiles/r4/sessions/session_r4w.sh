#!/bin/bash
# r4w: slot 1's level-0 grid cap in deep-tiles-first synchronous frames (pgrt_config.slot1_grid)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "tile_order or frame_parity or full_size or subtree" > gpurun_out/gpu_tests_r4w.log 2>&1; rc=$?
tail -1 gpurun_out/gpu_tests_r4w.log; [ $rc -eq 0 ] || exit $rc
tl() {  # name [args]
  local n=$1; shift
  timeout -k 10 300 python3 tools/frame_timeline.py --reps 21 --out gpurun_out/timeline_r4w_$n.json "$@" > gpurun_out/timeline_r4w_$n.txt 2>&1 || { tail -5 gpurun_out/timeline_r4w_$n.txt; exit 1; }
  echo "$n $(head -1 gpurun_out/timeline_r4w_$n.txt | grep -o '"host_ms_median_timeline_off.*')"
}
for r in 1 2; do
  tl nocap$r --cfg slot1_grid=-1
  tl g1024_$r
  tl g512_$r --cfg slot1_grid=512
  tl g1536_$r --cfg slot1_grid=1536
  tl g256_$r --cfg slot1_grid=256
done
