#!/bin/bash
# r4ad: the level-0 shade at 7 waves, bounce shades at 7 waves, vs HEAD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in l0f7 sh7; do
  PGRT_LIB=ablib/$v/libpgrt.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "frame_parity or geosphere or full_size or tile_order or subtree or batched" > gpurun_out/gpu_tests_r4ad_$v.log 2>&1; rc=$?
  echo "$v $(tail -1 gpurun_out/gpu_tests_r4ad_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
bash tools/ab_matrix.sh r4ad "ablib/head/libpgrt.so ablib/l0f7/libpgrt.so ablib/sh7/libpgrt.so" "--steps 20 --warmup 5" "--steps 400" || exit 1
