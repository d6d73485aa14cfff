#!/bin/bash
# r4z: 512-thread shade blocks (half the allocation atomics) and the 8-wave level-0 packet build for
# the avenger, against HEAD; parity of each variant on a subset
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in sb512 l0w8; do
  PGRT_LIB=ablib/$v/libpgrt.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "frame_parity or geosphere or full_size or tile_order or subtree or batched" > gpurun_out/gpu_tests_r4z_$v.log 2>&1; rc=$?
  echo "$v $(tail -1 gpurun_out/gpu_tests_r4z_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
bash tools/ab_matrix.sh r4z "ablib/head/libpgrt.so ablib/sb512/libpgrt.so ablib/l0w8/libpgrt.so" "--steps 20 --warmup 5" "--steps 400" || exit 1
