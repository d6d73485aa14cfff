#!/bin/bash
# r4aa: occupancy builds -- bounce-level packets at 8 waves, bounce shades at 8, the level-0 shade at 6 -- vs HEAD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in bpk8 sh8 l0f6; do
  PGRT_LIB=ablib/$v/libpgrt.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "frame_parity or geosphere or full_size or tile_order or subtree or batched" > gpurun_out/gpu_tests_r4aa_$v.log 2>&1; rc=$?
  echo "$v $(tail -1 gpurun_out/gpu_tests_r4aa_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
bash tools/ab_matrix.sh r4aa "ablib/head/libpgrt.so ablib/bpk8/libpgrt.so ablib/sh8/libpgrt.so ablib/l0f6/libpgrt.so" "--steps 20 --warmup 5" "--steps 400" || exit 1
