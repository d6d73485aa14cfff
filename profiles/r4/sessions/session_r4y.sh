#!/bin/bash
# r4y: primary-ray micro-work: lens hashes only for DoF, host-precomputed 1/S and jitter bounds, the frame index in the tile record, no run-time divisions at 1 spp --
# exhaustive check + full suite, then A/B against the HEAD build (driver's line, 400 frames, the
# synchronous frame)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "frame_parity or batched or distinct or dof or tile or path or full_size" > gpurun_out/gpu_tests_r4y_srgb.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r4y_srgb.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4y.log 2>&1; rc=$?
tail -1 gpurun_out/gpu_tests_r4y.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_matrix.sh r4y "ablib/head/libpgrt.so base" "--steps 20 --warmup 5" "--steps 400" || exit 1
for r in 1 2; do
for L in head base; do
  if [ $L = head ]; then export PGRT_LIB=ablib/head/libpgrt.so; else unset PGRT_LIB; fi
  timeout -k 10 300 python3 tools/frame_timeline.py --reps 15 --out gpurun_out/timeline_r4y_$L$r.json > gpurun_out/timeline_r4y_$L$r.txt 2>&1 || exit 1
  echo "$L $(head -1 gpurun_out/timeline_r4y_$L$r.txt | grep -o '"host_ms_median_timeline_off.*')  r20 $(grep '^r20' gpurun_out/timeline_r4y_$L$r.txt | grep -o '"host_ms_per_frame_off_median": [0-9.]*')"
done
done
