#!/bin/bash
# r5x: k_finish_pending with several 64-pixel masks per wave and their node loads interleaved
# (4 masks: base; 2: fin2; 8: fin8) vs HEAD (one mask per wave) -- parity subset, the driver's line
# and 400 frames (3 runs each)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "frame_parity or full_size or golden or batched or lights or geosphere or host" > gpurun_out/gpu_tests_r5x.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r5x.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r5x.log
bash tools/ab_matrix.sh r5x "base ablib/fin2/libpgrt.so ablib/fin8/libpgrt.so ablib/head/libpgrt.so" "--steps 20 --warmup 5" "--steps 400" || exit 1
