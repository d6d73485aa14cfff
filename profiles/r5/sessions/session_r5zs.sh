#!/bin/bash
# r5zs(b): bisect the branch-free packet step further: v1 = branchy step on the 1-based stack with the early top read; v3 = the branch-free step with a conditional push
# (offs) or the branch-free node step only (step): the golden / parity tests under each build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for lib in v1 v3; do
  PGRT_LIB=ablib/$lib/libpgrt.so timeout -k 10 300 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "frames_equal_golden or avenger_frame_parity or packet" > gpurun_out/gpu_tests_r5zs_$lib.log 2>&1
  rc=$?
  echo "$lib rc=$rc $(tail -1 gpurun_out/gpu_tests_r5zs_$lib.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
