#!/bin/bash
# r4d: which change broke test_gpu_frames_equal_golden: the library variants on the golden and
# frame-parity tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for L in ablib/r3head/libpgrt.so ablib/nocache/libpgrt.so ablib/stonly/libpgrt.so ablib/ldonly/libpgrt.so base; do
  if [ "$L" = base ]; then unset PGRT_LIB; else export PGRT_LIB=$L; fi
  timeout -k 10 300 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    -k "golden or frame_parity or geosphere or closest_hit" > gpurun_out/bisect.log 2>&1
  rc=$?
  echo "$L rc=$rc $(tail -1 gpurun_out/bisect.log)"
  grep -E "^FAILED" gpurun_out/bisect.log | head -8
  if [ $rc -gt 1 ]; then exit $rc; fi
done
unset PGRT_LIB
timeout -k 10 300 python -u -m pytest tests/test_golden.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/golden_base.log 2>&1
tail -30 gpurun_out/golden_base.log
