#!/bin/bash
# r6t: with ShadowFinal the pending finish has the dielectric pixels only (dispatch-bound: 130k-261k
# waves, p90 0.7 us): 8 / 32 mask words per wave (ablib/fw8, fw32) vs one (tree) -- parity, then the
# driver line and the 600-frame line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in fw8 fw32; do
  PGRT_LIB=ablib/$v/libpgrt.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py > gpurun_out/r6t_tests_$v.log 2>&1 || { tail -30 gpurun_out/r6t_tests_$v.log; exit 1; }
  tail -1 gpurun_out/r6t_tests_$v.log
done
RUNS=3 bash tools/ab_multi.sh r6t base ablib/fw8/libpgrt.so ablib/fw32/libpgrt.so || exit 1
RUNS=2 ARGS="--steps 600" bash tools/ab_multi.sh r6t600 base ablib/fw8/libpgrt.so ablib/fw32/libpgrt.so || exit 1
