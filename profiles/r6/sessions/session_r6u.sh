#!/bin/bash
# r6u: ShadowFinal at every level (the shadow trace writes the deeper levels' opaque node colours,
# k_combine skips them; tree) vs level 0 only (ablib/sfl0), and + 8 mask words per finish wave
# (ablib/fw8all): the GPU suite on the tree, parity of fw8all, the driver line, the 600-frame line,
# C3 (multi-spp: ShadowFinal off, must be unchanged)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh tests || exit 1
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1
grep -E "FAILED" gpurun_out/gpu_tests.log | head -5
PGRT_LIB=ablib/fw8all/libpgrt.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/r6u_tests_fw8all.log 2>&1 || { tail -30 gpurun_out/r6u_tests_fw8all.log; exit 1; }
tail -1 gpurun_out/r6u_tests_fw8all.log
RUNS=3 bash tools/ab_multi.sh r6u base ablib/sfl0/libpgrt.so ablib/fw8all/libpgrt.so || exit 1
RUNS=2 ARGS="--steps 600" bash tools/ab_multi.sh r6u600 base ablib/sfl0/libpgrt.so ablib/fw8all/libpgrt.so || exit 1
