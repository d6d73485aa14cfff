#!/bin/bash
# r6v: k_combine grid capped at 1024 / 256 blocks (each thread loops over several nodes; with ShadowFinal
# most nodes are skipped) vs 4096 (tree): parity subset, driver line, 600-frame line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PGRT_LIB=ablib/cg256/libpgrt.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "avenger or glass or geosphere or distinct" > gpurun_out/r6v_tests.log 2>&1 || { tail -30 gpurun_out/r6v_tests.log; exit 1; }
tail -1 gpurun_out/r6v_tests.log
RUNS=3 bash tools/ab_multi.sh r6v base ablib/cg1024/libpgrt.so ablib/cg256/libpgrt.so || exit 1
RUNS=2 ARGS="--steps 600" bash tools/ab_multi.sh r6v600 base ablib/cg1024/libpgrt.so ablib/cg256/libpgrt.so || exit 1
