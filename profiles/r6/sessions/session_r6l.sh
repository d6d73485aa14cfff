#!/bin/bash
# r6l: the pending finish packs the set bits of 8 mask words onto a wave's lanes (PGRT_FINISH_WORDS=8,
# in tree) against one wave per word (fw1 = head) and 4 / 16 words: parity first, then the driver line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py > gpurun_out/r6l_tests.log 2>&1 || { tail -30 gpurun_out/r6l_tests.log; exit 1; }
tail -2 gpurun_out/r6l_tests.log
RUNS=3 bash tools/ab_multi.sh r6l base ablib/fw1/libpgrt.so ablib/fw4/libpgrt.so ablib/fw16/libpgrt.so || exit 1
