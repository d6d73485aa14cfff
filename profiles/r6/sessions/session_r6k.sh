#!/bin/bash
# r6k: distributed calls no longer drain the frames in flight (finish_frame does not re-record a
# distributed set's ready event behind the later calls' gathers): the distributed GPU tests, then the
# emulated ranks of C2 at world 2 / 8 (r6e had 1.13x / 4.05x)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "distributed or multi_device" > gpurun_out/r6k_tests.log 2>&1 || { tail -30 gpurun_out/r6k_tests.log; exit 1; }
tail -3 gpurun_out/r6k_tests.log
timeout -k 10 600 python3 -u tools/emulate_ranks.py --configs C2 --worlds 2,8 --out gpurun_out/emulated_ranks_r6k.jsonl 2>&1 | tee gpurun_out/emulated_ranks_r6k.log
