#!/bin/bash
# r6y: a synchronous frame's deep-tile slot traces its bounce levels by lane groups in one launch
# (PGRT_DEEP_SLOT_NO_PKT=1, ablib/dsnp: its level 1 was a packet launch 29 us + a deferred-ray resume
# 69 us in r6fin3) vs the tree: parity subset, then 4 driver lines each (frame_latency_ms)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PGRT_LIB=ablib/dsnp/libpgrt.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/r6y_tests.log 2>&1 || { tail -30 gpurun_out/r6y_tests.log; exit 1; }
tail -n 1 gpurun_out/r6y_tests.log
RUNS=4 bash tools/ab_multi.sh r6y base ablib/dsnp/libpgrt.so || exit 1
