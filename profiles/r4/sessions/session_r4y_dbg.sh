#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "tile_order" > gpurun_out/r4y_dbg.log 2>&1; rc=$?
grep -n "Error\|assert\|exact\|diff\|rep\|passed\|failed" gpurun_out/r4y_dbg.log | head -30
exit $rc
