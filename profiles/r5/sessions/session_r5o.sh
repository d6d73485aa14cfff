#!/bin/bash
# r5o: split host copy as the in-flight default -- host parity tests, host_fb (default mode), the
# synchronous / asynchronous host-output timelines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "host or batched" > gpurun_out/gpu_tests_r5o.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r5o.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r5o.log
timeout -k 10 200 python3 tools/host_fb.py --async 8x4 2x4 > gpurun_out/host_r5o.json 2>&1 && cat gpurun_out/host_r5o.json || exit 1
timeout -k 10 300 python3 tools/frame_timeline.py --host --out gpurun_out/timeline_r5o.json > gpurun_out/timeline_r5o.txt 2>&1 || { tail -5 gpurun_out/timeline_r5o.txt; exit 1; }
grep -n "^sync_host" -A40 gpurun_out/timeline_r5o.txt | cut -c1-170
