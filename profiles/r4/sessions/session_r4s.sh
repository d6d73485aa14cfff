#!/bin/bash
# r4s: call_order 2 (each call's level-0 trace waits for the previous call's level-0 trace) vs the
# default (calls free) and call_order 1, on the driver's line and the 400-frame line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "frames_in_flight or batched or distinct or call_order" > gpurun_out/gpu_tests_r4s.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests_r4s.log; [ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
for r in 1 2 3; do
  for c in 0 2 1; do
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline --steps 20 --warmup 5 --cfg call_order=$c > gpurun_out/r4s.json 2>gpurun_out/r4s.err || { tail -3 gpurun_out/r4s.err; exit 1; }
    echo "r20 call_order=$c $(python3 -c "import json; d=json.load(open('gpurun_out/r4s.json')); print(d['ms_per_step'], d['frame_latency_ms'])")"
  done
done
for c in 0 2; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline --steps 400 --cfg call_order=$c > gpurun_out/r4s.json 2>gpurun_out/r4s.err || exit 1
  echo "400 call_order=$c $(python3 -c "import json; d=json.load(open('gpurun_out/r4s.json')); print(d['ms_per_step'])")"
done
timeout -k 10 300 python3 tools/frame_timeline.py --reps 5 --cfg call_order=2 --out gpurun_out/timeline_r4s_co2.json > gpurun_out/timeline_r4s_co2.txt 2>&1
