#!/bin/bash
# r4t: deep tiles first for multi-frame calls in flight (each call: a high-priority deep slot +
# the rest) -- full GPU suite, then the driver's line and the 400-frame line, tile_order 0 vs -1
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4t.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r4t.log
[ $rc -eq 0 ] || exit $rc
b() {  # label args...
  local n=$1; shift
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline "$@" > gpurun_out/r4t.json 2>gpurun_out/r4t.err || { tail -3 gpurun_out/r4t.err; exit 1; }
  echo "$n $(python3 -c "import json; d=json.load(open('gpurun_out/r4t.json')); print(d['ms_per_step'], d['frame_latency_ms'])")"
}
for r in 1 2 3; do
  b "r20 deep" --steps 20 --warmup 5
  b "r20 rr  " --steps 20 --warmup 5 --cfg tile_order=-1
  b "r20 deep if6" --steps 20 --warmup 5 --in-flight 6
done
for r in 1 2; do
  b "400 deep" --steps 400
  b "400 rr  " --steps 400 --cfg tile_order=-1
done
timeout -k 10 300 python3 tools/frame_timeline.py --reps 5 --out gpurun_out/timeline_r4t.json > gpurun_out/timeline_r4t.txt 2>&1
