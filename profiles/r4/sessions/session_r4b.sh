#!/bin/bash
# r4b: parity (the subtree launch included), then same-box A/B: r3 head / the pruned library without
# the streaming cache policy / with it (default), device timelines, the driver's line per subtree level
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4b.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_r4b.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/gpu_tests_r4b.log | head -20; exit $rc; fi
for pair in "ablib/r3head/libpgrt.so ablib/nocache/libpgrt.so" "ablib/nocache/libpgrt.so base"; do
  bash tools/ab_pair.sh r4b $pair 3 || exit 1
done
PGRT_LIB=ablib/nocache/libpgrt.so timeout -k 10 300 python tools/frame_timeline.py --out gpurun_out/timeline_r4b_nocache.json > gpurun_out/timeline_r4b_nocache.txt 2>&1 || exit 1
echo "nocache: $(head -1 gpurun_out/timeline_r4b_nocache.txt | cut -c1-400)"
echo "nocache: $(grep '^r20' gpurun_out/timeline_r4b_nocache.txt | cut -c1-600)"
for sub in -1 1 2 3 4; do
  timeout -k 10 300 python tools/frame_timeline.py --cfg subtree_level=$sub --out gpurun_out/timeline_r4b_sub$sub.json > gpurun_out/timeline_r4b_sub$sub.txt 2>&1 || exit 1
  echo "sub $sub: $(head -1 gpurun_out/timeline_r4b_sub$sub.txt | cut -c1-400)"
  echo "sub $sub: $(grep '^r20' gpurun_out/timeline_r4b_sub$sub.txt | cut -c1-600)"
done
for r in 1 2; do
  for sub in -1 1 2 3; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 20 --warmup 5 --cfg subtree_level=$sub > gpurun_out/b.json 2> gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/b.json')); print('sub $sub [--steps 20]', d['ms_per_step'], 'latency', d['frame_latency_ms'])" | tee -a gpurun_out/ab_r4b_sub.txt
  done
done
