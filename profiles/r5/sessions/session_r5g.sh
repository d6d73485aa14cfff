#!/bin/bash
# r5g: work-sharing subtree launch (refraction children of a block's ray trees taken by idle
# groups) -- subtree parity first, the full suite, the synchronous-frame timeline, the driver line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "subtree" > gpurun_out/gpu_tests_sub_r5g.log 2>&1 || { tail -30 gpurun_out/gpu_tests_sub_r5g.log; exit 1; }
tail -2 gpurun_out/gpu_tests_sub_r5g.log
bash tools/gpu_check.sh tests smoke || exit 1
timeout -k 10 300 python3 tools/frame_timeline.py --host --out gpurun_out/timeline_r5g.json > gpurun_out/timeline_r5g.txt 2>&1 || { tail -5 gpurun_out/timeline_r5g.txt; exit 1; }
grep -E "^(sync|sync_host|async_host|r20) " gpurun_out/timeline_r5g.txt
grep -E "subtree" gpurun_out/timeline_r5g.txt | head -6
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r5g_$r.json 2> gpurun_out/bench_r5g_$r.err || { tail -5 gpurun_out/bench_r5g_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_r5g_$r.json')); h=d['host_framebuffer']; print('driver line', d['ms_per_step'], 'lat', d['frame_latency_ms'], 'host', h['ms_per_frame_sync_median'], h['ms_per_frame_async'])"
done
