#!/bin/bash
# r6a: round-6 starting point on a fresh box -- GPU suite + smoke, the driver's line twice, the
# synchronous / 20-frame device timelines at the r5 head
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh tests smoke || exit 1
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r6a_C2_k20_$r.json 2> gpurun_out/bench_r6a_C2_k20_$r.err || { tail -5 gpurun_out/bench_r6a_C2_k20_$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], 'driver line', d['ms_per_step'], 'lat', d.get('frame_latency_ms'), 'frac', r['frac'], r['frame']['frac'])" gpurun_out/bench_r6a_C2_k20_$r.json
done
timeout -k 10 300 python3 tools/frame_timeline.py --out gpurun_out/timeline_r6a.json > gpurun_out/timeline_r6a.txt 2>&1 || { tail -5 gpurun_out/timeline_r6a.txt; exit 1; }
