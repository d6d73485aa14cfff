#!/bin/bash
# r5a: baseline of the r4 head on this round's boxes -- full GPU suite + smoke, the D2H bandwidth
# probe (host framebuffer design), the driver's line x3, the steady-state breakdown (400 frames,
# PMC) and the device timeline (synchronous frame + driver region)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh tests smoke || exit 1
echo "=== d2h probe"
timeout -k 10 120 ./build/d2h_probe > gpurun_out/d2h_probe_r5a.txt 2>&1 || { tail -5 gpurun_out/d2h_probe_r5a.txt; exit 1; }
cat gpurun_out/d2h_probe_r5a.txt
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r5a_k20_$r.json 2> gpurun_out/bench_r5a_k20_$r.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/bench_r5a_k20_$r.json')); print('driver line', d['ms_per_step'], 'lat', d['frame_latency_ms'], 'host', d['host_framebuffer']['ms_per_frame_sync_median'], d['host_framebuffer']['ms_per_frame_async'], 'frac', d['roofline']['frame']['frac'])"
done
bash tools/steady_profile.sh r5a || exit 1
echo "=== timeline"
timeout -k 10 300 python3 tools/frame_timeline.py --out gpurun_out/timeline_r5a.json > gpurun_out/timeline_r5a.txt 2>&1 || { tail -5 gpurun_out/timeline_r5a.txt; exit 1; }
echo done
