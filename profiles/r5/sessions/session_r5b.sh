#!/bin/bash
# r5b: the split library + Embree depth test + per-slot host export -- full GPU suite + smoke, the
# driver's line x3, C5's line (timed-configuration roofline), the C2 roofline profile (kernel trace
# + PMC of exactly the roofline calls), the synchronous timeline, and the GPU suite once more
# against the host-sanitized library (ASan + UBSan on the host translation units only)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh tests smoke || exit 1
for r in 1 2 3; do
  a=""; [ $r -gt 1 ] && a="--no-cpu-baseline"
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $a > gpurun_out/bench_r5b_k20_$r.json 2> gpurun_out/bench_r5b_k20_$r.err || { tail -5 gpurun_out/bench_r5b_k20_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_r5b_k20_$r.json')); r=d['roofline']; print('driver line', d['ms_per_step'], 'lat', d['frame_latency_ms'], 'host', d['host_framebuffer']['ms_per_frame_sync_median'], d['host_framebuffer']['ms_per_frame_async'], d['host_framebuffer']['pcie_d2h_gbs'], 'frac', r['frac'], r['frame']['frac'], 'timed', r.get('timed', {}).get('frac'), r.get('timed', {}).get('trace_busy_ms_per_frame'))"
done
timeout -k 10 400 python3 bench.py --config C5 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_r5b_C5.json 2> gpurun_out/bench_r5b_C5.err || { tail -5 gpurun_out/bench_r5b_C5.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_r5b_C5.json')); r=d['roofline']; print('C5', d['ms_per_step'], 'frac', r['frac'], 'trace ms/frame', r['trace_ms_per_frame'], 'timed', r.get('timed'))"
bash tools/profile.sh r5b C2 || exit 1
echo "=== timeline"
timeout -k 10 300 python3 tools/frame_timeline.py --out gpurun_out/timeline_r5b.json > gpurun_out/timeline_r5b.txt 2>&1 || { tail -5 gpurun_out/timeline_r5b.txt; exit 1; }
# (a GPU-suite pass under the host-sanitized library was tried here and abandoned: it replaced the
# harness's preload; the sanitized host build runs on the CPU only, tools/asan_check.sh)
