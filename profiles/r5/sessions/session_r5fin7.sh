#!/bin/bash
# r5fin7: final-head evidence (r5fin6 + full-width triangle loads in the packet traversal) -- GPU suite + smoke, every config's bench line (round_bench), the driver's
# line twice more, the path line, the C2 and C5 roofline profiles (kernel trace + PMC of exactly the
# roofline calls), the synchronous / 20-frame device timelines, the host-framebuffer figures
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh tests smoke || exit 1
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1
bash tools/round_bench.sh r5fin7 || exit 1
for r in 2 3; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r5fin7_C2_k20_$r.json 2> gpurun_out/bench_r5fin7_C2_k20_$r.err || { tail -5 gpurun_out/bench_r5fin7_C2_k20_$r.err; exit 1; }
done
for f in gpurun_out/bench_r5fin7_C2_k20*.json; do
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], 'driver line', d['ms_per_step'], 'lat', d.get('frame_latency_ms'), 'frac', r['frac'], r['frame']['frac'], 'timed', r.get('timed', {}).get('frac'))" "$f"
done
timeout -k 10 400 python3 bench.py --mode path --steps 20 --warmup 3 > gpurun_out/bench_r5fin7_path.json 2> gpurun_out/bench_r5fin7_path.err || { tail -5 gpurun_out/bench_r5fin7_path.err; exit 1; }
bash tools/profile.sh r5fin7 C2 || exit 1
bash tools/profile.sh r5fin7 C5 || exit 1
timeout -k 10 300 python3 tools/frame_timeline.py --out gpurun_out/timeline_r5fin7.json > gpurun_out/timeline_r5fin7.txt 2>&1 || { tail -5 gpurun_out/timeline_r5fin7.txt; exit 1; }
timeout -k 10 200 python3 tools/host_fb.py --async > gpurun_out/host_r5fin7.json 2>&1 && cat gpurun_out/host_r5fin7.json
timeout -k 10 300 python3 tools/frame_timeline.py --host --out gpurun_out/timeline_host_r5fin7.json > gpurun_out/timeline_host_r5fin7.txt 2>&1 || exit 1
