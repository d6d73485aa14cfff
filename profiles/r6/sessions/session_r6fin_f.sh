#!/bin/bash
# r6fin (part f): the default line (no flags: 600 frames, now 32 frames per call) twice and the
# driver's line once more, at the final head
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 400 python3 bench.py > gpurun_out/bench_r6fin_default_$r.json 2> gpurun_out/bench_r6fin_default_$r.err || { tail -5 gpurun_out/bench_r6fin_default_$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('default line', d['ms_per_step'], d['frames_per_call'], 'frac', r['frac'], r['frac_source'], 'frame', r['frame']['frac'], 'host', d['host_framebuffer']['ms_per_frame_sync_median'], d['host_framebuffer']['ms_per_frame_async'])" gpurun_out/bench_r6fin_default_$r.json
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r6fin_C2_k20_4.json 2> gpurun_out/bench_r6fin_C2_k20_4.err || { tail -5 gpurun_out/bench_r6fin_C2_k20_4.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('driver line', d['ms_per_step'], d['frames_per_call'], 'lat', d.get('frame_latency_ms'))" gpurun_out/bench_r6fin_C2_k20_4.json
