#!/bin/bash
# r6fin3 (part c): the cleaned final head (rejected A/B switches removed: chain priority, non-temporal
# texels, multi-word finish) -- GPU suite + smoke and two driver lines, then the steady throughput
# breakdown without the synchronous latency frames (--no-latency), 400 frames in 8-frame calls
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh tests smoke || exit 1
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r6fin3c_C2_k20_$r.json 2> gpurun_out/bench_r6fin3c_C2_k20_$r.err || { tail -5 gpurun_out/bench_r6fin3c_C2_k20_$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('driver line', d['ms_per_step'], 'lat', d.get('frame_latency_ms'))" gpurun_out/bench_r6fin3c_C2_k20_$r.json
done
bash tools/steady_profile.sh r6fin3s8 --steps 400 --frames-per-call 8 || exit 1
