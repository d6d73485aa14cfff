#!/bin/bash
# r6fin3 (part b): final head -- GPU suite + smoke, every config's bench line, the driver's line twice
# more, the default line, the path line, the steady 400-frame breakdown
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh tests smoke || exit 1
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -1
bash tools/round_bench.sh r6fin3 || exit 1
for r in 2 3; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r6fin3_C2_k20_$r.json 2> gpurun_out/bench_r6fin3_C2_k20_$r.err || { tail -5 gpurun_out/bench_r6fin3_C2_k20_$r.err; exit 1; }
done
for f in gpurun_out/bench_r6fin3_C2_k20*.json; do
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], 'driver line', d['ms_per_step'], 'lat', d.get('frame_latency_ms'), 'frac', r['frac'], r.get('frac_source'), r['frame']['frac'])" "$f"
done
timeout -k 10 400 python3 bench.py --mode path --steps 20 --warmup 3 > gpurun_out/bench_r6fin3_path.json 2> gpurun_out/bench_r6fin3_path.err || { tail -5 gpurun_out/bench_r6fin3_path.err; exit 1; }
