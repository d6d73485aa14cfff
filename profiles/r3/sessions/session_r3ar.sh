#!/bin/bash
# r3ar (final head, tag r3fin): rocprofv3 kernel stats + PMC traffic for C2 and C5 first (the new
# traffic files replace profiles/r3/traffic_C2/C5.json so the bench lines carry this head's
# counters), then every BASELINE config (tools/round_bench.sh) and the path tracer
set -u
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
bash tools/profile.sh r3fin C2 || exit 1
bash tools/profile.sh r3fin C5 || exit 1
cp gpurun_out/prof_r3fin_C2/traffic_C2.json profiles/r3/traffic_C2.json || exit 1
cp gpurun_out/prof_r3fin_C5/traffic_C5.json profiles/r3/traffic_C5.json || exit 1
bash tools/round_bench.sh r3fin || exit 1
timeout -k 10 300 python3 bench.py --mode path --no-cpu-baseline > gpurun_out/bench_r3fin_path.json 2> gpurun_out/bench_r3fin_path.err || { tail -5 gpurun_out/bench_r3fin_path.err; exit 1; }
