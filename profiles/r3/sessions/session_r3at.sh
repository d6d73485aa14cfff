#!/bin/bash
# r3at: C4 PMC traffic (tools/profile.sh) and the C4 bench line with its CPU baseline (every 16th row)
set -u
cd "$(dirname "$0")/.."
export PYTHONUNBUFFERED=1
bash tools/profile.sh r3fin C4 || exit 1
cp gpurun_out/prof_r3fin_C4/traffic_C4.json profiles/r3/traffic_C4.json || exit 1
timeout -k 10 500 python3 bench.py --config C4 --steps 6 --warmup 2 > gpurun_out/bench_r3fin_C4.json 2> gpurun_out/bench_r3fin_C4.err || { tail -5 gpurun_out/bench_r3fin_C4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_r3fin_C4.json')); print(d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('traffic'), d['roofline'].get('traffic_frac'), (d.get('cpu_baseline') or {}).get('value'))"
