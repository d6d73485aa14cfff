#!/bin/bash
# r4fin: head evidence -- GPU suite + smoke, every config's bench line, the C2 rocprof kernel stats and
# PMC traffic, the synchronous / 20-frame device timelines, the path-tracing line with its CPU baseline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh tests smoke || exit 1
bash tools/round_bench.sh r4fin || exit 1
timeout -k 10 400 python3 bench.py --mode path --steps 20 --warmup 3 > gpurun_out/bench_r4fin_path.json 2> gpurun_out/bench_r4fin_path.err || exit 1
bash tools/profile.sh r4fin C2 || exit 1
timeout -k 10 300 python3 tools/frame_timeline.py --out gpurun_out/timeline_r4fin.json > gpurun_out/timeline_r4fin.txt 2>&1 || exit 1
