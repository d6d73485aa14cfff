#!/bin/bash
# r6fin (part e): the C5 line again with the timed roofline's busy time capped at ms_per_step, and
# frames per call on the 600-frame default line (8 vs 32 vs 64)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --config C5 --steps 20 --warmup 3 > gpurun_out/bench_r6fin_C5_capped.json 2> gpurun_out/bench_r6fin_C5_capped.err || { tail -5 gpurun_out/bench_r6fin_C5_capped.err; exit 1; }
RUNS=2 ARGS="--steps 600" bash tools/ab_multi.sh r6fin600 base "f32=--frames-per-call 32" "f64=--frames-per-call 64" || exit 1
