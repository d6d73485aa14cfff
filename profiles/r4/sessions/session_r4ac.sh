#!/bin/bash
# r4ac: the level-0 shade at 6 waves per SIMD -- full GPU suite + smoke, the driver's line (3 runs, with
# the full line once) and 400 frames
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh tests smoke || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench_r4ac_C2_k20.json 2> gpurun_out/bench_r4ac.err || exit 1
bash tools/ab_matrix.sh r4ac "base" "--steps 20 --warmup 5" "--steps 400" || exit 1
