#!/bin/bash
# r4r: finish groups per wave (2 / 4 / 16 vs HEAD's one thread per pixel), C5 bench line + profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_matrix.sh r4r "ablib/head/libpgrt.so ablib/fin2/libpgrt.so ablib/fin4/libpgrt.so base" "--steps 20 --warmup 5" "--steps 400" || exit 1
timeout -k 10 400 python3 bench.py --config C5 --steps 20 --warmup 3 > gpurun_out/bench_r4r_C5.json 2> gpurun_out/bench_r4r_C5.err || exit 1
bash tools/profile.sh r4r C5
