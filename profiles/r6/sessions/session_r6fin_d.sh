#!/bin/bash
# r6fin (part d): every rank of world 2 / 4 / 8 on one GPU (emulated) -- C2 and C4 in steady state,
# C2 as the driver-shaped 20-frame job
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python3 -u tools/emulate_ranks.py --out gpurun_out/emulated_ranks_r6fin.jsonl 2>&1 | tee gpurun_out/emulated_ranks_r6fin.log || exit 1
timeout -k 10 400 python3 -u tools/emulate_ranks.py --configs C2 --frames 20 --warmup 5 --repeat 5 --out gpurun_out/emulated_ranks_r6fin_k20.jsonl 2>&1 | tee gpurun_out/emulated_ranks_r6fin_k20.log || exit 1
