#!/bin/bash
# r6e: every rank of world 2 / 4 / 8 rendered on one GPU (emulated, PGRT_EMULATE_RANK) for C2 and C4
# (verdict r5 #7): per-rank ms/frame, max/mean, rank 0's unpack; no RCCL, no xGMI transfer
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u tools/emulate_ranks.py --out gpurun_out/emulated_ranks_r6e.jsonl 2>&1 | tee gpurun_out/emulated_ranks_r6e.log
