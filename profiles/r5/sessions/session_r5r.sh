#!/bin/bash
# r5r: the driver's line (--steps 20 --warmup 5) under schedule settings: 8-lane group threshold,
# frames per call, bounce-level packet budget (3 runs each, same box)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash tools/ab_matrix.sh r5r "base" "--steps 20 --warmup 5" "--steps 20 --warmup 5 --group-max 300000" \
  "--steps 20 --warmup 5 --group-max 600000" "--steps 20 --warmup 5 --frames-per-call 10" \
  "--steps 20 --warmup 5 --frames-per-call 7" "--steps 20 --warmup 5 --cfg packet_budget=128" \
  "--steps 20 --warmup 5 --cfg packet_budget=64" "--steps 20 --warmup 5 --packet-levels 2" "--steps 20 --warmup 5"
