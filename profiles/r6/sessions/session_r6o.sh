#!/bin/bash
# r6o: the driver-shaped 20-frame job per emulated rank of C2 at world 2 / 8: whole ray trees from level
# 2 / 3 for the ranks' multi-frame calls (--cfg subtree_level), one call of 20 frames (F = 64 rule) or 8
# per call; then the one-shot AUTO probe (in tree) on the one-GPU driver line against the head
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for f in 0 8; do
  for sl in 2 3; do
    extra=""; [ $f -gt 0 ] && extra="--fpc $f"
    timeout -k 10 300 python3 -u tools/emulate_ranks.py --configs C2 --worlds 2,8 --frames 20 --warmup 5 --repeat 5 $extra \
      --cfg subtree_level=$sl --out gpurun_out/emu_r6o_fpc${f}_sub$sl.jsonl 2>&1 | tee gpurun_out/emu_r6o_fpc${f}_sub$sl.log || exit 1
  done
done
RUNS=3 bash tools/ab_multi.sh r6o base ablib/head/libpgrt.so || exit 1
