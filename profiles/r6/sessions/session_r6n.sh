#!/bin/bash
# r6n: the driver-shaped job (20 frames after 5 warm-up frames, median of 5) per emulated rank of C2 at
# world 2 / 8, with bench.py's frames-per-call rule (8 x world) and with 8 / 4 frames per call
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for f in 0 8 4; do
  extra=""; [ $f -gt 0 ] && extra="--fpc $f"
  timeout -k 10 380 python3 -u tools/emulate_ranks.py --configs C2 --worlds 2,8 --frames 20 --warmup 5 --repeat 5 $extra \
    --out gpurun_out/emu_r6n_fpc$f.jsonl 2>&1 | tee gpurun_out/emu_r6n_fpc$f.log || exit 1
done
