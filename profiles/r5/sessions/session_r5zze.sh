#!/bin/bash
# r5zze: the shade kernels' occupancy bound re-tuned after the offset changes -- bounce levels at 5 / 7
# waves per SIMD (bw5 / bw7; head 6: 80 VGPRs, 18 dwords spilled; 5: 89, none; 7: 72, 5 spilled) and
# level 0 at 5 / 7 (lw5 / lw7; head 6: 37 spilled; 5: 90, none; 7: 72, 37) -- driver line and 400
# frames, 3 runs per cell, same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash tools/ab_matrix.sh r5zze "base ablib/bw5/libpgrt.so ablib/bw7/libpgrt.so ablib/lw5/libpgrt.so ablib/lw7/libpgrt.so" "--steps 20 --warmup 5" "--steps 400" || exit 1
