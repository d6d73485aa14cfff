#!/bin/bash
# r5zzg: the 1-spp finish's workgroup size (PGRT_FINISH_BLOCK) 64 / 128 / 256 (head) after 1024 was
# 2x slower (r5zzf) -- driver line, 400 frames, C5, 3 runs per cell, same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash tools/ab_matrix.sh r5zzg "ablib/fb256/libpgrt.so ablib/fb64/libpgrt.so ablib/fb128/libpgrt.so" "--steps 20 --warmup 5" "--steps 400" "--config C5 --steps 20 --warmup 3" || exit 1
