#!/bin/bash
# r4q: compact k_finish_pending (16 mask groups per wave) against the HEAD build, same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_head.sh r4q "frame_parity or geosphere or full_size or tile_order or subtree"
