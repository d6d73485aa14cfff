#!/bin/bash
# r6j: spread tree mapping in k_subtree (PGRT_SUBTREE_SPREAD=1: the trees of a wave lie a grid apart in
# the queue) against the head, for the synchronous frame (subtree from level 2) and for multi-frame calls
# with subtree from level 3/4, same box, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
RUNS=3 bash tools/ab_multi.sh r6j base ablib/spread/libpgrt.so "ablib/spread/libpgrt.so@--cfg subtree_level=3" "ablib/spread/libpgrt.so@--cfg subtree_level=4" || exit 1
