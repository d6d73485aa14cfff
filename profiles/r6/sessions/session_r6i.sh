#!/bin/bash
# r6i: the synchronous frame -- whole ray trees from level 1 (--cfg subtree_level=1, both slots) and the
# cooperative kernel with one trace call site (ablib/coopu) against the head, same box, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
RUNS=3 bash tools/ab_multi.sh r6i base "sub1=--cfg subtree_level=1" ablib/coopu/libpgrt.so || exit 1
