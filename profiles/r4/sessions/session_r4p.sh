#!/bin/bash
# r4p: steady-state (600-frame) kernel breakdown with FETCH / WRITE / SQ counters at the head
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/steady_profile.sh r4p --steps 400
