#!/bin/bash
# r5zm: steady-state per-kernel breakdown at the head (400 frames, kernel trace + FETCH/WRITE +
# two SQ counter passes): the level-0 shade's SQ_WAIT_ANY share after the two-part shades
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
bash tools/steady_profile.sh r5zm || exit 1
