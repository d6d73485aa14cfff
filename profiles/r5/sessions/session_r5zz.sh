#!/bin/bash
# r5zz: steady-state per-kernel breakdown at the head after the offset-addressing changes (400 frames,
# two SQ counter passes): the level-0 shade's SQ_WAIT_ANY share after the two-part shades
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
bash tools/steady_profile.sh r5zz || exit 1
