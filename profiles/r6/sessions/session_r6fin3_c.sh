#!/bin/bash
# r6fin3 (part c): the steady throughput breakdown at the final head without the synchronous latency
# frames in the trace (--no-latency; earlier breakdowns counted their per-slot k_export_counters as
# calls): 400 frames in 8-frame calls and in 32-frame calls (the default for long jobs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/steady_profile.sh r6fin3s8 --steps 400 --frames-per-call 8 || exit 1
