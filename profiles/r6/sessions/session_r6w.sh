#!/bin/bash
# r6w: which TA / TCP (vector L1) counters this rocprofv3 offers on gfx950 (for the one-lane
# traversal's L1-throughput question)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
grep -E "^\s*(TA_|TCP_|TD_)" gpurun_out/rocprof_counters.txt | head -80 || true
grep -c "" gpurun_out/rocprof_counters.txt
