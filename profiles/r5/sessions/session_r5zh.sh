#!/bin/bash
# r5zh: what the synchronous frame's slowest subtree waves do -- a diagnostics build (ablib/stdiag:
# every ray tree of the subtree launch with > 100 node visits printf's its traces, visits, shadow
# rays and cycles) over 3 synchronous C2 frames
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
PGRT_LIB=ablib/stdiag/libpgrt.so timeout -k 10 200 python3 tools/sync_frames.py 3 > gpurun_out/stdiag_r5zh.txt 2>&1 || { tail -5 gpurun_out/stdiag_r5zh.txt; exit 1; }
grep -c TREE gpurun_out/stdiag_r5zh.txt
grep TREE gpurun_out/stdiag_r5zh.txt | sort -t' ' -k16 -n | tail -15
