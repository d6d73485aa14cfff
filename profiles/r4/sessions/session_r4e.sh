#!/bin/bash
# r4e: stamps with a non-clobbering entry clock vs stamps compiled out (same box, interleaved),
# then the device timeline of the fixed build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_pair.sh r4e base ablib/nostamp/libpgrt.so 3 || exit 1
bash tools/ab_pair.sh r4e3 base ablib/r3head/libpgrt.so 2 || exit 1
timeout -k 10 300 python3 tools/frame_timeline.py --out gpurun_out/timeline_r4e.json > gpurun_out/timeline_r4e.txt 2>&1 || { tail -5 gpurun_out/timeline_r4e.txt; exit 1; }
head -1 gpurun_out/timeline_r4e.txt; grep '^r20' gpurun_out/timeline_r4e.txt
