#!/bin/bash
# r6d: cooperative ray trees (k_subtree_coop, ablib/coop: PGRT_SUBTREE_COOP=1) -- a tiny frame first
# (smoke, 60 s), then the whole GPU parity suite on that library, then same-box A/B of the
# synchronous frame and the driver line against the head, and the coop timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PGRT_LIB=ablib/coop/libpgrt.so timeout -k 10 60 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6d_smoke.log 2>&1; rc=$?
cat gpurun_out/r6d_smoke.log | tail -3
[ $rc -eq 0 ] || exit 1
PGRT_LIB=ablib/coop/libpgrt.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r6d_gpu_tests_coop.log 2>&1; rc=$?
tail -3 gpurun_out/r6d_gpu_tests_coop.log
[ $rc -le 1 ] || exit 1
RUNS=3 bash tools/ab_multi.sh r6d base ablib/coop/libpgrt.so || exit 1
PGRT_LIB=ablib/coop/libpgrt.so timeout -k 10 200 python3 tools/frame_timeline.py --out gpurun_out/timeline_r6d_coop.json > gpurun_out/timeline_r6d_coop.txt 2>&1 || { tail -5 gpurun_out/timeline_r6d_coop.txt; exit 1; }
head -25 gpurun_out/timeline_r6d_coop.txt
