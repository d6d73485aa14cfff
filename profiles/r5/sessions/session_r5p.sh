#!/bin/bash
# r5p: the deep-tile slot's subtree launch off XCD 0 while the bulk slot's host export runs there
# (synchronous frames into page-locked memory) -- parity subset, host_fb A/B vs noavoid (3 runs
# each, interleaved), the synchronous host-output timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "host or subtree or frame_parity or distributed or overflow or multi_device" > gpurun_out/gpu_tests_r5p.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r5p.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r5p.log
for rep in 1 2 3; do
  for lib in base noavoid; do
    if [ $lib = base ]; then unset PGRT_LIB; else export PGRT_LIB=ablib/$lib/libpgrt.so; fi
    timeout -k 10 200 python3 tools/host_fb.py --reps 30 --async > gpurun_out/host_r5p_${lib}_$rep.json 2>&1 || { tail -5 gpurun_out/host_r5p_${lib}_$rep.json; exit 1; }
    cat gpurun_out/host_r5p_${lib}_$rep.json
  done
done
unset PGRT_LIB
timeout -k 10 300 python3 tools/frame_timeline.py --host --out gpurun_out/timeline_r5p.json > gpurun_out/timeline_r5p.txt 2>&1 || { tail -5 gpurun_out/timeline_r5p.txt; exit 1; }
grep -n "^sync_host" -A32 gpurun_out/timeline_r5p.txt | cut -c1-170
