#!/bin/bash
# r5zd: the work-sharing subtree form (r5g, pending dielectric nodes in LDS, refraction children taken
# by idle groups of the block) at the synchronous frame's new level-2 start (trees 3 levels deep)
# vs the one-group-per-tree launch (nows) -- subtree parity, host ms of a synchronous frame (4
# interleaved runs) with the slot-0 subtree launch, and the driver's line (unaffected: level 3+,
# per-level launches for calls in flight)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "subtree or frame_parity or full_size" > gpurun_out/gpu_tests_r5zd.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r5zd.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r5zd.log
for rep in 1 2 3 4; do
  for lib in base nows; do
    if [ $lib = base ]; then unset PGRT_LIB; else export PGRT_LIB=ablib/$lib/libpgrt.so; fi
    timeout -k 10 200 python3 tools/frame_timeline.py --reps 25 > gpurun_out/tl_r5zd_$lib.txt 2>&1 || { tail -5 gpurun_out/tl_r5zd_$lib.txt; exit 1; }
    echo "$lib $(head -1 gpurun_out/tl_r5zd_$lib.txt | grep -o '"host_ms_median_timeline_off": [0-9.]*') $(head -1 gpurun_out/tl_r5zd_$lib.txt | grep -o '"device_span_ms_median": [0-9.]*') $(grep -m1 's0 subtree' gpurun_out/tl_r5zd_$lib.txt | cut -c1-140)"
  done
done
