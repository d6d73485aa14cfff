#!/bin/bash
# r5zj: work-sharing subtree, one round of resident blocks (4 per CU), home rays interleaved over the blocks (base) / 8 blocks per CU (ws8) / contiguous home rays (wscontig)
# vs one group per tree (nows) -- subtree parity, host ms of a synchronous frame (4 interleaved runs) with
# the slot-0 subtree launch
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "subtree or frame_parity or full_size" > gpurun_out/gpu_tests_r5zj.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r5zj.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r5zj.log
for rep in 1 2 3 4; do
  for lib in base ws8 wscontig nows; do
    if [ $lib = base ]; then unset PGRT_LIB; else export PGRT_LIB=ablib/$lib/libpgrt.so; fi
    timeout -k 10 200 python3 tools/frame_timeline.py --reps 25 > gpurun_out/tl_r5zj_$lib.txt 2>&1 || { tail -5 gpurun_out/tl_r5zj_$lib.txt; exit 1; }
    echo "$lib $(head -1 gpurun_out/tl_r5zj_$lib.txt | grep -o '"host_ms_median_timeline_off": [0-9.]*') $(head -1 gpurun_out/tl_r5zj_$lib.txt | grep -o '"device_span_ms_median": [0-9.]*') $(grep -m1 's0 subtree' gpurun_out/tl_r5zj_$lib.txt | cut -c1-140)"
  done
done
