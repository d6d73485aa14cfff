#!/bin/bash
# r5zc: the synchronous frame's level-2 subtree launch (~122k rays, 15k waves of 8 lanes: ~4 rounds
# of the 4096 resident) -- 4 lanes per ray from 40k rays (g4at40k), the 5-wave build (w5) vs base;
# host ms (median of 25, timeline off), 4 interleaved runs each; subtree parity
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for lib in g4at40k w5; do
  PGRT_LIB=ablib/$lib/libpgrt.so timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "subtree or frame_parity" > gpurun_out/gpu_tests_r5zc_$lib.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r5zc_$lib.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/gpu_tests_r5zc_$lib.log)"
done
for rep in 1 2 3 4; do
  for lib in base g4at40k w5; do
    if [ $lib = base ]; then unset PGRT_LIB; else export PGRT_LIB=ablib/$lib/libpgrt.so; fi
    timeout -k 10 200 python3 tools/frame_timeline.py --reps 25 > gpurun_out/tl_r5zc_$lib.txt 2>&1 || { tail -5 gpurun_out/tl_r5zc_$lib.txt; exit 1; }
    echo "$lib $(head -1 gpurun_out/tl_r5zc_$lib.txt | grep -o '"host_ms_median_timeline_off": [0-9.]*') $(head -1 gpurun_out/tl_r5zc_$lib.txt | grep -o '"device_span_ms_median": [0-9.]*') $(grep -m1 's0 subtree' gpurun_out/tl_r5zc_$lib.txt | cut -c1-140)"
  done
done
