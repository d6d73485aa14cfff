#!/bin/bash
# r5u: the synchronous frame's level-3 subtree launch -- its ~5300 working waves exceed the 4096
# resident at 4 waves per SIMD (101 VGPRs); variants: 4 lanes per ray (half the waves: all resident)
# and a 5-wave build (96 VGPRs, 6 spilled) -- device timeline of the synchronous frame, 3 runs each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "subtree" > gpurun_out/gpu_tests_r5u.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r5u.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r5u.log
for rep in 1 2 3; do
  for lib in base sub_g4 sub_w5; do
    if [ $lib = base ]; then unset PGRT_LIB; else export PGRT_LIB=ablib/$lib/libpgrt.so; fi
    timeout -k 10 300 python3 tools/frame_timeline.py --out gpurun_out/tl_r5u_${lib}_$rep.json > gpurun_out/tl_r5u_${lib}_$rep.txt 2>&1 || { tail -5 gpurun_out/tl_r5u_${lib}_$rep.txt; exit 1; }
    echo "$lib $rep $(head -1 gpurun_out/tl_r5u_${lib}_$rep.txt | grep -o '"host_ms_median_timeline_off": [0-9.]*') $(grep -m1 's0 subtree' gpurun_out/tl_r5u_${lib}_$rep.txt | tail -1 | cut -c1-120)"
    grep -m1 "s0 export" gpurun_out/tl_r5u_${lib}_$rep.txt | cut -c1-40
  done
done
