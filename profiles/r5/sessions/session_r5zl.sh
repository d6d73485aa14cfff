#!/bin/bash
# r5zl: the subtree launch fetches the next 8-wide node during each triangle phase (trace8_group PF)
# vs without (nopf) -- full GPU suite, synchronous frame latency (4 interleaved runs), the driver line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r5zl.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r5zl.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r5zl.log
for rep in 1 2 3 4; do
  for lib in base nopf; do
    if [ $lib = base ]; then unset PGRT_LIB; else export PGRT_LIB=ablib/$lib/libpgrt.so; fi
    timeout -k 10 200 python3 tools/frame_timeline.py --reps 25 > gpurun_out/tl_r5zl_$lib.txt 2>&1 || { tail -5 gpurun_out/tl_r5zl_$lib.txt; exit 1; }
    echo "$lib $(head -1 gpurun_out/tl_r5zl_$lib.txt | grep -o '"host_ms_median_timeline_off": [0-9.]*') $(head -1 gpurun_out/tl_r5zl_$lib.txt | grep -o '"device_span_ms_median": [0-9.]*') $(grep -m1 's0 subtree' gpurun_out/tl_r5zl_$lib.txt | cut -c1-140)"
  done
done
unset PGRT_LIB
bash tools/ab_matrix.sh r5zl "base ablib/nopf/libpgrt.so" "--steps 20 --warmup 5" || exit 1
