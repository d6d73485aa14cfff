#!/bin/bash
# r5zk: 8-wide nodes with each slot half's (lo, hi) plane words adjacent -- a group lane loads its
# 8 bytes per axis and takes every plane with one v_perm_b32 (per-lane selectors) -- vs HEAD:
# full GPU suite, synchronous frame latency (4 interleaved runs), driver line / 400 frames / C5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r5zk.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r5zk.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r5zk.log
for rep in 1 2 3 4; do
  for lib in base head; do
    if [ $lib = base ]; then unset PGRT_LIB; else export PGRT_LIB=ablib/$lib/libpgrt.so; fi
    timeout -k 10 200 python3 tools/frame_timeline.py --reps 25 > gpurun_out/tl_r5zk_$lib.txt 2>&1 || { tail -5 gpurun_out/tl_r5zk_$lib.txt; exit 1; }
    echo "$lib $(head -1 gpurun_out/tl_r5zk_$lib.txt | grep -o '"host_ms_median_timeline_off": [0-9.]*') $(head -1 gpurun_out/tl_r5zk_$lib.txt | grep -o '"device_span_ms_median": [0-9.]*') $(grep -m1 's0 subtree' gpurun_out/tl_r5zk_$lib.txt | cut -c1-140)"
  done
done
unset PGRT_LIB
bash tools/ab_matrix.sh r5zk "base ablib/head/libpgrt.so" "--steps 20 --warmup 5" "--steps 400" "--config C5 --steps 10 --warmup 3" || exit 1
