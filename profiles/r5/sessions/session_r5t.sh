#!/bin/bash
# r5t: the level-0 shade of 1-spp batches split around the allocation as well (shade_eval_a / _b) vs
# l0nosplit (the previous head: bounce levels split only) -- parity subset, the driver line and 400 frames (3 runs
# each), steady per-kernel breakdowns
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "frame_parity or full_size or golden or batched or subtree or path or geosphere or lights" > gpurun_out/gpu_tests_r5t.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r5t.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r5t.log
bash tools/ab_matrix.sh r5t "base ablib/l0nosplit/libpgrt.so" "--steps 20 --warmup 5" "--steps 400" || exit 1
for lib in base l0nosplit; do
  if [ $lib = base ]; then unset PGRT_LIB; else export PGRT_LIB=ablib/$lib/libpgrt.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kt_r5t_$lib -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --no-roofline --steps 400 > gpurun_out/kt_r5t_$lib.log 2>&1 || { tail -5 gpurun_out/kt_r5t_$lib.log; exit 1; }
  python3 tools/throughput_breakdown.py "$(find gpurun_out/kt_r5t_$lib -name '*kernel_trace.csv' | head -1)" 8 > gpurun_out/kt_r5t_$lib.txt 2>&1; head -8 gpurun_out/kt_r5t_$lib.txt | sed "s/^/$lib  /"
done
