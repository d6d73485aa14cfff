#!/bin/bash
# r5i: pipelined level-0 shade (k_shade_l0p: the next ray's attribute / texel loads behind the
# block's allocation atomic) -- parity subset, then same-box A/B vs k_shade (l0base) and the 5-wave
# build: the driver's line and 400 frames (3 runs each), and the steady per-kernel breakdown of each
# library (kernel trace only); host export workgroups 48 / 64 on XCD 0
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "frame_parity or full_size or golden or batched or subtree or host_framebuffer" > gpurun_out/gpu_tests_r5i.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r5i.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r5i.log
bash tools/ab_matrix.sh r5i "base ablib/l0base/libpgrt.so ablib/l0p5/libpgrt.so" "--steps 20 --warmup 5" "--steps 400" || exit 1
for lib in base l0base l0p5; do
  if [ $lib = base ]; then unset PGRT_LIB; else export PGRT_LIB=ablib/$lib/libpgrt.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kt_r5i_$lib -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --no-roofline --steps 400 > gpurun_out/kt_r5i_$lib.log 2>&1 || { tail -5 gpurun_out/kt_r5i_$lib.log; exit 1; }
  python3 tools/throughput_breakdown.py "$(find gpurun_out/kt_r5i_$lib -name '*kernel_trace.csv' | head -1)" 8 | head -8 | sed "s/^/$lib  /"
done
unset PGRT_LIB
for lib in xwg48 xwg64; do
  PGRT_LIB=ablib/$lib/libpgrt.so timeout -k 10 200 python3 tools/host_fb.py --async > gpurun_out/host_r5i_$lib.json 2>&1 || exit 1
  cat gpurun_out/host_r5i_$lib.json
done
timeout -k 10 200 python3 tools/host_fb.py --async > gpurun_out/host_r5i_base.json 2>&1 && cat gpurun_out/host_r5i_base.json
