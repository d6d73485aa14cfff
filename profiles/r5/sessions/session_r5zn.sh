#!/bin/bash
# r5zn: a call in flight's host export kernel on a high-priority side stream (base) vs on the call's
# own stream (lopri) vs high priority with 64 copying workgroups (hipri64) -- host parity tests,
# tools/host_fb.py (8x4 / 2x4 calls in flight, synchronous frame), 3 interleaved runs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "host or batched" > gpurun_out/gpu_tests_r5zn.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r5zn.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r5zn.log
timeout -k 10 120 ./build/d2h_probe > gpurun_out/d2h_probe_r5zn.txt 2>&1 || exit 1
grep -E "1 stream\(s\)|grid 64" gpurun_out/d2h_probe_r5zn.txt | head -2
for rep in 1 2 3; do
  for lib in base lopri hipri64; do
    if [ $lib = base ]; then unset PGRT_LIB; else export PGRT_LIB=ablib/$lib/libpgrt.so; fi
    timeout -k 10 300 python3 tools/host_fb.py --reps 10 --async 8x4 2x4 > gpurun_out/host_r5zn_$lib.json 2>&1 || { tail -5 gpurun_out/host_r5zn_$lib.json; exit 1; }
    echo "$lib $(cat gpurun_out/host_r5zn_$lib.json)"
  done
done
