#!/bin/bash
# r5h: synchronous host frame -- export kernel confined to XCD 0 (blockIdx % 8 == 0: its PCIe
# stores then queue in one XCD's L2 / fabric port) vs spread (default grid 32), plus grid 16; and the
# async host path per call: DMA copy (default) vs export kernels (host_export=1) on this box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
timeout -k 10 120 ./build/d2h_probe > gpurun_out/d2h_probe_r5h.txt 2>&1 || exit 1
grep -A3 "pass 1" gpurun_out/d2h_probe_r5h.txt
bash tools/gpu_check.sh tests smoke || exit 1
for r in 1 2; do
  for lib in base xcd256 xcd64 g16; do
    if [ $lib = base ]; then unset PGRT_LIB; else export PGRT_LIB=ablib/$lib/libpgrt.so; fi
    timeout -k 10 200 python3 tools/host_fb.py --async > gpurun_out/host_r5h_$lib.json 2> gpurun_out/host_r5h_$lib.err || { tail -5 gpurun_out/host_r5h_$lib.err; exit 1; }
    cat gpurun_out/host_r5h_$lib.json
  done
  unset PGRT_LIB
  timeout -k 10 200 python3 tools/host_fb.py --cfg host_export=1 --async 8x4 2x4 > gpurun_out/host_r5h_k.json 2> gpurun_out/host_r5h_k.err || exit 1
  cat gpurun_out/host_r5h_k.json
  timeout -k 10 200 python3 tools/host_fb.py --async 8x4 2x4 > gpurun_out/host_r5h_c.json 2> gpurun_out/host_r5h_c.err || exit 1
  cat gpurun_out/host_r5h_c.json
done
