#!/bin/bash
# r5d: host-export grid A/B (the export kernel's host stores share every CU's memory pipeline with
# the deep-tile slot: fewer export workgroups -> fewer CUs stalled behind PCIe writes) and the
# async host-output call shape (frames per call x calls in flight)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
for r in 1 2; do
  for lib in base exg8 exg16 exg32 exg64 r4head; do
    if [ $lib = base ]; then unset PGRT_LIB; else export PGRT_LIB=ablib/$lib/libpgrt.so; fi
    timeout -k 10 200 python3 tools/host_fb.py --async 8x4 2x4 2x2 1x4 > gpurun_out/host_r5d_$lib.json 2> gpurun_out/host_r5d_$lib.err || { tail -5 gpurun_out/host_r5d_$lib.err; exit 1; }
    cat gpurun_out/host_r5d_$lib.json
  done
done
