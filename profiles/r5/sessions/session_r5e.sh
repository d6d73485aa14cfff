#!/bin/bash
# r5e: host_export modes (config ABI 2) -- GPU suite, then the host-framebuffer A/B: per-slot
# export kernels (32 workgroups, default), per-slot DMA copies of tile runs (2), one copy (-1),
# export kernels for calls in flight too (1); r4 head for reference
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
bash tools/gpu_check.sh tests || exit 1
for r in 1 2; do
  for mode in 0 2 -1 1; do
    timeout -k 10 200 python3 tools/host_fb.py --cfg host_export=$mode --async 8x4 2x4 > gpurun_out/host_r5e_$mode.json 2> gpurun_out/host_r5e_$mode.err || { tail -5 gpurun_out/host_r5e_$mode.err; exit 1; }
    cat gpurun_out/host_r5e_$mode.json
  done
  PGRT_LIB=ablib/r4head/libpgrt.so timeout -k 10 200 python3 tools/host_fb.py --async 8x4 2x4 > gpurun_out/host_r5e_r4.json 2> gpurun_out/host_r5e_r4.err || { tail -5 gpurun_out/host_r5e_r4.err; exit 1; }
  cat gpurun_out/host_r5e_r4.json
done
