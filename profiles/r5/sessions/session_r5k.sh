#!/bin/bash
# r5k: asynchronous host frames -- one DMA copy per call (default) vs the XCD-0-confined export
# kernel (host_export=1), with the box's D2H probe (SDMA vs blit kernel) beside them
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 120 ./build/d2h_probe > gpurun_out/d2h_probe_r5k.txt 2>&1 || exit 1
grep -E "1 stream\(s\)|grid 64|half" gpurun_out/d2h_probe_r5k.txt | head -4
for rep in 1 2; do
  for c in host_export=0 host_export=1 host_export=-1; do
    timeout -k 10 200 python3 tools/host_fb.py --cfg $c --async 8x4 2x4 1x4 > gpurun_out/host_r5k_${c}_$rep.json 2>&1 || { tail -5 gpurun_out/host_r5k_${c}_$rep.json; exit 1; }
    cat gpurun_out/host_r5k_${c}_$rep.json
  done
done
