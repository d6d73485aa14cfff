#!/bin/bash
# r5c: host framebuffer -- D2H probe (blit grid sizes), the device timeline of synchronous and
# asynchronous frames into page-locked host memory, and a same-box A/B of bench.py's host figures
# against the r4 head's library (SDMA copies)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./build/d2h_probe > gpurun_out/d2h_probe_r5c.txt 2>&1 || { tail -5 gpurun_out/d2h_probe_r5c.txt; exit 1; }
grep -A20 "pass 1" gpurun_out/d2h_probe_r5c.txt
timeout -k 10 300 python3 tools/frame_timeline.py --host --reps 9 --out gpurun_out/timeline_r5c.json > gpurun_out/timeline_r5c.txt 2>&1 || { tail -5 gpurun_out/timeline_r5c.txt; exit 1; }
grep -E "^(sync|sync_host|async_host|r20) " gpurun_out/timeline_r5c.txt
for r in 1 2; do
  for lib in r4head new; do
    if [ $lib = r4head ]; then export PGRT_LIB=ablib/r4head/libpgrt.so; else unset PGRT_LIB; fi
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_r5c_$lib.json 2> gpurun_out/ab_r5c_$lib.err || { tail -5 gpurun_out/ab_r5c_$lib.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_r5c_$lib.json')); h=d['host_framebuffer']; print('$lib', d['ms_per_step'], d['frame_latency_ms'], 'host sync', h['ms_per_frame_sync_median'], 'async', h['ms_per_frame_async'], h['pcie_d2h_gbs'])"
  done
done
unset PGRT_LIB
