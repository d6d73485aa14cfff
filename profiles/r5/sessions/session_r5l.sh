#!/bin/bash
# r5l: NUMA placement of the page-locked framebuffer vs device-to-host bandwidth (tools/numa_probe.hip),
# twice, plus the D2H probe for comparison
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
timeout -k 10 120 ./build/numa_probe > gpurun_out/numa_probe_r5l_1.txt 2>&1; rc=$?; cat gpurun_out/numa_probe_r5l_1.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./build/numa_probe > gpurun_out/numa_probe_r5l_2.txt 2>&1; rc=$?; cat gpurun_out/numa_probe_r5l_2.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./build/d2h_probe > gpurun_out/d2h_probe_r5l.txt 2>&1 || exit 1
grep -E "1 stream\(s\)|grid 64" gpurun_out/d2h_probe_r5l.txt | head -3
