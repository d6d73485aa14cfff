#!/bin/bash
# r5q: which launches run inside the driver's timed calls (kernel trace of the driver-style line;
# calls delimited by k_export_counters) -- AUTO probe launches in the timed region?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kt_r5q -o kt --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/kt_r5q.log 2>&1 || { tail -5 gpurun_out/kt_r5q.log; exit 1; }
f=$(find gpurun_out/kt_r5q -name '*kernel_trace.csv' | head -1)
head -1 "$f"
python3 tools/call_kernels.py "$f" 8 12 > gpurun_out/kt_r5q_calls.txt; grep -c . gpurun_out/kt_r5q_calls.txt; grep -E "trace_pkt.*grid +65536 " gpurun_out/kt_r5q_calls.txt || true; tail -1 gpurun_out/kt_r5q_calls.txt
