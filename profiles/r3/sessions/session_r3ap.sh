#!/bin/bash
# r3ap: kernel stats of the C5 line (20 frames) at the current head
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r3ap
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o c5 --output-format csv -- python3 bench.py --config C5 --steps 20 --warmup 3 --no-roofline --no-cpu-baseline > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
grep '"metric"' "$OUT/bench.log" | cut -c1-200
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/c5_kernel_stats.csv" \;
