#!/bin/bash
# r3am: kernel stats of the steady C2 line (200 frames) at the current head
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r3am
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o steady --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-roofline --no-cpu-baseline > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-300
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/steady_kernel_stats.csv" \;
ls "$OUT"
