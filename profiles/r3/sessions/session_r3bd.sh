#!/bin/bash
# r3bd: the one-lane kernel with the short LDS stack (PGRT_TRACE_SPILL=1: 16 entries in LDS, the
# rest in global memory; 16 KB per block instead of (depth + 2) KB -> more blocks per CU).
# Parity subset with it on, level timings at 8 frames per call (levels >= 1 one lane per ray),
# then the C2 driver line (default config: levels 3-5 and the shadow queue are one-lane).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r3bd
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
PGRT_TRACE_SPILL=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "frame_parity or geosphere or full_size or packet_levels or layouts or maximum_depth" > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
echo "parity (spill 1): $(tail -1 "$OUT/gpu_tests.log")"
for sp in 0 1 0 1; do
  PGRT_TRACE_SPILL=$sp DIAG_FRAMES=8 DIAG_REPS=5 DIAG_CFG=packet_levels=1,group_max=-1 timeout -k 10 120 python3 tools/diag.py > "$OUT/diag_$sp.txt" 2>&1 || { tail -5 "$OUT/diag_$sp.txt"; exit 1; }
  echo "spill $sp (8 frames, one lane, levels >= 1): $(grep -E '^L[0-9]' "$OUT/diag_$sp.txt" | sed -E 's/^(L[0-9]+): rays +([0-9]+).*trace +([0-9.]+) us.*/\1 \3/' | tr '\n' ' ')"
done
for sp in 0 1; do
  PGRT_TRACE_SPILL=$sp DIAG_FRAMES=1 DIAG_REPS=9 timeout -k 10 120 python3 tools/diag.py > "$OUT/diag1_$sp.txt" 2>&1 || { tail -5 "$OUT/diag1_$sp.txt"; exit 1; }
  echo "spill $sp (1 frame, default): $(grep -E '^L[0-9]' "$OUT/diag1_$sp.txt" | sed -E 's/^(L[0-9]+): rays +([0-9]+).*trace +([0-9.]+) us.*/\1 \3/' | tr '\n' ' ')"
done
for sp in 0 1 0 1 0 1; do
  PGRT_TRACE_SPILL=$sp timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline --steps 20 --warmup 5 > "$OUT/b.json" 2> "$OUT/b.err" || { tail -5 "$OUT/b.err"; exit 1; }
  echo "[driver line] spill $sp: $(python3 -c "import json; d=json.load(open('$OUT/b.json')); print(d['ms_per_step'], d['frame_latency_ms'], sep='/')")"
done
