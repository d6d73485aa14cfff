#!/bin/bash
# r3ba: lane refill for the one-lane kernel (k_trace_rf, PGRT_REFILL = idle lanes that trigger a
# refill, 0 = lockstep k_trace).  Parity subset with refill on (shadow queues and, with packets
# and groups off, every bounce level go through it), level timings at 8 frames per call with
# levels >= 1 one lane per ray, then the C2 driver line per setting.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r3ba
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
PGRT_REFILL=16 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "frame_parity or geosphere or full_size or packet_levels or layouts or maximum_depth" > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
echo "parity (refill 16): $(tail -1 "$OUT/gpu_tests.log")"
for r in 0 8 16 32 0; do
  PGRT_REFILL=$r DIAG_FRAMES=8 DIAG_REPS=5 DIAG_CFG=packet_levels=1,group_max=-1 timeout -k 10 120 python3 tools/diag.py > "$OUT/diag_$r.txt" 2>&1 || { tail -5 "$OUT/diag_$r.txt"; exit 1; }
  echo "refill $r (one lane, levels >= 1):"; grep -E "^L[0-9]" "$OUT/diag_$r.txt" | sed -E 's/^(L[0-9]+): rays +([0-9]+).*trace +([0-9.]+) us.*/  \1 rays \2 trace \3 us/'
done
for args in "" "--packet-levels 1 --group-max -1"; do
  for r in 0 16 0 16; do
    PGRT_REFILL=$r timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline --steps 20 --warmup 5 $args > "$OUT/b.json" 2> "$OUT/b.err" || { tail -5 "$OUT/b.err"; exit 1; }
    echo "[$args] refill $r: $(python3 -c "import json; d=json.load(open('$OUT/b.json')); print(d['ms_per_step'], d['frame_latency_ms'], sep='/')")"
  done
done
