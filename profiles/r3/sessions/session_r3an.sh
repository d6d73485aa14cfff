#!/bin/bash
# r3an: L2 warm-up before the deep-level traces (PGRT_WARM_LEVEL = first warmed level, 0 = off):
# parity subset with warming on, then C2 20 / 400 frames (ms/frame / one synchronous frame's ms)
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r3an
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
PGRT_WARM_LEVEL=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "frame_parity or geosphere or full_size" > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
echo "parity (warm 1): $(tail -1 "$OUT/gpu_tests.log")"
for args in "--steps 20 --warmup 5" "--steps 400"; do
  for w in 0 1 3 0 1 3; do
    v=""
    for r in 1 2; do
      PGRT_WARM_LEVEL=$w timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline $args > "$OUT/b.json" 2> "$OUT/b.err" || { tail -5 "$OUT/b.err"; exit 1; }
      v="$v $(python3 -c "import json; d=json.load(open('$OUT/b.json')); print(d['ms_per_step'], d['frame_latency_ms'], sep='/')")"
    done
    echo "[$args] warm $w:$v"
  done
done
