#!/bin/bash
# r3bg: fused resolve of 1-spp pending pixels (k_resolve_pending, PGRT_FUSED_RESOLVE=1): one launch
# walks each pixel's ray tree instead of max_level - 1 combines + the finish.  Parity subset with
# it on, the combine stage at 1 and 8 frames per call, then the C2 driver line and one frame.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r3bg
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
PGRT_FUSED_RESOLVE=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "frame_parity or geosphere or full_size or packet_levels or maximum_depth or distinct or batched" > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
echo "parity (fused resolve): $(tail -1 "$OUT/gpu_tests.log")"
for rep in 1 2; do
  for fr in 0 1; do
    for F in 1 8; do
      PGRT_FUSED_RESOLVE=$fr DIAG_FRAMES=$F DIAG_REPS=9 timeout -k 10 120 python3 tools/diag.py > "$OUT/d_${fr}_$F.txt" 2>&1 || { tail -5 "$OUT/d_${fr}_$F.txt"; exit 1; }
      echo "fused $fr, $F frames: $(python3 -c "import json; d=json.loads(open('$OUT/d_${fr}_$F.txt').read().splitlines()[1]); print(d['stage_ms']['ms_combine'], d['stage_ms']['ms_total'])")"
    done
  done
done
for fr in 0 1 0 1 0 1; do
  PGRT_FUSED_RESOLVE=$fr timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline --steps 20 --warmup 5 > "$OUT/b.json" 2> "$OUT/b.err" || { tail -5 "$OUT/b.err"; exit 1; }
  echo "[driver line] fused $fr: $(python3 -c "import json; d=json.load(open('$OUT/b.json')); print(d['ms_per_step'], d['frame_latency_ms'], sep='/')")"
done
