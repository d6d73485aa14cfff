#!/bin/bash
# r3bi: one-frame batches trace their bounce levels with 8 / 4-lane groups instead of packets
# (default now; PGRT_SMALL_GROUPS=0 restores packets).  Whole GPU suite with the new default,
# then the C2 driver line / one synchronous frame and the path tracer, A/B.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r3bi
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
echo "GPU suite (small-batch groups): $(tail -1 "$OUT/gpu_tests.log")"
for sg in 0 1 0 1 0 1; do
  PGRT_SMALL_GROUPS=$sg timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline --steps 20 --warmup 5 > "$OUT/b.json" 2> "$OUT/b.err" || { tail -5 "$OUT/b.err"; exit 1; }
  echo "[driver line] small groups $sg: $(python3 -c "import json; d=json.load(open('$OUT/b.json')); print(d['ms_per_step'], d['frame_latency_ms'], sep='/')")"
done
for sg in 0 1; do
  PGRT_SMALL_GROUPS=$sg timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline --mode path --steps 40 --warmup 8 > "$OUT/p.json" 2> "$OUT/p.err" || { tail -5 "$OUT/p.err"; exit 1; }
  echo "[path] small groups $sg: $(python3 -c "import json; d=json.load(open('$OUT/p.json')); print(d['ms_per_step'], d.get('frame_latency_ms'), sep='/')")"
done
