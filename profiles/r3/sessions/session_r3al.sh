#!/bin/bash
# r3al: the whole GPU suite, smoke() and the driver's bench command at the current head
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r3al
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline'].get('frame',{}).get('frac') if isinstance(d['roofline'].get('frame'),dict) else d['roofline'].get('frame'), d.get('frame_latency_ms'))"
