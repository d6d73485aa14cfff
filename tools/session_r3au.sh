#!/bin/bash
# r3au: per-rank share of N-GPU C2 frames (PGRT_EMULATE_RANK=0/N, --dist-path) with the batch-size packet
# budget (default: 64 steps below 4M level-0 rays per call) vs a forced 256-step budget
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r3au
mkdir -p "$OUT"
for N in 4 8; do
  for args in "--steps 20 --warmup 5" "--steps 400"; do
    for c in "" "--cfg packet_budget=256"; do
      v=""
      for r in 1 2 3; do
        PGRT_EMULATE_RANK=0/$N timeout -k 10 200 python3 bench.py --dist-path --no-cpu-baseline --no-roofline $args $c > "$OUT/b.json" 2> "$OUT/b.err" || { tail -5 "$OUT/b.err"; exit 1; }
        v="$v $(python3 -c "import json; d=json.load(open('$OUT/b.json')); print(d['ms_per_step'])")"
      done
      echo "[N=$N $args $c] ms/frame:$v"
    done
  done
done
