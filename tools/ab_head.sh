#!/bin/bash
# A/B of the working tree's library against ablib/head/libpgrt.so (the last commit's build, made
# with tools/build_variant.sh from `git archive HEAD`): a parity subset, then C2 20 / 400 frames
# (3 runs each, same box) and optional extra bench args (AB_EXTRA="--config C5 --steps 20 --warmup 3").
# usage: tools/ab_head.sh <tag> [pytest -k expression]
set -u
cd "$(dirname "$0")/.."
TAG=$1; K=${2:-"frame_parity or geosphere or full_size"}
OUT=gpurun_out/abh_$TAG
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "$K" > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
echo "parity: $(tail -1 "$OUT/gpu_tests.log")"
for args in "--steps 20 --warmup 5" "--steps 400" ${AB_EXTRA:+"$AB_EXTRA"}; do
  for lib in head new; do
    v=""
    for r in 1 2 3; do
      if [ $lib = head ]; then export PGRT_LIB=ablib/head/libpgrt.so; else unset PGRT_LIB; fi
      timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline $args > "$OUT/b.json" 2> "$OUT/b.err" || { tail -5 "$OUT/b.err"; exit 1; }
      v="$v $(python3 -c "import json; d=json.load(open('$OUT/b.json')); print(d['ms_per_step'])")"
    done
    unset PGRT_LIB
    echo "[$args] $lib ms/frame:$v"
  done
done
