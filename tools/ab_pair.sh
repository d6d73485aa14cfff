#!/bin/bash
# Same-box A/B of two library builds on the driver's line and the steady line, runs interleaved
# (A B A B ...), every run a fresh process.
# usage: tools/ab_pair.sh <tag> <libA|base> <libB|base> [runs] [bench args...]
set -u
cd "$(dirname "$0")/.."
TAG=$1; A=$2; B=$3; RUNS=${4:-3}; shift 4 2>/dev/null || shift $#
ARGS=${*:-"--steps 20 --warmup 5"}
OUT=gpurun_out/abp_$TAG
mkdir -p "$OUT"
for r in $(seq 1 "$RUNS"); do
  for L in "$A" "$B"; do
    if [ "$L" = base ]; then unset PGRT_LIB; name=base; else export PGRT_LIB=$L; name=$(basename "$(dirname "$L")"); fi
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline $ARGS > "$OUT/b.json" 2> "$OUT/b.err" || { tail -5 "$OUT/b.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b.json')); print('$name', '[$ARGS]', d['ms_per_step'], 'latency', d['frame_latency_ms'])" | tee -a "$OUT/summary.txt"
  done
done
unset PGRT_LIB
