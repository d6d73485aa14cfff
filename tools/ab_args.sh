#!/bin/bash
# A/B of bench.py argument sets (same library): per setting, 3 runs of the C2 (or BENCH_CONFIG)
# throughput line, ms/frame printed per setting.
# usage: tools/ab_args.sh <tag> "<args 1>" "<args 2>" ...
set -u
cd "$(dirname "$0")/.."
TAG=$1; shift
OUT=gpurun_out/ab_$TAG
mkdir -p "$OUT"
i=0
for A in "$@"; do
  i=$((i + 1))
  for r in 1 2 3; do
    timeout -k 10 180 python3 bench.py --config ${BENCH_CONFIG:-C2} --no-cpu-baseline --no-roofline $A \
      > "$OUT/s$i.bench$r.json" 2> "$OUT/s$i.err" || { tail -5 "$OUT/s$i.err"; exit 1; }
  done
  python3 -c "import json; v=[json.load(open('$OUT/s$i.bench%d.json'%r))['ms_per_step'] for r in (1,2,3)]; print('[$A] ms/frame', v)"
done
