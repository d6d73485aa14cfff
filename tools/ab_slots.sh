#!/bin/bash
# A/B of pipeline slot counts / stagger on the C2 bench (each setting its own process)
cd "$(dirname "$0")/.."
for cfg in "$@"; do
  echo "### $cfg"
  env $cfg timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-roofline $BENCH_ARGS | cut -c1-200 || exit 1
done
