#!/bin/bash
# r5zg: the driver's region with the calls' level-0 work ordered (call_order 1: each call's level-0
# trace waits for the previous call's level-0 shade, so the first calls' bounce chains overlap the
# later calls' level 0), at 8 / 5 / 4 frames per call; 5 runs each, same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/ab_r5zg; mkdir -p $OUT
i=0
for A in "" "--cfg call_order=1" "--frames-per-call 5 --cfg call_order=1" "--frames-per-call 4 --cfg call_order=1" "--frames-per-call 4" ""; do
  i=$((i + 1)); v=""
  for r in 1 2 3 4 5; do
    timeout -k 10 180 python3 bench.py --no-cpu-baseline --no-roofline --steps 20 --warmup 5 $A > $OUT/s$i.$r.json 2> $OUT/s$i.err || { tail -5 $OUT/s$i.err; exit 1; }
    v="$v $(python3 -c "import json; print(json.load(open('$OUT/s$i.$r.json'))['ms_per_step'])")"
  done
  echo "[$A] ms/frame:$v"
done
