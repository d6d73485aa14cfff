#!/bin/bash
# r5v: (1) call sizes of the driver's 20-frame region (8+8+4 default; the 4-frame call first; 7+7+6;
# 5x4; 10+10) -- 5 runs each, same box, after the two-part shades;
# (2) opaque_color's loads side by side vs HEAD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/ab_r5v; mkdir -p $OUT
i=0
for A in "" "--remainder-first" "--frames-per-call 7" "--frames-per-call 7 --remainder-first" "--frames-per-call 5" "--frames-per-call 10" ""; do
  i=$((i + 1)); v=""
  for r in 1 2 3 4 5; do
    timeout -k 10 180 python3 bench.py --no-cpu-baseline --no-roofline --steps 20 --warmup 5 $A > $OUT/s$i.$r.json 2> $OUT/s$i.err || { tail -5 $OUT/s$i.err; exit 1; }
    v="$v $(python3 -c "import json; print(json.load(open('$OUT/s$i.$r.json'))['ms_per_step'])")"
  done
  echo "[$A] ms/frame:$v"
done
# the shadow verdict and the Phong term loaded together in opaque_color (finish / combine) vs HEAD
bash tools/ab_matrix.sh r5v2 "base ablib/head/libpgrt.so" "--steps 20 --warmup 5" "--steps 400" || exit 1
