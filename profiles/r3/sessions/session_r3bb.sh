#!/bin/bash
# r3bb: lane refill (PGRT_REFILL) with larger grids (PGRT_REFILL_GRID x resident blocks): is the
# r3ba slowdown the resident-sized grid?  Level timings at 8 frames per call, levels >= 1 one lane per ray.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r3bb
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
for rg in 0:1 16:1 16:3 16:100 4:100 0:1; do
  r=${rg%%:*}; g=${rg##*:}
  PGRT_REFILL=$r PGRT_REFILL_GRID=$g DIAG_FRAMES=8 DIAG_REPS=5 DIAG_CFG=packet_levels=1,group_max=-1 timeout -k 10 120 python3 tools/diag.py > "$OUT/diag_${r}_$g.txt" 2>&1 || { tail -5 "$OUT/diag_${r}_$g.txt"; exit 1; }
  echo "refill $r grid x$g: $(grep -E '^L[0-9]' "$OUT/diag_${r}_$g.txt" | sed -E 's/^(L[0-9]+): rays +([0-9]+).*trace +([0-9.]+) us.*/\1 \3/' | tr '\n' ' ')"
done
