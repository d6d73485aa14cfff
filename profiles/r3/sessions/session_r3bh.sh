#!/bin/bash
# r3bh: one synchronous C2 frame -- bounce levels 1-2 as packets (default) vs 8-lane groups
# (packet_levels=1: only level 0 as packets; groups for queues <= group_max).  Level timings.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r3bh
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
lv() { grep -E '^L[0-9]' "$1" | sed -E 's/^(L[0-9]+): rays +([0-9]+).*trace +([0-9.]+) us shade +([0-9.]+) us.*/\1 \3+\4/' | tr '\n' ' '; }
for rep in 1 2; do
  for v in "default:" "pkt1:packet_levels=1" "pkt1_g4m:packet_levels=1,group_max=4000000" "pkt2:packet_levels=2"; do
    name=${v%%:*}; cfg=${v#*:}
    DIAG_FRAMES=1 DIAG_REPS=9 DIAG_CFG=$cfg timeout -k 10 120 python3 tools/diag.py > "$OUT/d_$name.txt" 2>&1 || { tail -5 "$OUT/d_$name.txt"; exit 1; }
    echo "1 frame $name: total $(python3 -c "import json; d=json.loads(open('$OUT/d_$name.txt').read().splitlines()[1]); print(d['stage_ms']['ms_total'])") | $(lv "$OUT/d_$name.txt")"
  done
done
