#!/bin/bash
# r3bf: child prefetch in the one-lane kernel (k_trace_pf; PGRT_TRACE_PF = the largest expected
# queue that takes it, 0 = never).  Parity subset with it on for every one-lane launch, level
# timings (1 frame: default 8-lane groups vs one lane vs one lane + prefetch; 8 frames), then the
# C2 driver line and one synchronous frame.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r3bf
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
BIG=1073741824
PGRT_TRACE_PF=$BIG timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "frame_parity or geosphere or full_size or packet_levels or layouts or maximum_depth or closest_hit" > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
echo "parity (prefetch on): $(tail -1 "$OUT/gpu_tests.log")"
lv() { grep -E '^L[0-9]' "$1" | sed -E 's/^(L[0-9]+): rays +([0-9]+).*trace +([0-9.]+) us.*/\1 \3/' | tr '\n' ' '; }
for rep in 1 2; do
  for v in "default:0:" "onelane:0:group_max=-1" "onelane_pf:$BIG:group_max=-1"; do
    name=${v%%:*}; rest=${v#*:}; pf=${rest%%:*}; cfg=${rest#*:}
    PGRT_TRACE_PF=$pf DIAG_FRAMES=1 DIAG_REPS=9 DIAG_CFG=$cfg timeout -k 10 120 python3 tools/diag.py > "$OUT/d1_$name.txt" 2>&1 || { tail -5 "$OUT/d1_$name.txt"; exit 1; }
    echo "1 frame $name: $(lv "$OUT/d1_$name.txt")"
  done
  for pf in 0 $BIG; do
    PGRT_TRACE_PF=$pf DIAG_FRAMES=8 DIAG_REPS=5 timeout -k 10 120 python3 tools/diag.py > "$OUT/d8_$pf.txt" 2>&1 || { tail -5 "$OUT/d8_$pf.txt"; exit 1; }
    echo "8 frames default, pf $pf: $(lv "$OUT/d8_$pf.txt")"
  done
done
for args in "" "--group-max -1"; do
  for pf in 0 $BIG 0 $BIG; do
    PGRT_TRACE_PF=$pf timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline --steps 20 --warmup 5 $args > "$OUT/b.json" 2> "$OUT/b.err" || { tail -5 "$OUT/b.err"; exit 1; }
    echo "[driver line $args] pf $pf: $(python3 -c "import json; d=json.load(open('$OUT/b.json')); print(d['ms_per_step'], d['frame_latency_ms'], sep='/')")"
  done
done
