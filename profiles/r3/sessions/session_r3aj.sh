#!/bin/bash
# r3aj: resume-grid sizing for unknown deferral counts -- parity subset, then head vs new on the
# C5 roofline-only run (first packet frames), C5 / path / C2 lines (3 runs each, same box)
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r3aj
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "budget or c5 or path or frame_parity or geosphere" > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
echo "parity: $(tail -1 "$OUT/gpu_tests.log")"
field() { python3 -c "import json,sys; d=json.load(open('$OUT/b.json')); print(eval(sys.argv[1]))" "$1"; }
for args in "--config C5 --roofline-only" "--config C5 --steps 40 --warmup 3 --no-roofline" "--mode path --steps 100 --no-roofline" \
            "--steps 20 --warmup 5 --no-roofline" "--steps 400 --no-roofline"; do
  for lib in head new; do
    v=""
    for r in 1 2 3; do
      if [ $lib = head ]; then export PGRT_LIB=ablib/head/libpgrt.so; else unset PGRT_LIB; fi
      timeout -k 10 300 python3 bench.py --no-cpu-baseline $args > "$OUT/b.json" 2> "$OUT/b.err" || { tail -5 "$OUT/b.err"; exit 1; }
      case "$args" in
        *roofline-only*) v="$v $(field "d['roofline']['trace_ms_per_frame']")";;
        *) v="$v $(field "d['ms_per_step']")";;
      esac
    done
    unset PGRT_LIB
    echo "[$args] $lib:$v"
  done
done
