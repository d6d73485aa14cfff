#!/bin/bash
# Same-box A/B of several settings on one bench line, runs interleaved (A B C A B C ...), every
# run a fresh process.  A setting is "base", a library path (ablib/<name>/libpgrt.so), or
# "<name>=<extra bench args>" (e.g. "sub3=--cfg subtree_level=3"), or "<lib>@<extra args>".
# usage: RUNS=3 ARGS="--steps 20 --warmup 5" tools/ab_multi.sh <tag> <setting> ...
set -u
cd "$(dirname "$0")/.."
TAG=$1; shift
RUNS=${RUNS:-3}
ARGS=${ARGS:-"--steps 20 --warmup 5"}
OUT=gpurun_out/abm_$TAG
mkdir -p "$OUT"
for r in $(seq 1 "$RUNS"); do
  for S in "$@"; do
    lib=""; extra=""
    if [ "$S" = base ]; then name=base
    elif [[ "$S" == *@* ]]; then lib=${S%%@*}; extra=${S#*@}; name=$(basename "$(dirname "$lib")")+$(echo "$extra" | tr -d ' -')
    elif [[ "$S" == *=* ]]; then name=${S%%=*}; extra=${S#*=}
    else lib=$S; name=$(basename "$(dirname "$S")"); fi
    if [ -n "$lib" ]; then export PGRT_LIB=$lib; else unset PGRT_LIB; fi
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline $ARGS $extra > "$OUT/b.json" 2> "$OUT/b.err" || { tail -5 "$OUT/b.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b.json')); print('%-28s' % '$name', '[$ARGS]', d['ms_per_step'], 'latency', d.get('frame_latency_ms'))" | tee -a "$OUT/summary.txt"
  done
done
unset PGRT_LIB
