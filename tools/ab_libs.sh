#!/bin/bash
# A/B of library builds / environment knobs: per setting, C2 throughput (bench, default frames
# per call / in flight, 3 runs) and a rocprofv3 kernel trace of the synchronous roofline frames.
# usage: tools/ab_libs.sh <tag> <setting> ...
#   setting = "base" | <path to a libpgrt.so> | "<name>:<ENV=value ...>" (PGRT_LIB=... allowed)
set -u
cd "$(dirname "$0")/.."
TAG=$1; shift
OUT=gpurun_out/ab_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for L in "$@"; do
  envs=""
  if [ "$L" = base ]; then name=base
  elif [[ "$L" == *:* ]]; then name=${L%%:*}; envs=${L#*:}
  else name=$(basename "$(dirname "$L")"); envs="PGRT_LIB=$L"; fi
  for r in 1 2 3; do
    env $envs timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-roofline --steps 960 ${BENCH_ARGS:-} \
      > "$OUT/$name.bench$r.json" 2> "$OUT/$name.err" || { tail -5 "$OUT/$name.err"; exit 1; }
  done
  python3 -c "import json; v=[json.load(open('$OUT/$name.bench%d.json'%r))['ms_per_step'] for r in (1,2,3)]; print('$name ms/frame', v)"
  [ -n "${NO_TRACE:-}" ] && continue
  env $envs timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/$name.kt" -o kt --output-format csv -- \
    python3 bench.py --roofline-only ${BENCH_ARGS:-} > "$OUT/$name.kt.log" 2>&1 || { tail -5 "$OUT/$name.kt.log"; exit 1; }
  f=$(find "$OUT/$name.kt" -name "*kernel_trace.csv" | head -1)
  python3 tools/kernel_summary.py "$f" > "$OUT/$name.summary.txt" 2>&1
  python3 tools/call_seq.py "$f"
done
