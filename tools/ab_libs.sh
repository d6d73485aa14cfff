#!/bin/bash
# A/B of library builds: per build, C2 throughput (bench, default frames per call / in flight,
# 3 runs) and a rocprofv3 kernel trace of the synchronous roofline frames (per-launch durations).
# usage: tools/ab_libs.sh <tag> <lib1> <lib2> ...   ("base" = the in-tree build)
set -u
cd "$(dirname "$0")/.."
TAG=$1; shift
OUT=gpurun_out/ab_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for L in "$@"; do
  name=$(basename "$(dirname "$L")"); [ "$L" = base ] && name=base
  lib=""; [ "$L" != base ] && lib="$L"
  for r in 1 2 3; do
    PGRT_LIB=$lib timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-roofline --steps 960 ${BENCH_ARGS:-} \
      > "$OUT/$name.bench$r.json" 2> "$OUT/$name.err" || { tail -5 "$OUT/$name.err"; exit 1; }
  done
  python3 -c "import json; v=[json.load(open('$OUT/$name.bench%d.json'%r))['ms_per_step'] for r in (1,2,3)]; print('$name ms/frame', v)"
  PGRT_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/$name.kt" -o kt --output-format csv -- \
    python3 bench.py --roofline-only ${BENCH_ARGS:-} > "$OUT/$name.kt.log" 2>&1 || { tail -5 "$OUT/$name.kt.log"; exit 1; }
  f=$(find "$OUT/$name.kt" -name "*kernel_trace.csv" | head -1)
  python3 tools/kernel_summary.py "$f" > "$OUT/$name.summary.txt" 2>&1
  grep -A30 "per-launch" "$OUT/$name.summary.txt" | head -24
done
