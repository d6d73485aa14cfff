#!/bin/bash
# Every BASELINE config through bench.py on one GPU (run on the GPU box via gpurun); one JSON
# line per config into gpurun_out/bench_<tag>.txt.  usage: tools/round_bench.sh <tag>
set -u
cd "$(dirname "$0")/.."
TAG=${1:-r1}
OUT=gpurun_out/bench_$TAG.txt
: > "$OUT"
echo "=== C2 driver-style (--steps 20 --warmup 5)" >&2
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > "gpurun_out/bench_${TAG}_C2_k20.json" 2> "gpurun_out/bench_${TAG}_C2_k20.err" || exit $?
for cfg in C2 C3 C4 C5; do
    extra=""
    steps=""
    [ $cfg = C3 ] && steps="--steps 20 --warmup 3"
    [ $cfg = C4 ] && steps="--steps 6 --warmup 2"
    [ $cfg = C5 ] && steps="--steps 20 --warmup 3"
    echo "=== $cfg" >&2
    timeout -k 10 400 python3 bench.py --config $cfg $extra $steps >> "$OUT" 2> "gpurun_out/bench_${TAG}_$cfg.err"
    rc=$?
    if [ $rc -ne 0 ]; then echo "$cfg rc=$rc" >&2; tail -5 "gpurun_out/bench_${TAG}_$cfg.err" >&2; exit $rc; fi
done
cat "$OUT"
