#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel trace only -- never combined with
# sys/runtime tracing) over a short bench run; summarise with tools/pmc_summary.py.
# usage: tools/pmc.sh <tag> "<group1>" "<group2>" ...   (a group = space-separated counters)
set -u
cd "$(dirname "$0")/.."
TAG=$1
shift
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "$@"; do
    i=$((i + 1))
    echo "=== pass $i: $grp"
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o p$i --output-format csv -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline ${BENCH_ARGS:-} > "$OUT/p$i.log" 2>&1
    rc=$?
    echo "=== pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt" 2>&1
cat "$OUT/summary.txt"
