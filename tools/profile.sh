#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box via gpurun):
#   1. kernel trace + stats (per-kernel average durations)
#   2./3. PMC passes, one counter group each (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass)
# Usage: tools/profile.sh <tag> [bench args...]
set -u
cd "$(dirname "$0")/.."
TAG=${1:-r1}
shift || true
ARGS=${*:-"--roofline-only"}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name limit rocprof-args...
    local name=$1 limit=$2
    shift 2
    echo "=== $name"
    timeout -k 10 "$limit" rocprofv3 "$@" -d "$OUT/$name" -o "$name" --output-format csv -- \
        python3 bench.py $ARGS > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
run trace 400 --kernel-trace --stats
run pmc_fetch 400 --kernel-trace --pmc FETCH_SIZE
run pmc_write 400 --kernel-trace --pmc WRITE_SIZE
run pmc_l2 400 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum
python3 tools/traffic.py "$OUT" "$OUT/traffic_c2.json" "$TAG"
find "$OUT" -name "*.csv" | head -20
