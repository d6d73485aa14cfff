#!/bin/bash
# rocprofv3 passes for one bench workload (run on the GPU box via gpurun):
#   1. kernel trace + stats (per-kernel average durations)
#   2.-5. PMC passes, one counter group each (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass):
#         FETCH_SIZE | WRITE_SIZE | TCC hit/miss | VALU instructions + GRBM cycles
# Usage: tools/profile.sh <tag> <config> [bench args...]   (config: C2 | C3 | C4 | C5)
set -u
cd "$(dirname "$0")/.."
TAG=${1:-r2}
CFG=${2:-C2}
shift 2 || shift $#
ARGS="--config $CFG ${*:---roofline-only}"
OUT=gpurun_out/prof_${TAG}_${CFG}
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
run trace 300 --kernel-trace --stats
run pmc_fetch 300 --kernel-trace --pmc FETCH_SIZE
run pmc_write 300 --kernel-trace --pmc WRITE_SIZE
run pmc_l2 300 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum
run pmc_valu 300 --kernel-trace --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE
# bench.py --roofline-only's frames per call and profile=1 calls for this config (traffic.py)
if [ "$CFG" = C2 ]; then export FRAMES_PER_CALL=8 ROOF_CALLS=5; else export FRAMES_PER_CALL=1 ROOF_CALLS=2; fi
python3 tools/traffic.py "$OUT" "$OUT/traffic_${CFG}.json" "$TAG" "$(grep -o '"workload": "[^"]*"' "$OUT/trace.log" | head -1 | sed 's/"workload": "//; s/"$//')"
