#!/bin/bash
# r4n: L2 hit rates of every kernel of synchronous C2 frames (PMC, one counter group per pass)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
OUT=gpurun_out/pmc_r4n
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i + 1))
  echo "=== pass $i: $grp"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o p$i --output-format csv -- python3 tools/sync_frames.py 12 > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "=== pass $i rc=$rc"; tail -2 "$OUT/p$i.log"
  [ $rc -eq 0 ] || break
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt" 2>&1
cat "$OUT/summary.txt"
