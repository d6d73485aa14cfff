#!/bin/bash
# r4k: level-0 step budget (pgrt_config.l0_budget) -- parity, then the synchronous frame's
# device timeline and the driver's line at several budgets (same box)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4k.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r4k.log
[ $rc -eq 0 ] || exit $rc
tl() {  # name [args]
  local n=$1; shift
  timeout -k 10 300 python3 tools/frame_timeline.py --reps 15 --out gpurun_out/timeline_r4k_$n.json "$@" > gpurun_out/timeline_r4k_$n.txt 2>&1 || { tail -5 gpurun_out/timeline_r4k_$n.txt; exit 1; }
  echo "$n $(head -1 gpurun_out/timeline_r4k_$n.txt | grep -o '"host_ms_median_timeline_off.*')  r20 $(grep '^r20' gpurun_out/timeline_r4k_$n.txt | grep -o '"host_ms_per_frame_off_median": [0-9.]*')"
}
for r in 1 2; do
  tl off$r --cfg l0_budget=-1
  tl b96_$r
  tl b48_$r --cfg l0_budget=48
  tl b160_$r --cfg l0_budget=160
  tl b32_$r --cfg l0_budget=32
done
