#!/bin/bash
# r6h: the lock-free cooperative ray-tree kernel -- the C3 multi-batch test on the watchdog build first
# (90 s), then the whole GPU suite on the coop library, then same-box A/B (synchronous frame + driver
# line) and the coop timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PGRT_LIB=ablib/coopwd/libpgrt.so timeout -k 10 100 python3 -u -m pytest tests/test_gpu_configs.py -k "test_c3_multi_batch" -x -q -s -p no:cacheprovider --timeout 90 --timeout-method thread > gpurun_out/r6h_coopwd.log 2>&1; rc=$?
echo "watchdog-build C3 multi-batch rc=$rc"; grep -m 10 "watchdog" gpurun_out/r6h_coopwd.log; tail -2 gpurun_out/r6h_coopwd.log
[ $rc -eq 0 ] || exit 1
for v in coop coopu; do
  PGRT_LIB=ablib/$v/libpgrt.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r6h_gpu_tests_$v.log 2>&1; rc=$?
  echo "$v suite rc=$rc"; tail -3 gpurun_out/r6h_gpu_tests_$v.log
  [ $rc -eq 0 ] || exit 1
done
RUNS=3 bash tools/ab_multi.sh r6h base ablib/coop/libpgrt.so ablib/coopu/libpgrt.so || exit 1
PGRT_LIB=ablib/coopu/libpgrt.so timeout -k 10 200 python3 tools/frame_timeline.py --out gpurun_out/timeline_r6h_coopu.json > gpurun_out/timeline_r6h_coopu.txt 2>&1 || { tail -5 gpurun_out/timeline_r6h_coopu.txt; exit 1; }
head -24 gpurun_out/timeline_r6h_coopu.txt
