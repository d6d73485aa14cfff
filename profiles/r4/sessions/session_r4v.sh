#!/bin/bash
# r4v: level-0 misses finished inside the level-0 packet traversal (environment texel + gamma ->
# framebuffer; directions stored for the hits only; the level-0 shade skips the misses) --
# full GPU suite, then A/B against the HEAD build on the driver's line, 400 frames, the
# synchronous frame; then the path line's PMC traffic at this head
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4v.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_r4v.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
bash tools/ab_matrix.sh r4v "ablib/head/libpgrt.so base" "--steps 20 --warmup 5" "--steps 400" || exit 1
for L in head base; do
  if [ $L = head ]; then export PGRT_LIB=ablib/head/libpgrt.so; else unset PGRT_LIB; fi
  timeout -k 10 300 python3 tools/frame_timeline.py --reps 15 --out gpurun_out/timeline_r4v_$L.json > gpurun_out/timeline_r4v_$L.txt 2>&1 || exit 1
  echo "$L $(head -1 gpurun_out/timeline_r4v_$L.txt | grep -o '"host_ms_median_timeline_off.*')  r20 $(grep '^r20' gpurun_out/timeline_r4v_$L.txt | grep -o '"host_ms_per_frame_off_median": [0-9.]*')"
done
unset PGRT_LIB
bash tools/profile.sh r4v C2 --roofline-only --mode path
