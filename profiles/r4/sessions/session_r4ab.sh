#!/bin/bash
# r4fin: head evidence -- GPU suite + smoke, every config's bench line, the C2 rocprof kernel stats and
# PMC traffic, the synchronous / 20-frame device timelines, the path-tracing line with its CPU baseline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_check.sh tests smoke || exit 1
bash tools/round_bench.sh r4fin || exit 1
timeout -k 10 400 python3 bench.py --mode path --steps 20 --warmup 3 > gpurun_out/bench_r4fin_path.json 2> gpurun_out/bench_r4fin_path.err || exit 1
bash tools/profile.sh r4fin C2 || exit 1
timeout -k 10 300 python3 tools/frame_timeline.py --out gpurun_out/timeline_r4fin.json > gpurun_out/timeline_r4fin.txt 2>&1 || exit 1

# then the occupancy / budget A/B (r4aa)
for v in bpk8 sh8 l0f6; do
  PGRT_LIB=ablib/$v/libpgrt.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "frame_parity or geosphere or full_size or tile_order or subtree or batched" > gpurun_out/gpu_tests_r4aa_$v.log 2>&1; rc=$?
  echo "$v $(tail -1 gpurun_out/gpu_tests_r4aa_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
bash tools/ab_matrix.sh r4aa "ablib/head/libpgrt.so ablib/bpk8/libpgrt.so ablib/sh8/libpgrt.so ablib/l0f6/libpgrt.so" "--steps 20 --warmup 5" "--steps 400" || exit 1
# bounce-level packet budget for multi-frame batches (default 256 steps)
for b in 128 512 256; do
  v=""
  for r in 1 2 3; do
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline --steps 400 --cfg packet_budget=$b > gpurun_out/r4aa.json 2>gpurun_out/r4aa.err || exit 1
    v="$v $(python3 -c "import json; print(json.load(open('gpurun_out/r4aa.json'))['ms_per_step'])")"
  done
  echo "[--steps 400 --cfg packet_budget=$b] ms/frame:$v"
done
