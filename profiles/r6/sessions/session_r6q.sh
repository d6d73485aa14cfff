#!/bin/bash
# r6q: (1) the C5 line with the timed roofline's busy time capped at ms_per_step; (2) one-lane trace
# occupancy: all-LDS stack of depth + 2 entries (31 KB per block: 5 waves per SIMD, head) vs a 16-entry
# LDS stack spilling to global past it (tsp: 6 waves by VGPRs), + launch bound 7 (tsp7: 68 VGPRs) / 8
# (tsp8: 64 VGPRs, 4 spilled) -- parity of tsp7 / tsp8, then the driver line and the 400-frame line;
# (3) frames per call on the 600-frame default line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --config C5 --steps 20 --warmup 3 > gpurun_out/bench_r6fin_C5_capped.json 2> gpurun_out/bench_r6fin_C5_capped.err || { tail -5 gpurun_out/bench_r6fin_C5_capped.err; exit 1; }
for v in tsp7 tsp8; do
  PGRT_LIB=ablib/$v/libpgrt.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/r6q_tests_$v.log 2>&1 || { tail -30 gpurun_out/r6q_tests_$v.log; exit 1; }
  tail -1 gpurun_out/r6q_tests_$v.log
done
RUNS=3 bash tools/ab_multi.sh r6q base ablib/tsp/libpgrt.so ablib/tsp7/libpgrt.so ablib/tsp8/libpgrt.so || exit 1
RUNS=2 ARGS="--steps 400" bash tools/ab_multi.sh r6q400 base ablib/tsp7/libpgrt.so ablib/tsp8/libpgrt.so || exit 1
RUNS=2 ARGS="--steps 600" bash tools/ab_multi.sh r6fin600 base "f32=--frames-per-call 32" "f64=--frames-per-call 64" || exit 1
