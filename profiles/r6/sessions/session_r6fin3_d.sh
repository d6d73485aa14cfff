#!/bin/bash
# r6fin3 (part d): at the final head -- the C++ drop-in's bench mode twice, and every rank of world
# 2 / 4 / 8 on one GPU (emulated) for C2, steady and driver-shaped
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 120 build/pg1_pgrt bench assets/avenger/6887_allied_avenger_proxy.obj assets/spherical_map_windows.jpg 20 5 > gpurun_out/cpp_dropin_r6fin3_$r.out 2> gpurun_out/cpp_dropin_r6fin3.err || { tail -5 gpurun_out/cpp_dropin_r6fin3.err; exit 1; }
  tail -n 1 gpurun_out/cpp_dropin_r6fin3_$r.out
done
timeout -k 10 500 python3 -u tools/emulate_ranks.py --configs C2 --out gpurun_out/emulated_ranks_r6fin3.jsonl 2>&1 | tee gpurun_out/emulated_ranks_r6fin3.log || exit 1
timeout -k 10 400 python3 -u tools/emulate_ranks.py --configs C2 --frames 20 --warmup 5 --repeat 5 --out gpurun_out/emulated_ranks_r6fin3_k20.jsonl 2>&1 | tee gpurun_out/emulated_ranks_r6fin3_k20.log || exit 1
