#!/bin/bash
# r6fin (part c): the steady 400-frame throughput profile (kernel trace, DRAM bytes, SQ counters per
# kernel: tools/throughput_breakdown.py), the C++ drop-in's bench mode twice
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/steady_profile.sh r6fin || exit 1
for r in 1 2; do
  timeout -k 10 120 build/pg1_pgrt bench assets/avenger/6887_allied_avenger_proxy.obj assets/spherical_map_windows.jpg 20 5 > gpurun_out/cpp_dropin_r6fin_$r.out 2> gpurun_out/cpp_dropin_r6fin.err || { tail -5 gpurun_out/cpp_dropin_r6fin.err; exit 1; }
  tail -1 gpurun_out/cpp_dropin_r6fin_$r.out
done
bash tools/profile.sh r6finpath C2 --mode path --roofline-only || exit 1
