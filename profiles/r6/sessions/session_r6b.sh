#!/bin/bash
# r6b: new abort-path tests; same-box A/B of the critical-chain wave priority (s_setprio 2 / 3) and
# nontemporal texel loads on the driver's line (+ synchronous frame latency); subtree_level for
# multi-frame calls
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm_abort.py tests/test_gpu_parity.py::test_config_size_is_checked -x -v -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/r6b_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r6b_tests.log
[ $rc -le 1 ] || exit $rc
RUNS=3 bash tools/ab_multi.sh r6b base ablib/prio2/libpgrt.so ablib/prio3/libpgrt.so ablib/ntex/libpgrt.so ablib/prio3ntex/libpgrt.so || exit 1
RUNS=2 bash tools/ab_multi.sh r6b_sub base "sub3=--cfg subtree_level=3" "sub4=--cfg subtree_level=4" "sub5=--cfg subtree_level=5" || exit 1
# GPU_MAX_HW_QUEUES: 16 (bench default) vs 4 (HIP's default) on the driver line; the C++ drop-in's
# C2 line (its facade sets 16) and with an explicit 4
RUNS=3 bash tools/ab_multi.sh r6b_hwq base "hwq4=--hw-queues 4" "hwq8=--hw-queues 8" || exit 1
for r in 1 2; do
  timeout -k 10 200 build/pg1_pgrt bench assets/avenger/6887_allied_avenger_proxy.obj assets/spherical_map_windows.jpg 20 5 > gpurun_out/cpp_dropin_k20_$r.json 2> gpurun_out/cpp_dropin.err || { tail -5 gpurun_out/cpp_dropin.err; exit 1; }
  tail -1 gpurun_out/cpp_dropin_k20_$r.json
done
GPU_MAX_HW_QUEUES=4 timeout -k 10 200 build/pg1_pgrt bench assets/avenger/6887_allied_avenger_proxy.obj assets/spherical_map_windows.jpg 20 5 > gpurun_out/cpp_dropin_k20_hwq4.json 2>> gpurun_out/cpp_dropin.err || exit 1
tail -1 gpurun_out/cpp_dropin_k20_hwq4.json
timeout -k 10 200 build/pg1_pgrt bench assets/avenger/6887_allied_avenger_proxy.obj assets/spherical_map_windows.jpg 600 5 > gpurun_out/cpp_dropin_k600.json 2>> gpurun_out/cpp_dropin.err || exit 1
tail -1 gpurun_out/cpp_dropin_k600.json
