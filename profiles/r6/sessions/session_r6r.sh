#!/bin/bash
# r6r: the synchronous frame's ray-tree launch taking the L2 queue from its end (PGRT_SUBTREE_REVERSE=1,
# ablib/srev: the heavy canopy trees' wave started ~35 us into the launch in r6c) vs the tree; the
# one-frame timeline (sync block) for each, then 4 driver lines each (frame_latency_ms)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PGRT_LIB=ablib/srev/libpgrt.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "avenger or subtree or glass or geosphere" > gpurun_out/r6r_tests.log 2>&1 || { tail -30 gpurun_out/r6r_tests.log; exit 1; }
tail -1 gpurun_out/r6r_tests.log
RUNS=4 bash tools/ab_multi.sh r6r base ablib/srev/libpgrt.so || exit 1
