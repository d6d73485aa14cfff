#!/bin/bash
# r6p: the packet traversal requests both children's node records before its box tests
# (PGRT_PKT_PREFETCH=1, ablib/pktpf): parity with that build, then A/B on the driver line, the 400-frame
# line and C5 against the tree (base)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PGRT_LIB=ablib/pktpf/libpgrt.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py > gpurun_out/r6p_tests.log 2>&1 || { tail -30 gpurun_out/r6p_tests.log; exit 1; }
tail -2 gpurun_out/r6p_tests.log
RUNS=3 bash tools/ab_multi.sh r6p base ablib/pktpf/libpgrt.so || exit 1
RUNS=2 ARGS="--steps 400" bash tools/ab_multi.sh r6p400 base ablib/pktpf/libpgrt.so || exit 1
RUNS=2 ARGS="--config C5 --steps 10 --warmup 2" bash tools/ab_multi.sh r6pC5 base ablib/pktpf/libpgrt.so || exit 1
