#!/bin/bash
# r5m: asynchronous host frames -- DMA (-1), export kernels (1), split kernel/DMA (2: 50 % by the
# blit kernel; sp33 / sp70 libraries: 33 / 70 %), every mode measured inside one process, 2 rounds;
# parity of the host frames first
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "host" > gpurun_out/gpu_tests_r5m.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r5m.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r5m.log
for lib in base sp33 sp70; do
  if [ $lib = base ]; then unset PGRT_LIB; else export PGRT_LIB=ablib/$lib/libpgrt.so; fi
  for rep in 1 2; do
    timeout -k 10 300 python3 tools/host_fb.py --modes -1 1 2 --rounds 2 --reps 10 --async 8x4 2x4 > gpurun_out/host_r5m_${lib}_$rep.json 2>&1 || { tail -5 gpurun_out/host_r5m_${lib}_$rep.json; exit 1; }
    cat gpurun_out/host_r5m_${lib}_$rep.json
  done
done
