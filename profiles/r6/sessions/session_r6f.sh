#!/bin/bash
# r6f: the cooperative ray-tree kernel's hang in test_c3_multi_batch_64spp_dof (r6d) -- the same test
# on a watchdog build (PGRT_COOP_WATCHDOG: a wave past 2^20 iterations prints its block's state and
# stops), 90 s limit; then the shade-phase record (diagnostics build) over the driver's 20 frames
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PGRT_LIB=ablib/coopwd/libpgrt.so timeout -k 10 90 python3 -u -m pytest tests/test_gpu_configs.py -k "test_c3_multi_batch" -x -q -s -p no:cacheprovider --timeout 80 --timeout-method thread > gpurun_out/r6f_coopwd.log 2>&1
echo "rc=$?"
grep -m 20 "watchdog" gpurun_out/r6f_coopwd.log
tail -5 gpurun_out/r6f_coopwd.log
PGRT_LIB=ablib/stepprof2/libpgrt.so timeout -k 10 90 python3 tools/step_profile.py --shade --out gpurun_out/shade_profile_r6f.json > gpurun_out/shade_profile_r6f.log 2>&1 || { tail -20 gpurun_out/shade_profile_r6f.log; exit 1; }
head -c 2500 gpurun_out/shade_profile_r6f.json
