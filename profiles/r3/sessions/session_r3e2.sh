set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3e
export PYTHONUNBUFFERED=1
timeout -k 10 120 python tools/diff_libs.py ablib/base/libpgrt.so pgi_raytracing_amd/lib/libpgrt.so 48 36 5 1 0
timeout -k 10 120 python tools/diff_libs.py ablib/base/libpgrt.so pgi_raytracing_amd/lib/libpgrt.so 48 36 0 1 0
timeout -k 10 120 python tools/diff_libs.py ablib/base/libpgrt.so pgi_raytracing_amd/lib/libpgrt.so 48 36 5 2 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r3e/gpu_tests2.log 2>&1; grep -E "passed|failed|FAILED" gpurun_out/r3e/gpu_tests2.log | tail -30
