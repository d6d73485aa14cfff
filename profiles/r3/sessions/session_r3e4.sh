set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3e
export PYTHONUNBUFFERED=1
timeout -k 10 120 python tools/diff_libs.py ablib/base/libpgrt.so pgi_raytracing_amd/lib/libpgrt.so 48 36 5 2 1 | head -3
timeout -k 10 120 python tools/diff_libs.py ablib/base/libpgrt.so pgi_raytracing_amd/lib/libpgrt.so 64 48 5 1 0 | head -3
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r3e/gpu_tests3.log 2>&1; grep -E "passed|failed|FAILED" gpurun_out/r3e/gpu_tests3.log | tail -12
