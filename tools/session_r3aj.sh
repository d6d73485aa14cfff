# r3aj: C++ facade on several ranks (pgrt_create_devices) + the call-split A/B of r3ai
set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3aj
timeout -k 10 300 python -u -m pytest tests/test_gpu_cpp_host.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r3aj/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3aj/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3aj/gpu_tests.log
bash tools/session_r3ai.sh
