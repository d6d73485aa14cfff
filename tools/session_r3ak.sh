# r3ak: maximum depth / samples test, smoke()
set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3ak
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 250 --timeout-method thread -k "maximum_depth" > gpurun_out/r3ak/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3ak/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3ak/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
