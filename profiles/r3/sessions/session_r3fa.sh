# r3fin-a: empty scene + degenerate image sizes (new tests), then the whole GPU suite
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3fin
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "empty_scene or degenerate_image" > gpurun_out/r3fin/new_tests.log 2>&1 || { tail -40 gpurun_out/r3fin/new_tests.log; exit 1; }
tail -1 gpurun_out/r3fin/new_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r3fin/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3fin/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3fin/gpu_tests.log
