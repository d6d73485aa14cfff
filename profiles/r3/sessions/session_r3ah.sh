# r3ah: parity with the 32M default batch (C3 full size, multi-batch, C4 tiles), C2 unchanged check
set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3ah
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_path.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "c3 or c4 or batch or path" > gpurun_out/r3ah/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3ah/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3ah/gpu_tests.log
bash tools/ab_args.sh r3ah "--steps 20 --warmup 5" || exit 1
