# r3ab (pass 2): the default call_order (ordered for scenes above 262144 triangles) -- C2 / C5
# default vs forced free / ordered, parity of the ordered path
set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r3ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "frames_in_flight or batched or new_frame_sets or distinct or c5" > gpurun_out/r3ab/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3ab/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3ab/gpu_tests.log
bash tools/ab_args.sh r3ab "--steps 20 --warmup 5" "--steps 20 --warmup 5 --cfg call_order=-1" || exit 1
BENCH_CONFIG=C5 bash tools/ab_args.sh r3ab5 "--steps 20 --warmup 3" "--steps 20 --warmup 3 --cfg call_order=-1" || exit 1
