# r3u: sibling-pair BVH node layout -- parity (layouts, C5 scale, tutorial KAT), then A/B of
# bvh_layout 0 vs -1 on C2 (20 / 400 frames) and C5
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3u
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_path.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "bvh_layouts or tutorial1 or closest_hit or c5 or random or geosphere or path_avenger" > gpurun_out/r3u/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3u/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3u/gpu_tests.log
bash tools/ab_args.sh r3u "--steps 20 --warmup 5" "--steps 20 --warmup 5 --cfg bvh_layout=-1" "--steps 400" "--steps 400 --cfg bvh_layout=-1" || exit 1
BENCH_CONFIG=C5 bash tools/ab_args.sh r3u5 "--steps 10 --warmup 2" "--steps 10 --warmup 2 --cfg bvh_layout=-1" || exit 1
