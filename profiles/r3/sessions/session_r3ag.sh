# r3ag: level-0 rays per sample batch for C3 / C4 (default 16M = 2^24)
set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
BENCH_CONFIG=C3 bash tools/ab_args.sh r3ag3 "--steps 12 --warmup 3" "--steps 12 --warmup 3 --cfg max_batch_rays=33554432" "--steps 12 --warmup 3 --cfg max_batch_rays=67108864" || exit 1
BENCH_CONFIG=C4 bash tools/ab_args.sh r3ag4 "--steps 6 --warmup 2" "--steps 6 --warmup 2 --cfg max_batch_rays=33554432" "--steps 6 --warmup 2 --cfg max_batch_rays=67108864" || exit 1
