# r3af: C3 -- level-0 rays per sample batch (pgrt_config.max_batch_rays, default 16M) and calls in flight
set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
BENCH_CONFIG=C3 bash tools/ab_args.sh r3af3 "--steps 12 --warmup 3" "--steps 12 --warmup 3 --cfg max_batch_rays=33554432" "--steps 12 --warmup 3 --cfg max_batch_rays=8388608" "--steps 12 --warmup 3 --in-flight 3" "--steps 12 --warmup 3 --in-flight 10" || exit 1
