# r3ae: C5 with the sibling-pair node layout (bvh_layout 1) now that level 0 is ordered
set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
BENCH_CONFIG=C5 bash tools/ab_args.sh r3ae5 "--steps 20 --warmup 3" "--steps 20 --warmup 3 --cfg bvh_layout=1" "--steps 20 --warmup 3 --cfg split_beta=0.3" || exit 1
