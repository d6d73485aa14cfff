# r3ad: EXPERIMENT call_order 3 -- the next call's level-0 trace waits for this call's level-0
# TRACE only (its shade overlaps the next trace) -- C2 20 / 400, C3, C5
set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/ab_args.sh r3ad "--steps 20 --warmup 5" "--steps 20 --warmup 5 --cfg call_order=3" "--steps 400" "--steps 400 --cfg call_order=3" || exit 1
BENCH_CONFIG=C3 bash tools/ab_args.sh r3ad3 "--steps 12 --warmup 3" "--steps 12 --warmup 3 --cfg call_order=3" || exit 1
BENCH_CONFIG=C5 bash tools/ab_args.sh r3ad5 "--steps 20 --warmup 3" "--steps 20 --warmup 3 --cfg call_order=3" || exit 1
