# r3ac: C5 -- call_order 2 (every level in submission order) and calls in flight 2 / 4 / 6 with
# the default ordering; C2 with call_order 2
set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
BENCH_CONFIG=C5 bash tools/ab_args.sh r3ac5 "--steps 20 --warmup 3" "--steps 20 --warmup 3 --cfg call_order=2" "--steps 20 --warmup 3 --in-flight 3" "--steps 20 --warmup 3 --in-flight 4" "--steps 20 --warmup 3 --in-flight 8" || exit 1
bash tools/ab_args.sh r3ac "--steps 20 --warmup 5" "--steps 20 --warmup 5 --cfg call_order=2" || exit 1
