# r3ai: the driver's 20 frames as 8 + 8 + 4 (default) vs 4 + 8 + 8 (--remainder-first)
set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/ab_args.sh r3ai "--steps 20 --warmup 5" "--steps 20 --warmup 5 --remainder-first" "--steps 20 --warmup 5 --frames-per-call 7" "--steps 20 --warmup 5 --frames-per-call 7 --remainder-first" "--steps 20 --warmup 5 --frames-per-call 6 --remainder-first" || exit 1
