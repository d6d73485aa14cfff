# r3o: frames per call x calls in flight for the driver's 20-frame region
set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/ab_args.sh r3o "--steps 20 --warmup 5" "--steps 20 --warmup 5 --frames-per-call 1 --in-flight 16" "--steps 20 --warmup 5 --frames-per-call 2 --in-flight 10" "--steps 20 --warmup 5 --frames-per-call 4 --in-flight 5" "--steps 20 --warmup 5 --frames-per-call 10 --in-flight 2" "--steps 20 --warmup 5 --frames-per-call 20 --in-flight 1"
