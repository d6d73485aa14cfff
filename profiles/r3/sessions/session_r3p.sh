# r3p: packet levels / group_max for the driver's 20-frame region and the long run
set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/ab_args.sh r3p "--steps 20 --warmup 5" "--steps 20 --warmup 5 --cfg packet_levels=1" "--steps 20 --warmup 5 --cfg packet_levels=1 --cfg group_max=400000" "--steps 20 --warmup 5 --cfg group_max=400000" "--steps 400" "--steps 400 --cfg packet_levels=1"
