# r3d: latency vs throughput of the existing bounce-level kernel choices (packets / 8 lanes per
# ray / one lane per ray): one-frame and 8-frame per-level diag, and the 20- / 400-frame lines
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3d
export PYTHONUNBUFFERED=1
for cfg in "" "packet_levels=1,group_max=4000000" "packet_levels=1,group_max=-1" "group_max=4000000"; do
  for F in 1 8; do
    echo "== diag cfg=[$cfg] F=$F"
    DIAG_CFG=$cfg DIAG_FRAMES=$F timeout -k 10 120 python tools/diag.py 1920 1080 5 1 0 > gpurun_out/r3d/diag_${F}_${cfg//[=,]/_}.txt 2>&1 || exit 1
    grep -E "^L[0-9]|stage_ms" gpurun_out/r3d/diag_${F}_${cfg//[=,]/_}.txt | cut -c1-200
  done
done
bash tools/ab_args.sh r3d "--steps 20 --warmup 5" "--steps 20 --warmup 5 --packet-levels 1 --group-max 4000000" "--steps 20 --warmup 5 --group-max 4000000" "--steps 400" "--steps 400 --packet-levels 1 --group-max 4000000" "--steps 400 --group-max 4000000"
