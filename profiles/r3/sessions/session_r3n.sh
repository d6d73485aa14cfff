# r3n: longest-ray profile of the one-lane deep-level kernel (group_max -1), one frame and 4 frames
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3n
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for F in 1 4; do
for cfg in "group_max=-1" "group_max=-1,packet_levels=-1"; do
  echo "== diag cfg=[$cfg] F=$F"
  DIAG_CFG=$cfg DIAG_FRAMES=$F timeout -k 10 120 python tools/diag.py 1920 1080 5 1 0 > gpurun_out/r3n/diag_${F}_${cfg//[=.,]/_}.txt 2>&1 || exit 1
  grep -E "^L[0-9]" gpurun_out/r3n/diag_${F}_${cfg//[=.,]/_}.txt | cut -c1-400
done
done
