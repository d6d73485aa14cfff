# r3c: stable binning A/B + device-ordered gather (tests)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r3c.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r3c.log; exit 1; }
tail -3 gpurun_out/gpu_tests_r3c.log
for cfg in "" "ray_binning=-1"; do
  for F in 1 8; do
    echo "== diag cfg=[$cfg] F=$F"
    DIAG_CFG=$cfg DIAG_FRAMES=$F timeout -k 10 120 python tools/diag.py 1920 1080 5 1 0 2>&1 | grep -E "^L[0-9]|stage_ms" | cut -c1-60,270-400
  done
done
bash tools/ab_args.sh r3c_bin "--steps 20 --warmup 5" "--steps 20 --warmup 5 --cfg ray_binning=-1" "--steps 400" "--steps 400 --cfg ray_binning=-1"
