# r3g: persistent tail (tail.hip) -- parity first (tail tests alone, then the suite), then per-level
# diag and the A/B of tail on / off
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3g
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "persistent_tail" -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r3g/tail_tests.log 2>&1 || { tail -40 gpurun_out/r3g/tail_tests.log; exit 1; }
tail -3 gpurun_out/r3g/tail_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r3g/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3g/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3g/gpu_tests.log
for cfg in "tail_level=-1" ""; do
  for F in 1 8; do
    echo "== diag cfg=[$cfg] F=$F"
    DIAG_CFG=$cfg DIAG_FRAMES=$F timeout -k 10 120 python tools/diag.py 1920 1080 5 1 0 > gpurun_out/r3g/diag_${F}_${cfg//[=,]/_}.txt 2>&1 || exit 1
    grep -E "^L[0-9]|stage_ms" gpurun_out/r3g/diag_${F}_${cfg//[=,]/_}.txt | sed -E 's/ \| shadow.*\| trace/ | trace/' | cut -c1-170
  done
done
bash tools/ab_args.sh r3g "--steps 20 --warmup 5 --cfg tail_level=-1" "--steps 20 --warmup 5" "--steps 20 --warmup 5 --cfg tail_level=2" "--steps 400 --cfg tail_level=-1" "--steps 400" "--steps 400 --cfg tail_level=2"
