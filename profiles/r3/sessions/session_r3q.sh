# r3q: bounce-level packets over the 8-wide BVH -- parity, per-level diag, A/B
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3q
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "wide_packets or packet_budget or packet_levels" > gpurun_out/r3q/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3q/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3q/gpu_tests.log
for cfg in "" "packet_width=8" "packet_width=8,packet_budget=-1"; do
  for F in 1 8; do
    echo "== diag cfg=[$cfg] F=$F"
    DIAG_CFG=$cfg DIAG_FRAMES=$F timeout -k 10 120 python tools/diag.py 1920 1080 5 1 0 > gpurun_out/r3q/diag_${F}_${cfg//[=.,]/_}.txt 2>&1 || exit 1
    grep -E "^L[0-2]" gpurun_out/r3q/diag_${F}_${cfg//[=.,]/_}.txt | sed -E 's/ \| shadow.*\| trace/ | trace/' | cut -c1-150
  done
done
bash tools/ab_args.sh r3q "--steps 20 --warmup 5" "--steps 20 --warmup 5 --cfg packet_width=8" "--steps 400" "--steps 400 --cfg packet_width=8"
