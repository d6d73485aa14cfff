# r3f: bounce-level packet step budget (deferred rays to k_trace8g<RESUME>): parity, per-level
# diag, A/B of the budget
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3f
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r3f/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3f/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3f/gpu_tests.log
for cfg in "packet_budget=-1" "" "packet_budget=128" "packet_budget=64"; do
  for F in 1 8; do
    echo "== diag cfg=[$cfg] F=$F"
    DIAG_CFG=$cfg DIAG_FRAMES=$F timeout -k 10 120 python tools/diag.py 1920 1080 5 1 0 > gpurun_out/r3f/diag_${F}_${cfg//[=,]/_}.txt 2>&1 || exit 1
    grep -E "^L[0-9]" gpurun_out/r3f/diag_${F}_${cfg//[=,]/_}.txt | sed -E 's/ \| shadow.*\| trace/ | trace/' | cut -c1-150
  done
done
bash tools/ab_args.sh r3f "--steps 20 --warmup 5 --cfg packet_budget=-1" "--steps 20 --warmup 5" "--steps 20 --warmup 5 --cfg packet_budget=128" "--steps 20 --warmup 5 --cfg packet_budget=512" "--steps 400 --cfg packet_budget=-1" "--steps 400" "--steps 400 --cfg packet_budget=128" "--steps 400 --cfg packet_budget=512"
