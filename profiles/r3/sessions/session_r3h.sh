# r3h: persistent tail -- parity, then where its time goes (profile == 2 counters), then A/B
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3h
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "persistent_tail or geosphere or full_size" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r3h/tail_tests.log 2>&1 || { tail -40 gpurun_out/r3h/tail_tests.log; exit 1; }
tail -1 gpurun_out/r3h/tail_tests.log
for F in 1 8; do
  echo "== F=$F tail default"; DIAG_FRAMES=$F timeout -k 10 120 python tools/tail_diag.py 1920 1080 5 | head -9 || exit 1
done
bash tools/ab_args.sh r3h "--steps 20 --warmup 5 --cfg tail_level=-1" "--steps 20 --warmup 5" "--steps 400 --cfg tail_level=-1" "--steps 400"
