# r3s: queue-size-dependent default packet budget (64 steps below 2^20 expected rays) -- parity,
# driver line + frame latency A/B against the previous head (ablib/head), one-frame diag
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3s
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "frame_parity or geosphere or full_size or budget or frames_in_flight or batched" > gpurun_out/r3s/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3s/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3s/gpu_tests.log
for args in "--steps 20 --warmup 5" "--steps 400"; do
  for lib in head new; do
    v=""; l=""
    for r in 1 2 3; do
      if [ $lib = head ]; then export PGRT_LIB=ablib/head/libpgrt.so; else unset PGRT_LIB; fi
      timeout -k 10 180 python3 bench.py --no-cpu-baseline --no-roofline $args > gpurun_out/r3s/b.json 2> gpurun_out/r3s/b.err || { tail -5 gpurun_out/r3s/b.err; exit 1; }
      v="$v $(python3 -c "import json; print(json.load(open('gpurun_out/r3s/b.json'))['ms_per_step'])")"
      l="$l $(python3 -c "import json; print(json.load(open('gpurun_out/r3s/b.json'))['frame_latency_ms'])")"
    done
    echo "[$args] $lib ms/frame:$v | frame_latency_ms:$l"
  done
done
unset PGRT_LIB
DIAG_FRAMES=1 timeout -k 10 120 python tools/diag.py 1920 1080 5 1 0 > gpurun_out/r3s/diag_new.txt 2>&1 || exit 1
echo "== diag F=1 new"; grep -E "^L[0-9]" gpurun_out/r3s/diag_new.txt | sed -E 's/ \| shadow.*\| trace/ | trace/' | cut -c1-150
