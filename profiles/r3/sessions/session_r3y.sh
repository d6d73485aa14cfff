# r3y: k_shade block size (rays per allocation atomic) 256 (head) vs 512 / 1024 -- C2 20 / 400
# frames, 3 runs each, and the per-level shade times of one 8-frame call
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3y
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "frame_parity or geosphere" > gpurun_out/r3y/gpu_tests_cur.log 2>&1 || { tail -30 gpurun_out/r3y/gpu_tests_cur.log; exit 1; }
for v in cur shade512 shade1024; do
  if [ $v = cur ]; then unset PGRT_LIB; else export PGRT_LIB=ablib/$v/libpgrt.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "frame_parity or geosphere" > gpurun_out/r3y/gpu_tests_$v.log 2>&1 || { tail -30 gpurun_out/r3y/gpu_tests_$v.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/r3y/gpu_tests_$v.log)"
  for args in "--steps 20 --warmup 5" "--steps 400"; do
    vals=""
    for r in 1 2 3; do
      timeout -k 10 180 python3 bench.py --no-cpu-baseline --no-roofline $args > gpurun_out/r3y/b.json 2> gpurun_out/r3y/b.err || { tail -5 gpurun_out/r3y/b.err; exit 1; }
      vals="$vals $(python3 -c "import json; print(json.load(open('gpurun_out/r3y/b.json'))['ms_per_step'])")"
    done
    echo "[$args] $v ms/frame:$vals"
  done
  DIAG_FRAMES=8 timeout -k 10 120 python tools/diag.py 1920 1080 5 1 0 > gpurun_out/r3y/diag_$v.txt 2>&1 || exit 1
  echo "== $v F=8 shade us: $(grep -E '^L[0-9]' gpurun_out/r3y/diag_$v.txt | sed -E 's/.*shade *//; s/ us//' | tr '\n' ' ')"
done
