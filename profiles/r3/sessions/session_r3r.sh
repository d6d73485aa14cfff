# r3r: refraction statistics aggregated per block / launch (no per-wave same-address atomics) --
# parity, then A/B against the previous head (ablib/head)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3r
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_path.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "frame_parity or geosphere or tail or furnace or path_avenger or multiple_lights" > gpurun_out/r3r/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3r/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3r/gpu_tests.log
for args in "--steps 20 --warmup 5" "--steps 400"; do
  for lib in head new; do
    v=""
    for r in 1 2 3; do
      if [ $lib = head ]; then
        PGRT_LIB=ablib/head/libpgrt.so timeout -k 10 180 python3 bench.py --no-cpu-baseline --no-roofline $args > gpurun_out/r3r/b.json 2> gpurun_out/r3r/b.err || { tail -5 gpurun_out/r3r/b.err; exit 1; }
      else
        timeout -k 10 180 python3 bench.py --no-cpu-baseline --no-roofline $args > gpurun_out/r3r/b.json 2> gpurun_out/r3r/b.err || { tail -5 gpurun_out/r3r/b.err; exit 1; }
      fi
      v="$v $(python3 -c "import json; print(json.load(open('gpurun_out/r3r/b.json'))['ms_per_step'])")"
    done
    echo "[$args] $lib ms/frame:$v"
  done
done
for lib in head new; do
  if [ $lib = head ]; then export PGRT_LIB=ablib/head/libpgrt.so; else unset PGRT_LIB; fi
  DIAG_FRAMES=8 timeout -k 10 120 python tools/diag.py 1920 1080 5 1 0 > gpurun_out/r3r/diag_$lib.txt 2>&1 || exit 1
  echo "== diag F=8 $lib"; grep -E "^L[0-9]" gpurun_out/r3r/diag_$lib.txt | sed -E 's/.*\| trace/trace/'
done
