# r3e: k_shade_l0f (level-0 1-spp shade with env / attribute loads in flight together and the
# allocation atomic overlapped) vs HEAD's k_shade<LDS, L0F>; GPU suite first
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3e
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r3e/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3e/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3e/gpu_tests.log

for L in head:ablib/base/libpgrt.so new:pgi_raytracing_amd/lib/libpgrt.so; do
  name=${L%%:*}; lib=${L#*:}
  for args in "--steps 20 --warmup 5" "--steps 400"; do
    v=""
    for r in 1 2 3; do
      PGRT_LIB=$lib timeout -k 10 180 python3 bench.py --no-cpu-baseline --no-roofline $args > gpurun_out/r3e/b.json 2> gpurun_out/r3e/b.err || { tail -5 gpurun_out/r3e/b.err; exit 1; }
      v="$v $(python3 -c "import json; print(json.load(open('gpurun_out/r3e/b.json'))['ms_per_step'])")"
    done
    echo "$name [$args] ms/frame $v"
  done
done
export TMPDIR=/tmp
for L in head:ablib/base/libpgrt.so new:pgi_raytracing_amd/lib/libpgrt.so; do
  name=${L%%:*}; lib=${L#*:}
  PGRT_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3e/kt_$name -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --no-roofline --steps 200 > gpurun_out/r3e/kt_$name.log 2>&1 || { tail -5 gpurun_out/r3e/kt_$name.log; exit 1; }
  f=$(find gpurun_out/r3e/kt_$name -name "*kernel_stats.csv" | head -1)
  echo "== $name"; grep -E "k_shade|k_trace_pkt<false, true" "$f" | cut -d, -f1-4 | sed 's/(pgrt::SceneView[^"]*//'
done
