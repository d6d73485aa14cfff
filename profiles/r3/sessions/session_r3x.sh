# r3x (second pass: today's commits): where did C5 / C2-steady lose since r2k -- the current bench.py over library builds of
# earlier commits (ablib/c_<commit>), one run each: C5 20 frames, C2 400 frames
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3x
export PYTHONUNBUFFERED=1
for v in c_789530f c_5e64c14 c_9256189 c_122597c c_b8ff221 cur; do
  if [ $v = cur ]; then unset PGRT_LIB; else export PGRT_LIB=ablib/$v/libpgrt.so; fi
  timeout -k 10 200 python3 bench.py --config C5 --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/r3x/c5_$v.json 2> gpurun_out/r3x/c5_$v.err || { tail -5 gpurun_out/r3x/c5_$v.err; exit 1; }
  timeout -k 10 200 python3 bench.py --steps 400 --no-cpu-baseline --no-roofline > gpurun_out/r3x/c2_$v.json 2> gpurun_out/r3x/c2_$v.err || { tail -5 gpurun_out/r3x/c2_$v.err; exit 1; }
  timeout -k 10 200 python3 bench.py --mode path --steps 100 --no-cpu-baseline --no-roofline > gpurun_out/r3x/p_$v.json 2> gpurun_out/r3x/p_$v.err || { tail -5 gpurun_out/r3x/p_$v.err; exit 1; }
  echo "path $(python3 -c "import json; print(json.load(open('gpurun_out/r3x/p_$v.json'))['ms_per_step'])")"
  echo "$v C5 $(python3 -c "import json; print(json.load(open('gpurun_out/r3x/c5_$v.json'))['ms_per_step'])") C2-400 $(python3 -c "import json; print(json.load(open('gpurun_out/r3x/c2_$v.json'))['ms_per_step'])")"
done
