# r3v: every BASELINE config through bench.py (tools/round_bench.sh) + the path tracer at C2 size
set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/round_bench.sh r3v || exit 1
timeout -k 10 300 python3 bench.py --mode path --no-cpu-baseline > gpurun_out/bench_r3v_path.json 2> gpurun_out/bench_r3v_path.err || { tail -5 gpurun_out/bench_r3v_path.err; exit 1; }
cut -c1-200 gpurun_out/bench_r3v_path.json
