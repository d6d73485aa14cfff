# r3fin-b: the final head -- every BASELINE config (tools/round_bench.sh), the path tracer, and the
# rocprofv3 kernel stats + PMC traffic passes for C2 and C5 (tools/profile.sh)
set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/round_bench.sh r3fin || exit 1
timeout -k 10 300 python3 bench.py --mode path --no-cpu-baseline > gpurun_out/bench_r3fin_path.json 2> gpurun_out/bench_r3fin_path.err || { tail -5 gpurun_out/bench_r3fin_path.err; exit 1; }
bash tools/profile.sh r3fin C2 || exit 1
bash tools/profile.sh r3fin C5 || exit 1
