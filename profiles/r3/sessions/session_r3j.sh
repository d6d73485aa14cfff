# r3j: re-entry check of the head -- GPU suite, smoke, driver-style bench line
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3j
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r3j/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3j/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3j/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3j/smoke.log 2>&1 || { tail -20 gpurun_out/r3j/smoke.log; exit 1; }
tail -1 gpurun_out/r3j/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3j/bench_driver.json 2> gpurun_out/r3j/bench_driver.err || { tail -20 gpurun_out/r3j/bench_driver.err; exit 1; }
cut -c1-400 gpurun_out/r3j/bench_driver.json
