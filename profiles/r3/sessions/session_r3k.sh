# r3k: kernel timeline of the driver-style timed region (20 frames) and of one synchronous frame
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3k
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3k/kt -o kt -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/r3k/bench.json 2> gpurun_out/r3k/bench.err || { tail -20 gpurun_out/r3k/bench.err; exit 1; }
cut -c1-300 gpurun_out/r3k/bench.json
f=$(find gpurun_out/r3k/kt -name '*kernel_trace.csv' | head -1)
python3 tools/timeline.py $f 8 3 > gpurun_out/r3k/timeline_timed.txt
python3 tools/timeline.py $f 11 1 > gpurun_out/r3k/timeline_latency1.txt
python3 tools/timeline.py $f 12 1 > gpurun_out/r3k/timeline_latency2.txt
head -3 gpurun_out/r3k/timeline_timed.txt
