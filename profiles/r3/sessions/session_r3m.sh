# r3m: host launch stalls -- synchronous C2 frames under HIP_FORCE_DEV_KERNARG=0/1 (API trace)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3m
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for kv in 1 0; do
  echo "== HIP_FORCE_DEV_KERNARG=$kv"
  HIP_FORCE_DEV_KERNARG=$kv timeout -k 10 120 python3 tools/sync_frames.py 12 2>&1 | grep "frame ms"
  HIP_FORCE_DEV_KERNARG=$kv timeout -k 10 120 rocprofv3 --hip-trace --kernel-trace --output-format csv -d gpurun_out/r3m/api$kv -o api -- python3 tools/sync_frames.py 12 > gpurun_out/r3m/sync$kv.txt 2>&1 || { tail -20 gpurun_out/r3m/sync$kv.txt; exit 1; }
  a=$(find gpurun_out/r3m/api$kv -name '*hip_api_trace.csv' | head -1)
  k=$(find gpurun_out/r3m/api$kv -name '*kernel_trace.csv' | head -1)
  python3 tools/api_timeline.py $a $k 2 > gpurun_out/r3m/api_timeline$kv.txt
  head -3 gpurun_out/r3m/api_timeline$kv.txt
  HIP_FORCE_DEV_KERNARG=$kv timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > gpurun_out/r3m/bench$kv.json 2>gpurun_out/r3m/bench$kv.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r3m/bench$kv.json')); print('bench ms/frame', d['ms_per_step'], 'latency', d['frame_latency_ms'])"
done
