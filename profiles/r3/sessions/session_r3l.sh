# r3l: multi-device context test; BVH split clipping vs deep-level latency (diag F=1);
# host API timeline of one synchronous C2 frame
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3l
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "multi_device or distributed or frames_in_flight" > gpurun_out/r3l/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3l/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r3l/gpu_tests.log
for cfg in "" "split_beta=0.25" "split_beta=0.5" "split_beta=1.0" "bvh_builder=1"; do
  echo "== diag cfg=[$cfg] F=1"
  DIAG_CFG=$cfg DIAG_FRAMES=1 timeout -k 10 120 python tools/diag.py 1920 1080 5 1 0 > gpurun_out/r3l/diag_${cfg//[=.,]/_}.txt 2>&1 || exit 1
  head -2 gpurun_out/r3l/diag_${cfg//[=.,]/_}.txt | cut -c1-200
  grep -E "^L[0-9]" gpurun_out/r3l/diag_${cfg//[=.,]/_}.txt | sed -E 's/ \| shadow.*\| trace/ | trace/' | cut -c1-150
done
timeout -k 10 120 rocprofv3 --hip-trace --kernel-trace --output-format csv -d gpurun_out/r3l/api -o api -- python3 tools/sync_frames.py 12 > gpurun_out/r3l/sync_frames.txt 2>&1 || { tail -20 gpurun_out/r3l/sync_frames.txt; exit 1; }
grep "frame ms" gpurun_out/r3l/sync_frames.txt
a=$(find gpurun_out/r3l/api -name '*hip_api_trace.csv' | head -1)
k=$(find gpurun_out/r3l/api -name '*kernel_trace.csv' | head -1)
python3 tools/api_timeline.py $a $k > gpurun_out/r3l/api_timeline.txt
head -4 gpurun_out/r3l/api_timeline.txt
