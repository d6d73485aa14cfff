#!/bin/bash
# r6fin (part b): final-head roofline profiles of all four configs (kernel trace + PMC of exactly the
# bench's roofline calls; tools/traffic.py -> traffic_<cfg>.json for bench.py's TRAFFIC map), the
# synchronous / 20-frame device timelines, the host-framebuffer figures
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in C2 C3 C4 C5; do
  bash tools/profile.sh r6fin $c || exit 1
done
timeout -k 10 300 python3 tools/frame_timeline.py --out gpurun_out/timeline_r6fin.json > gpurun_out/timeline_r6fin.txt 2>&1 || { tail -5 gpurun_out/timeline_r6fin.txt; exit 1; }
timeout -k 10 200 python3 tools/host_fb.py --async > gpurun_out/host_r6fin.json 2>&1 && cat gpurun_out/host_r6fin.json
timeout -k 10 300 python3 tools/frame_timeline.py --host --out gpurun_out/timeline_host_r6fin.json > gpurun_out/timeline_host_r6fin.txt 2>&1 || exit 1
