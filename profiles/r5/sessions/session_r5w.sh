#!/bin/bash
# r5w: export kernels as the default for every page-locked destination -- host parity tests, the
# box's D2H probe, every host_export mode inside one process (0 default = kernels, 2 split, -1 DMA),
# and the bench's own host-framebuffer figures
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "host or batched" > gpurun_out/gpu_tests_r5w.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r5w.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r5w.log
timeout -k 10 120 ./build/d2h_probe > gpurun_out/d2h_probe_r5w.txt 2>&1 || exit 1
grep -E "1 stream\(s\)|grid 64" gpurun_out/d2h_probe_r5w.txt | head -3
for rep in 1 2; do
  timeout -k 10 300 python3 tools/host_fb.py --modes 0 2 -1 --rounds 2 --reps 10 --async 8x4 2x4 > gpurun_out/host_r5w_$rep.json 2>&1 || { tail -5 gpurun_out/host_r5w_$rep.json; exit 1; }
  cat gpurun_out/host_r5w_$rep.json
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_r5w_k20.json 2> gpurun_out/bench_r5w_k20.err || { tail -5 gpurun_out/bench_r5w_k20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_r5w_k20.json')); print('bench', d['ms_per_step'], d['host_framebuffer'])"
