#!/bin/bash
# r5n: the SDMA device-to-host rate per process (27 or 54 GB/s on the same box) under the runtime's
# engine-selection knobs: 6 processes each of the D2H probe's 1-stream copy
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
for envs in "X=0" "HSA_ENABLE_SDMA_RECOMMENDED_ENG=1" "HSA_ENABLE_SDMA_RECOMMENDED_ENG=0" "HSA_ENABLE_SDMA_GANG=1" "HSA_ENABLE_SDMA_GANG=0"; do
  line="$envs:"
  for r in 1 2 3 4 5 6; do
    env $envs timeout -k 10 60 ./build/d2h_probe > gpurun_out/d2h_r5n.txt 2>&1 || { tail -3 gpurun_out/d2h_r5n.txt; exit 1; }
    line="$line $(grep -m1 '1 stream(s)' gpurun_out/d2h_r5n.txt | awk '{print $(NF-1)}')"
  done
  echo "$line"
done | tee gpurun_out/sdma_r5n.txt
