#!/bin/bash
# A/B of BVH builders on the bench workload
cd "$(dirname "$0")/.."
for b in lbvh ploc; do
  echo "builder $b"
  PGRT_BVH=$b timeout -k 10 120 python tools/diag.py 2>&1
done
