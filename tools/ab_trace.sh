#!/bin/bash
# A/B of traversal schedules on the bench workload (one process per variant, same box)
cd "$(dirname "$0")/.."
for v in 0 1 2 3 0 1 2 3; do
  echo "variant $v"
  PGRT_TRACE_VARIANT=$v timeout -k 10 120 python tools/diag.py 2>&1 | grep stage_ms
done
