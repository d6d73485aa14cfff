#!/bin/bash
# r4c: where does the r3-head -> r4 C2 regression come from: same-box A/B with the stamps compiled
# out, then per-kernel rocprofv3 stats of the driver's line for r3 head and the r4 library
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_pair.sh r4c ablib/r3head/libpgrt.so ablib/nostamp/libpgrt.so 3 || exit 1
bash tools/ab_pair.sh r4c2 ablib/nocache/libpgrt.so ablib/nostamp/libpgrt.so 2 || exit 1
for L in r3head nocache; do
  PGRT_LIB=ablib/$L/libpgrt.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$L -o kt --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-roofline --steps 200 --warmup 5 > gpurun_out/kt_$L.log 2>&1 || { tail -5 gpurun_out/kt_$L.log; exit 1; }
  f=$(find gpurun_out/kt_$L -name "*kernel_stats.csv" | head -1)
  echo "== $L $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/kt_$L.log)"
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:16]:
    print('%-70s calls %6s avg %9.1f us total %9.1f ms'%(r['Name'][:70],r['Calls'],float(r['AverageNs'])/1e3,float(r['TotalDurationNs'])/1e6))
"
done
