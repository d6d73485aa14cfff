#!/bin/bash
# rocprofv3 passes over the THROUGHPUT run of bench.py (frames in flight; not the synchronous
# roofline calls): kernel trace, FETCH_SIZE, WRITE_SIZE -- then tools/throughput_breakdown.py.
# usage: tools/steady_profile.sh <tag> [bench args...]   (default: C2, 400 frames)
set -u
cd "$(dirname "$0")/.."
TAG=$1; shift
ARGS=${*:-"--steps 400"}
OUT=gpurun_out/steady_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for pass in trace fetch write; do
  case $pass in
    trace) P="--kernel-trace";;
    fetch) P="--kernel-trace --pmc FETCH_SIZE";;
    write) P="--kernel-trace --pmc WRITE_SIZE";;
  esac
  timeout -k 10 300 rocprofv3 $P -d "$OUT/$pass" -o $pass --output-format csv -- \
      python3 bench.py --no-cpu-baseline --no-roofline $ARGS > "$OUT/$pass.log" 2>&1
  rc=$?
  echo "=== $pass rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$pass.log"; exit $rc; fi
done
F=$(python3 -c "import json; print([json.loads(l) for l in open('$OUT/trace.log') if l.startswith('{\"metric')][-1]['frames_per_call'])")
python3 tools/throughput_breakdown.py "$(find $OUT/trace -name '*kernel_trace.csv' | head -1)" "$F" \
    "$(find $OUT/fetch -name '*counter_collection.csv' | head -1)" "$(find $OUT/write -name '*counter_collection.csv' | head -1)" \
    | tee "$OUT/breakdown.txt"
