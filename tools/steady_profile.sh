#!/bin/bash
# rocprofv3 passes over the THROUGHPUT run of bench.py (frames in flight; not the synchronous
# roofline calls, and without the synchronous latency frames after the timed region: their
# per-slot k_export_counters would count as calls in the breakdown's window -- fixed in r6): kernel trace, FETCH_SIZE, WRITE_SIZE -- then tools/throughput_breakdown.py.
# usage: tools/steady_profile.sh <tag> [bench args...]   (default: C2, 400 frames)
set -u
cd "$(dirname "$0")/.."
TAG=$1; shift
ARGS=${*:-"--steps 400"}
OUT=gpurun_out/steady_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for pass in trace fetch write sq sq2; do
  case $pass in
    trace) P="--kernel-trace";;
    fetch) P="--kernel-trace --pmc FETCH_SIZE";;
    write) P="--kernel-trace --pmc WRITE_SIZE";;
    sq) P="--kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_LDS GRBM_GUI_ACTIVE";;
    sq2) P="--kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC";;
  esac
  timeout -k 10 300 rocprofv3 $P -d "$OUT/$pass" -o $pass --output-format csv -- \
      python3 bench.py --no-cpu-baseline --no-roofline --no-latency $ARGS > "$OUT/$pass.log" 2>&1
  rc=$?
  echo "=== $pass rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$pass.log"; exit $rc; fi
done
F=$(python3 -c "import json; print([json.loads(l) for l in open('$OUT/trace.log') if l.startswith('{\"metric')][-1]['frames_per_call'])")
python3 tools/throughput_breakdown.py "$(find $OUT/trace -name '*kernel_trace.csv' | head -1)" "$F" \
    "$(find $OUT/fetch -name '*counter_collection.csv' | head -1)" "$(find $OUT/write -name '*counter_collection.csv' | head -1)" \
    "$(find $OUT/sq -name '*counter_collection.csv' | head -1)" "$(find $OUT/sq2 -name '*counter_collection.csv' | head -1)" \
    | tee "$OUT/breakdown.txt"
