#!/bin/bash
# frames-per-call x frames-in-flight scan of bench.py (C2 unless args given); one JSON line each
# usage: tools/fpc_scan.sh "<F list>" "<in-flight list>" [bench args...]
set -u
cd "$(dirname "$0")/.."
FS=$1; IFS_=$2; shift 2
for F in $FS; do
  for I in $IFS_; do
    timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-roofline --steps ${STEPS:-960} --frames-per-call $F --in-flight $I "$@" \
      > /tmp/fpc.json 2> /tmp/fpc.err || { cat /tmp/fpc.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('/tmp/fpc.json')); print(json.dumps({'F': $F, 'in_flight': $I, 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'latency': d['frame_latency_ms']}))"
  done
done
