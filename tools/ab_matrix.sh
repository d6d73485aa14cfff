#!/bin/bash
# A/B matrix: libraries x bench argument sets, 3 runs each, ms per frame printed per cell.
# usage: tools/ab_matrix.sh <tag> "<lib1> <lib2> ..." "<args 1>" "<args 2>" ...
#   lib = "base" (the in-tree libpgrt.so), a path to a libpgrt.so (tools/build_commit.sh), or
#         "<name>:<ENV=value,...>" (the in-tree library under extra environment variables)
set -u
cd "$(dirname "$0")/.."
TAG=$1; LIBS=$2; shift 2
OUT=gpurun_out/ab_$TAG
mkdir -p "$OUT"
i=0
for A in "$@"; do
  i=$((i + 1))
  for L in $LIBS; do
    if [ "$L" = base ]; then name=base; envs=""
    elif [[ "$L" == *:* ]]; then name=${L%%:*}; envs=${L#*:}; envs=${envs//,/ }
    else name=$(basename "$(dirname "$L")"); envs="PGRT_LIB=$L"; fi
    for r in 1 2 3; do
      env $envs timeout -k 10 180 python3 bench.py --no-cpu-baseline --no-roofline $A \
        > "$OUT/s$i.$name.$r.json" 2> "$OUT/s$i.$name.err" || { tail -5 "$OUT/s$i.$name.err"; exit 1; }
    done
    python3 -c "import json; v=[json.load(open('$OUT/s$i.$name.%d.json'%r))['ms_per_step'] for r in (1,2,3)]; print('[$A] $name ms/frame', v)"
  done
done
