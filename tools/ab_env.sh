#!/bin/bash
# A/B of environment knobs on the bench workload: each argument is one setting
# ("PGRT_TAIL_RPW=16 PGRT_TAIL_MAX=200000"), run in its own process through tools/diag.py.
# usage: tools/ab_env.sh "SETTING A" "SETTING B" ...   (diag args via DIAG_ARGS)
cd "$(dirname "$0")/.."
for cfg in "$@"; do
  echo "### $cfg"
  env $cfg timeout -k 10 120 python tools/diag.py $DIAG_ARGS 2>&1 || exit $?
done
