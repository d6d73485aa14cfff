#!/bin/bash
# One GPU session: parity tests, smoke, short bench.  Each GPU step has its own time limit;
# a crash/fault/timeout (exit >= 124 or signals) stops the session, plain test failures
# (pytest exit 1) do not.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() {  # name limit cmd...
    local name=$1 limit=$2
    shift 2
    echo "=== $name" | tee -a gpurun_out/session.log
    timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a gpurun_out/session.log
    tail -5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping: $name exited with $rc" | tee -a gpurun_out/session.log
        exit $rc
    fi
    return 0
}
rocm-smi --showproductname > gpurun_out/rocm_smi.log 2>&1 || true
for s in "$@"; do
    case $s in
        tests) step gpu_tests 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
        tests_all) step gpu_tests_all 1200 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
        smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) step bench 600 python bench.py --steps 20 --warmup 3 ;;
        bench_quick) step bench_quick 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ;;
        diag) step diag 300 python tools/diag.py ;;
        # the driver's line (--steps 20 --warmup 5), distinct frames (the default) and the r2
        # identical-frame workload (A/B), and the long default run of each
        bench_driver) step bench_driver 600 python bench.py --steps 20 --warmup 5 ;;
        bench_ident) step bench_ident 300 python bench.py --steps 20 --warmup 5 --frames identical --no-cpu-baseline ;;
        bench_long) step bench_long 300 python bench.py --no-cpu-baseline ;;
        bench_long_ident) step bench_long_ident 300 python bench.py --no-cpu-baseline --frames identical ;;
        # device-stamped launch timeline: one synchronous frame and the driver's 20-frame region
        timeline) step timeline 300 python tools/frame_timeline.py --out gpurun_out/timeline.json ;;
        bench_nocpu) step bench_nocpu 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
