#!/bin/bash
# Host-side sanitizer run: the CPU test files that drive libpgrt's host C++ (OBJ
# loader, tile deal / unpack, argument validation of the C ABI) and the oracle (CPU restatement),
# against the AddressSanitizer + UndefinedBehaviorSanitizer build of both (`make asan`: every host
# translation unit of libpgrt.so, and oracle.c).  Any report aborts the run.  No GPU needed; the
# log goes to ${1:-profiles/r5/asan_check.log}.
set -u
cd "$(dirname "$0")/.."
LOG=${1:-profiles/r5/asan_check.log}
mkdir -p "$(dirname "$LOG")"
make asan -j8 > /dev/null || exit 1
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
{
  echo "# make asan: build/asan/libpgrt.so (host TUs: -fsanitize=address,undefined -fno-sanitize-recover=all), build/asan/liboracle*.so"
  echo "# runtime: $RT"
  echo "# $(date -u +%FT%TZ) $(git rev-parse --short HEAD 2>/dev/null)"
} > "$LOG"
env LD_PRELOAD="$RT" ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 \
    UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 PGRT_LIB=build/asan/libpgrt.so ORACLE_LIB_DIR=build/asan \
    timeout -k 10 1200 python -m pytest tests/test_abi.py tests/test_oracle.py tests/test_golden.py \
    tests/test_tiles_gloo.py tests/test_obj_corpus.py -m "not gpu" -v -p no:cacheprovider >> "$LOG" 2>&1
rc=$?
tail -3 "$LOG"
grep -E "ERROR: AddressSanitizer|runtime error:" "$LOG" | head -5
exit $rc
