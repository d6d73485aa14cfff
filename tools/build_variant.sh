#!/bin/bash
# Build libpgrt.so from the working tree's csrc/ + include/ into ablib/<name>/ (objects under /tmp/pgrt_variants), optionally with one
# source file patched by a sed expression and/or extra compiler flags (EXTRA_FLAGS="-DFOO=1"), for
# same-session A/B (load it with PGRT_LIB=ablib/<name>/libpgrt.so, tools/ab_matrix.sh).
# usage: [EXTRA_FLAGS=...] tools/build_variant.sh <name> [<file in csrc/> <sed-expr>]
set -e
cd "$(dirname "$0")/.."
NAME=$1; SRC=${2:-}; EXPR=${3:-}
OUT=/tmp/pgrt_variants/$NAME
rm -rf "$OUT"; mkdir -p "$OUT/csrc" "$OUT/include"
cp pgi_raytracing_amd/csrc/* "$OUT/csrc/"
cp include/* "$OUT/include/"
if [ -n "$SRC" ]; then
  sed -i "$EXPR" "$OUT/csrc/$SRC"
  if cmp -s "$OUT/csrc/$SRC" "pgi_raytracing_amd/csrc/$SRC"; then echo "sed expression changed nothing" >&2; exit 1; fi
fi
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -I$OUT/include -I$OUT/csrc ${EXTRA_FLAGS:-}"
OBJS=""
for src in "$OUT"/csrc/*.hip "$OUT"/csrc/*.cpp; do
  base=$(basename "${src%.*}")
  o="$OUT/$base.o"
  extra=$(sed -n "s/^HIPFLAGS_$base := //p" Makefile)  # the Makefile's per-file flags
  /opt/rocm/bin/hipcc $FLAGS $extra -c "$src" -o "$o" &
  OBJS="$OBJS $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OUT/libpgrt.so" $OBJS -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
mkdir -p ablib/$NAME && cp "$OUT/libpgrt.so" ablib/$NAME/
echo "ablib/$NAME/libpgrt.so"
