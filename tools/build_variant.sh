#!/bin/bash
# Build libpgrt.so with one source file (or header) patched by a sed expression, for same-session
# A/B (load it with PGRT_LIB=build/<name>/libpgrt.so).
# usage: tools/build_variant.sh <name> <file in csrc/> <sed-expr>
set -e
cd "$(dirname "$0")/.."
NAME=$1; SRC=$2; EXPR=$3
OUT=build/$NAME
rm -rf "$OUT"; mkdir -p "$OUT/csrc"
cp pgi_raytracing_amd/csrc/* "$OUT/csrc/"
sed -i "$EXPR" "$OUT/csrc/$SRC"
if cmp -s "$OUT/csrc/$SRC" "pgi_raytracing_amd/csrc/$SRC"; then echo "sed expression changed nothing" >&2; exit 1; fi
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude -I$OUT/csrc"
OBJS=""
for f in trace render bvh ploc split bvh8 context objloader; do
  ext=hip; [ -f "$OUT/csrc/$f.cpp" ] && ext=cpp
  /opt/rocm/bin/hipcc $FLAGS -c "$OUT/csrc/$f.$ext" -o "$OUT/$f.o" &
  OBJS="$OBJS $OUT/$f.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OUT/libpgrt.so" $OBJS -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "$OUT/libpgrt.so"
