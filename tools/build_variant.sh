#!/bin/bash
# Build libpgrt.so with one source file patched by a sed expression, for same-session A/B
# (load it with PGRT_LIB=build/<name>/libpgrt.so).  usage: tools/build_variant.sh <name> <src> <sed-expr>
set -e
cd "$(dirname "$0")/.."
NAME=$1; SRC=$2; EXPR=$3
OUT=build/$NAME
mkdir -p "$OUT"
sed "$EXPR" "pgi_raytracing_amd/csrc/$SRC" > "$OUT/$SRC"
OBJS=""
for f in trace render bvh ploc split bvh8; do
  if [ "$f.hip" = "$SRC" ]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off \
      -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude -Ipgi_raytracing_amd/csrc -c "$OUT/$SRC" -o "$OUT/$f.o"
    OBJS="$OBJS $OUT/$f.o"
  else
    OBJS="$OBJS build/$f.o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OUT/libpgrt.so" $OBJS build/context.o build/objloader.o \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "$OUT/libpgrt.so"
