#!/bin/bash
# Build libpgrt.so from the csrc/ and include/ of a git revision into ablib/<name>/ (objects under /tmp/pgrt_variants) (same-session
# A/B against the working tree: PGRT_LIB=ablib/<name>/libpgrt.so, tools/ab_libs.sh).
# usage: tools/build_commit.sh <rev> <name>
set -e
cd "$(dirname "$0")/.."
REV=$1; NAME=$2
OUT=/tmp/pgrt_variants/$NAME
rm -rf "$OUT"; mkdir -p "$OUT/csrc" "$OUT/include"
for f in $(git ls-tree --name-only "$REV" pgi_raytracing_amd/csrc/); do git show "$REV:$f" > "$OUT/csrc/$(basename $f)"; done
for f in $(git ls-tree --name-only "$REV" include/); do git show "$REV:$f" > "$OUT/include/$(basename $f)"; done
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -I$OUT/include -I$OUT/csrc"
OBJS=""
for src in "$OUT"/csrc/*.hip "$OUT"/csrc/*.cpp; do
  o="$OUT/$(basename "${src%.*}").o"
  # per-file flags of the revision's Makefile (HIPFLAGS_<name> := ...)
  extra=$(git show "$REV:Makefile" | sed -n "s/^HIPFLAGS_$(basename "${src%.*}") := //p")
  /opt/rocm/bin/hipcc $FLAGS $extra -c "$src" -o "$o" &
  OBJS="$OBJS $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OUT/libpgrt.so" $OBJS -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
mkdir -p ablib/$NAME && cp "$OUT/libpgrt.so" ablib/$NAME/
echo "ablib/$NAME/libpgrt.so"
