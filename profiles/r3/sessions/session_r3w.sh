# r3w: what bounds the bounce-level shades -- per-level shade time (diag, one 8-frame call) of
# the head vs timing-only variants: no environment lookup (miss colour = direction), no slot
# allocation on levels >= 1 (children / shadow slots from the ray index; level 2+ then empty)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3w
export PYTHONUNBUFFERED=1
for v in cur noenv noalloc; do
  if [ $v = cur ]; then unset PGRT_LIB; else export PGRT_LIB=ablib/$v/libpgrt.so; fi
  for F in 8 1; do
    DIAG_FRAMES=$F timeout -k 10 120 python tools/diag.py 1920 1080 5 1 0 > gpurun_out/r3w/diag_${v}_$F.txt 2>&1 || { tail -5 gpurun_out/r3w/diag_${v}_$F.txt; exit 1; }
    echo "== $v F=$F"; grep -E "^L[0-9]" gpurun_out/r3w/diag_${v}_$F.txt | sed -E 's/.*\| trace/trace/'
  done
done
