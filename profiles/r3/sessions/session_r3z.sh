# r3z (pass 2: spread8 = 7 of 8 blocks count on dummy words -- timing only):
# r3z: the level-0 shade without its slot allocation (timing only): noalloc0 = no allocation at
# all (slots from the ray index, no barriers), noatomic0 = the block allocation without its
# atomic (every block gets base 0: barriers and LDS kept)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3z
export PYTHONUNBUFFERED=1
for v in cur spread8 noatomic0 cur; do
  if [ $v = cur ]; then unset PGRT_LIB; else export PGRT_LIB=ablib/$v/libpgrt.so; fi
  for F in 8 1; do
    DIAG_FRAMES=$F timeout -k 10 120 python tools/diag.py 1920 1080 5 1 0 > gpurun_out/r3z/diag_${v}_$F.txt 2>&1 || { tail -5 gpurun_out/r3z/diag_${v}_$F.txt; exit 1; }
    echo "== $v F=$F: $(grep -E '^L0' gpurun_out/r3z/diag_${v}_$F.txt | sed -E 's/.*\| trace/trace/')"
  done
done
