set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
for v in vB vC vD; do for cfg in "48 36 5 2 1" "64 48 5 1 0"; do echo "== $v [$cfg]"; timeout -k 10 120 python tools/diff_libs.py ablib/base/libpgrt.so ablib/$v/libpgrt.so $cfg | head -2; done; done
