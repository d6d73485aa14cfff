# r3i: round-3 evidence -- rocprofv3 kernel stats + PMC traffic passes for C2 and C3
set -u
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/profile.sh r3 C2 || exit 1
bash tools/profile.sh r3 C3 || exit 1
ls gpurun_out/prof_r3_C2 gpurun_out/prof_r3_C3
