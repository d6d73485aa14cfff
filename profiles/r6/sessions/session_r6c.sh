#!/bin/bash
# r6c: where a dependent traversal step's time goes (verdict r5 #1).
#  1. per-step record of the synchronous frame's ray-tree launch (diagnostics build, s_memtime stamps
#     around every 8-wide node step / triangle round and its loads, per tree: tools/step_profile.py)
#  2. one-lane per-level traversal diagnostics of one frame without the ray-tree launch (the deep
#     levels' longest ray: node / leaf / load cycles, tools/diag.py)
#  3. PMC of synchronous frames: L2 hit / miss and the SQ wait split per kernel launch
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PGRT_LIB=ablib/stepprof/libpgrt.so timeout -k 10 90 python3 tools/step_profile.py --out gpurun_out/step_profile_r6c.json > gpurun_out/step_profile_r6c.log 2>&1 || { tail -20 gpurun_out/step_profile_r6c.log; exit 1; }
head -c 3000 gpurun_out/step_profile_r6c.json
DIAG_CFG=subtree_level=-1 timeout -k 10 90 python3 tools/diag.py > gpurun_out/diag_r6c_one_lane.txt 2>&1 || { tail -20 gpurun_out/diag_r6c_one_lane.txt; exit 1; }
tail -8 gpurun_out/diag_r6c_one_lane.txt
OUT=gpurun_out/pmc_r6c
mkdir -p $OUT
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o p$i --output-format csv -- python3 tools/sync_frames.py 12 > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "=== pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -3 "$OUT/p$i.log"; exit 1; }
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt" 2>&1
grep -E "k_subtree|k_trace|k_shade" "$OUT/summary.txt" | head -40
# the bench line with the r6 roofline changes (level-0 byte charge from the launched kernels, frac rule)
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > gpurun_out/bench_r6c_C2_k20.json 2> gpurun_out/bench_r6c_C2_k20.err || { tail -5 gpurun_out/bench_r6c_C2_k20.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_r6c_C2_k20.json')); r=d['roofline']; print('driver line', d['ms_per_step'], 'lat', d.get('frame_latency_ms'), 'frac', r['frac'], r['frac_source'], r['level0_kernels'], r['level0_bytes_per_ray'], 'frame', r['frame']['frac'])"
for r in 1 2; do
  timeout -k 10 120 build/pg1_pgrt bench assets/avenger/6887_allied_avenger_proxy.obj assets/spherical_map_windows.jpg 20 5 > gpurun_out/cpp_dropin_r6c_k20_$r.json 2> gpurun_out/cpp_dropin_r6c.err || { tail -5 gpurun_out/cpp_dropin_r6c.err; exit 1; }
  cat gpurun_out/cpp_dropin_r6c_k20_$r.json
done
