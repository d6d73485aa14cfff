"""HIP API calls and kernels of the last synchronous frame of a rocprofv3 --hip-trace
--kernel-trace run of tools/sync_frames.py, on one clock (us after the frame's first API call).
usage: python tools/api_timeline.py <hip_api_trace.csv> <kernel_trace.csv>"""
import csv
import re
import sys


def short(name):
    m = re.match(r"(?:void )?(?:pgrt::)?(?:\(anonymous namespace\)::)?([A-Za-z_0-9]+)(<[^(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:30]


api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in csv.DictReader(open(sys.argv[1])))
ker = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
             for r in csv.DictReader(open(sys.argv[2])))
# frame boundaries: the end of each frame's k_export_counters kernel (its last launch)
ex = [k for k in ker if k[2] == "k_export_counters"]
t_prev_end = ex[-1 - int(sys.argv[3]) if len(sys.argv) > 3 else -3][1]
t_end = ex[-1][1] + 200_000
win_api = [a for a in api if t_prev_end < a[0] <= t_end]
win_k = [k for k in ker if t_prev_end < k[0] <= t_end]
t0 = t_prev_end
rows = [(s, e, "api", n) for s, e, n in win_api] + [(s, e, "GPU", n) for s, e, n in win_k]
rows.sort()
print(f"window: {(t_end - t0) / 1e3:.1f} us from the end of the previous frame's last kernel; {len(win_api)} API calls, {len(win_k)} kernels")
tot = {}
for s, e, n in win_api:
    tot[n] = tot.get(n, (0, 0.0))
    tot[n] = (tot[n][0] + 1, tot[n][1] + (e - s) / 1e3)
print("API totals:", ", ".join(f"{k} x{c} {v:.1f}us" for k, (c, v) in sorted(tot.items(), key=lambda x: -x[1][1])))
slow = [(e - s) / 1e3 for s, e, n in win_api if "Launch" in n and e - s > 20_000]
print(f"launch calls > 20 us: {len(slow)} ({sum(slow):.0f} us); launches {sum(1 for a in win_api if 'Launch' in a[2])}")
for s, e, kind, n in rows:
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {kind}  {n}")
