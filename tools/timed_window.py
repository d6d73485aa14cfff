"""Timeline of bench.py's timed region from a rocprofv3 kernel trace of
`bench.py --no-cpu-baseline --no-roofline --steps K ...` (warmup calls first, then the K timed
frames, then the synchronous latency frames).  Calls end with one k_export_counters per slot.
usage: python tools/timed_window.py <kernel_trace.csv> <warmup_calls> <timed_calls>"""
import csv
import re
import sys


def short(name):
    m = re.match(r"(?:void )?(?:pgrt::)?(?:\(anonymous namespace\)::)?([A-Za-z_0-9]+)(<[^(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:30]


rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
              for r in csv.DictReader(open(sys.argv[1])))
wc, tc = int(sys.argv[2]), int(sys.argv[3])
ends = [e for s, e, n in rows if n == "k_export_counters"]
t_prev = ends[wc - 1]
t_end = ends[wc + tc - 1]
win = [r for r in rows if r[0] > t_prev and r[1] <= t_end]
t0 = min(r[0] for r in win)
print(f"timed window: {(t_end - t0) / 1e3:.1f} us, {len(win)} kernels, gap after warmup {(t0 - t_prev) / 1e3:.1f} us")
B = 100_000  # 100 us buckets
nb = (t_end - t0) // B + 1
busy = [0.0] * nb
for s, e, n in win:
    for b in range((s - t0) // B, (e - t0) // B + 1):
        lo, hi = max(s, t0 + b * B), min(e, t0 + (b + 1) * B)
        if hi > lo:
            busy[b] += (hi - lo) / B
print("kernel-concurrency per 100 us:", " ".join(f"{x:.1f}" for x in busy))
# the last 30 % of the window: what runs
tail0 = t0 + int((t_end - t0) * 0.7)
agg = {}
for s, e, n in win:
    if e > tail0:
        agg[n] = agg.get(n, 0) + (e - max(s, tail0)) / 1e3
print("last 30 %:", ", ".join(f"{k} {v:.0f}us" for k, v in sorted(agg.items(), key=lambda x: -x[1])))
# per call chain: start -> end of each call's kernels (by export order is not enough: list exports)
print("export ends (us from t0):", [round((e - t0) / 1e3) for e in ends[wc:wc + tc]])
