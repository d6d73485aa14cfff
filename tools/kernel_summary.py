"""Summarise a rocprofv3 kernel trace (``*_kernel_trace.csv``) of bench.py.

Prints per-kernel totals and, for the render pipeline, the average duration of each launch
position inside a frame (frame = the kernels between two k_raygen dispatches), so per-level
trace / shade costs and the idle gaps between launches are visible.

usage: python tools/kernel_summary.py gpurun_out/kt/kt_kernel_trace.csv [frames_to_skip]
"""
import collections
import csv
import re
import sys


def short(name: str) -> str:
    m = re.match(r"(?:void )?(?:pgrt::)?(?:\(anonymous namespace\)::)?([A-Za-z_0-9]+)(<[^(]*>)?", name)
    base = m.group(1) if m else name[:40]
    if m and m.group(2) and base == "k_trace":
        base += m.group(2)
    return base


def main():
    path = sys.argv[1]
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))))
    rows.sort()
    tot = collections.defaultdict(lambda: [0, 0.0])
    for s, e, n, _ in rows:
        tot[n][0] += 1
        tot[n][1] += (e - s) / 1e3
    print("kernel totals (us):")
    for n, (c, t) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:15]:
        print(f"  {n:40s} calls {c:5d} total {t:10.1f} avg {t / c:8.2f}")
    frames, cur = [], None
    for r in rows:
        if r[2] == "k_raygen":
            if cur:
                frames.append(cur)
            cur = [r]
        elif cur is not None:
            cur.append(r)
    if cur:
        frames.append(cur)
    frames = [f for f in frames[skip:] if len(f) == len(frames[-1])]
    if not frames:
        return
    n = len(frames[0])
    print(f"\nper-launch position, {len(frames)} frames (us; gap = idle before the launch):")
    for k in range(n):
        d = sum((f[k][1] - f[k][0]) for f in frames) / len(frames) / 1e3
        g = sum((f[k][0] - f[k - 1][1]) for f in frames) / len(frames) / 1e3 if k else 0.0
        print(f"  {k:2d} {frames[0][k][2]:34s} grid {frames[0][k][3]:6d} dur {d:8.2f} gap {g:6.2f}")
    span = sum((f[-1][1] - f[0][0]) for f in frames) / len(frames) / 1e3
    print(f"  frame span (raygen start -> last end) {span:.1f} us")


if __name__ == "__main__":
    main()
