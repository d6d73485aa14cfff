"""Kernel-by-kernel timeline of bench.py's timed region from a rocprofv3 kernel trace (the
format of profiles/r2/c2_driver_style_timeline_r2k.txt): start / end / duration in us after the
previous call's last kernel, hardware queue, kernel, grid size.
usage: python tools/timeline.py <kernel_trace.csv> <warmup_calls> <timed_calls>"""
import csv
import re
import sys


def short(name):
    m = re.match(r"(?:void )?(?:pgrt::)?(?:\(anonymous namespace\)::)?([A-Za-z_0-9]+)(<[^(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:30]


def main():
    rows = []
    for r in csv.DictReader(open(sys.argv[1])):
        grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                     r.get("Queue_Id", "?"), grid))
    rows.sort()
    wc, tc = int(sys.argv[2]), int(sys.argv[3])
    ends = [e for s, e, n, q, g in rows if n == "k_export_counters"]
    t_prev = ends[wc - 1]
    t_end = ends[wc + tc - 1]
    win = [r for r in rows if r[0] > t_prev and r[1] <= t_end]
    print(f"window {(t_end - t_prev) / 1e3:.1f} us after the previous call's last kernel, {len(win)} kernels")
    print(f"{'start':>8} {'end':>8} {'dur':>7}  queue  kernel  grid")
    for s, e, n, q, g in win:
        print(f"{(s - t_prev) / 1e3:8.1f} {(e - t_prev) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  q{q:<4} {n}  {g}")


if __name__ == "__main__":
    main()
