"""Steady-state per-kernel breakdown of a bench.py throughput run (frames in flight) from a
rocprofv3 kernel trace, optionally with PMC counter CSVs of separate passes of the same command.

Window: the middle 80 % of the trace's render calls (a call ends with one k_export_counters per
pipeline slot); per kernel: launches, device us per frame (durations overlap across calls in
flight, so the column sums above the wall time), and, when given, HBM-side bytes per frame
(FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md's gfx950 correction).
Further counter CSVs (extra arguments after fetch / write) are reported per kernel as the counter
per frame (mean per launch x launches per frame), e.g. SQ_INSTS_VALU: wave-instructions per frame.
usage: python tools/throughput_breakdown.py <kernel_trace.csv> <frames_per_call> [fetch.csv write.csv [more.csv ...]]"""
import collections
import csv
import re
import sys


def short(name):
    m = re.match(r"(?:void )?(?:pgrt::)?(?:\(anonymous namespace\)::)?([A-Za-z_0-9]+)(<[^(]*>)?", name)
    base = m.group(1) if m else name[:40]
    return base + (m.group(2) if m and m.group(2) else "")


def load_trace(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         r.get("Dispatch_Id")))
    rows.sort()
    return rows


def load_pmc(path, counter=None):
    """counter given: {kernel: [per-dispatch values]}; else {counter: {kernel: [values]}}"""
    per = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    with open(path) as f:
        for r in csv.DictReader(f):  # one row per dispatch x counter (x instance: summed)
            per[r["Counter_Name"]][short(r["Kernel_Name"])][r["Dispatch_Id"]] += float(r["Counter_Value"])
    out = {c: {k: list(d.values()) for k, d in kd.items()} for c, kd in per.items()}
    return out.get(counter, {}) if counter else out


def main():
    rows = load_trace(sys.argv[1])
    F = int(sys.argv[2])
    ends = [e for s, e, n, _ in rows if n == "k_export_counters"]
    if len(ends) < 10:
        print("too few calls in the trace")
        return
    lo, hi = ends[len(ends) // 10], ends[len(ends) * 9 // 10]
    calls = sum(1 for e in ends if lo < e <= hi)
    frames = calls * F
    win = [r for r in rows if r[0] >= lo and r[1] <= hi]
    wall = (hi - lo) / 1e3
    per = collections.defaultdict(lambda: [0, 0.0])
    for s, e, n, _ in win:
        per[n][0] += 1
        per[n][1] += (e - s) / 1e3
    busy, cur_s, cur_e = 0.0, None, None  # union of kernel intervals
    for s, e, _, _ in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    fetch = write = None
    if len(sys.argv) > 4:
        fetch = load_pmc(sys.argv[3], "FETCH_SIZE")
        write = load_pmc(sys.argv[4], "WRITE_SIZE")
    print(f"window {wall:.1f} us, {calls} calls x {F} frames = {frames} frames: {wall / frames:.4f} ms/frame wall "
          f"(x1e3 us), device busy (union) {busy / 1e3 / wall * 100:.1f} %")
    tot = sum(t for _, t in per.values())
    print(f"{'kernel':40s} {'launch':>7s} {'us/frame':>9s} {'share':>6s}" + ("  MB/frame (2F+W)" if fetch else ""))
    for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        line = f"{n:40s} {c:7d} {t / frames:9.2f} {t / tot * 100:5.1f}%"
        if fetch and n in fetch:
            # counters are from separate runs: mean KB per launch x launches per frame
            f_kb = sum(fetch[n]) / len(fetch[n])
            w_kb = sum(write.get(n, [0])) / max(1, len(write.get(n, [1])))
            line += f"  {(2 * f_kb + w_kb) * 1024 * c / frames / 1e6:8.1f}"
        print(line)
    print(f"{'sum of kernel durations':40s} {'':7s} {tot / frames:9.2f}")
    for extra in sys.argv[5:]:
        for counter, kd in sorted(load_pmc(extra).items()):
            print(f"\n{counter} per frame (launch-weighted):")
            total = 0.0
            for n, (c, _) in sorted(per.items(), key=lambda kv: -kv[1][1]):
                if n in kd:
                    v = sum(kd[n]) / len(kd[n]) * c / frames
                    total += v
                    print(f"  {n:40s} {v:14.4g}")
            print(f"  {'total':40s} {total:14.4g}")


if __name__ == "__main__":
    main()
