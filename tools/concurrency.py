"""Device concurrency of a rocprofv3 kernel trace (frames in flight): union-busy fraction of the
window, time-weighted mean number of kernels resident, and per-kernel summed durations.

usage: python tools/concurrency.py <kernel_trace.csv> [skip_fraction]
"""
import collections
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from kernel_summary import short  # noqa: E402


def main():
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.3
    rows = rows[int(len(rows) * skip):]  # drop build / warmup
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    ev = []
    for s, e, _ in rows:
        ev.append((s, 1))
        ev.append((e, -1))
    ev.sort()
    busy = 0
    weighted = 0
    cur = 0
    last = t0
    hist = collections.Counter()
    for t, d in ev:
        if cur > 0:
            busy += t - last
        weighted += cur * (t - last)
        hist[min(cur, 8)] += t - last
        cur += d
        last = t
    span = t1 - t0
    print(f"window {span / 1e6:.3f} ms, {len(rows)} kernels, busy {busy / span:.3f}, "
          f"mean resident kernels {weighted / span:.2f}")
    print("time with k kernels resident: " + " ".join(f"{k}:{hist[k] / span:.2f}" for k in sorted(hist)))
    tot = collections.defaultdict(lambda: [0, 0])
    for s, e, n in rows:
        tot[n][0] += e - s
        tot[n][1] += 1
    for n, (d, c) in sorted(tot.items(), key=lambda x: -x[1][0]):
        print(f"{n:32s} n={c:6d} sum {d / 1e6:9.3f} ms avg {d / c / 1e3:8.1f} us")


if __name__ == "__main__":
    main()
