"""Summarise rocprofv3 --pmc counter CSVs (tools/pmc.sh): per kernel and grid size (a Whitted
level's launch), the mean of every counter over the profiled frames.

usage: python tools/pmc_summary.py gpurun_out/pmc_<tag>"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    m = re.match(r"(?:void )?(?:pgrt::)?(?:\(anonymous namespace\)::)?([A-Za-z_0-9]+)(<[^(]*>)?", name)
    b = m.group(1) if m else name[:40]
    return b + (m.group(2) if m and m.group(2) and b.startswith("k_trace") else "")


def main():
    root = sys.argv[1]
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        per = collections.defaultdict(dict)
        with open(f) as fh:
            for r in csv.DictReader(fh):
                key = (short(r["Kernel_Name"]), int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0))
                per[(r["Dispatch_Id"], key)][r["Counter_Name"]] = float(r["Counter_Value"])
        for (_, key), cs in per.items():
            for c, v in cs.items():
                vals[key][c].append(v)
    keys = sorted(vals, key=lambda k: (k[0], -k[1]))
    for k in keys:
        if not k[0].startswith(("k_", "rocprim")):
            continue
        items = " ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(vals[k].items()))
        print(f"{k[0]:28s} grid {k[1]:9d}: {items}")


if __name__ == "__main__":
    main()
