"""Kernel sequence (name, us) of the last two uninstrumented render calls in a rocprofv3 kernel
trace (a call ends at k_export_counters; instrumented profile=2 calls are skipped).
usage: python tools/call_seq.py <kernel_trace.csv>"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
calls, cur = [], []
for r in rows:
    name = r["Kernel_Name"]
    if not any(k in name for k in ("k_trace", "k_shade", "k_env", "k_finish", "k_combine", "k_raygen", "k_export")):
        continue
    cur.append(r)
    if "k_export_counters" in name:
        if not any("<true" in x["Kernel_Name"] and "k_trace" in x["Kernel_Name"] for x in cur):
            calls.append(cur)
        cur = []
for seq in calls[-2:]:
    tot = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seq) / 1e3
    print(f"[sum {tot:.0f} us] " + " ".join(
        f"{r['Kernel_Name'].split('(')[0].replace('void ', '').replace('pgrt::', '')[:18]}:"
        f"{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:.0f}" for r in seq))
