"""Kernel sequence (name, us) of the last two uninstrumented render calls in a rocprofv3 kernel
trace (a call starts at k_raygen).  usage: python tools/call_seq.py <kernel_trace.csv>"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# a call starts at k_raygen, or at the level-0 packet traversal when it generates the rays itself
starts = [i for i, r in enumerate(rows)
          if "k_raygen" in r["Kernel_Name"]
          or ("k_trace_pkt" in r["Kernel_Name"] and (i == 0 or "k_raygen" not in rows[i - 1]["Kernel_Name"]))]
calls = []
for a, b in zip(starts, starts[1:] + [len(rows)]):
    seq = rows[a:b]
    if any("<true" in r["Kernel_Name"] and "k_trace" in r["Kernel_Name"] for r in seq):
        continue  # instrumented (profile=2) call
    calls.append(seq)
for seq in calls[-2:]:
    print(" ".join(f"{r['Kernel_Name'].split('(')[0].replace('void ', '').replace('pgrt::', '')[:18]}:"
                   f"{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:.0f}" for r in seq))
