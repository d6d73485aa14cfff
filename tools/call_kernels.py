"""List the kernels of each frame call in a rocprofv3 kernel trace (calls delimited by their
k_export_counters dispatch): per call, its launches in dispatch order with grid size and duration.
Finds e.g. AUTO probe launches (k_trace_pkt over kProbeRays = 65536 rays) inside timed calls.
usage: python tools/call_kernels.py <kernel_trace.csv> [first_call] [last_call]"""
import csv
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Dispatch_Id"]))
    lo = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    hi = int(sys.argv[3]) if len(sys.argv) > 3 else 10 ** 9
    call, out = 0, []
    for r in rows:
        name = r["Kernel_Name"]
        short = name.replace("void pgrt::", "").split("(")[0]
        if lo <= call <= hi:
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            out.append(f"call {call:3d}  {short:45s} grid {int(r.get('Grid_Size') or r['Grid_Size_X']):9d}  {dur:8.1f} us")
        if "k_export_counters" in name:
            call += 1
    print("\n".join(out))
    print(f"{call} calls")


if __name__ == "__main__":
    main()
