"""HBM traffic of the closest-hit launches from tools/profile.sh's PMC passes.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts half the bytes of wide
coalesced reads -> x2; WRITE_SIZE exact; both in KB (1024 B).  Reports the mean bytes per
closest-hit launch (k_trace / k_trace8g / k_trace8, every level and the shadow queue), the same
unit as bench.py's roofline `achieved`.

Also (optional passes) the VALU issue rate of the closest-hit launches: SQ_INSTS_VALU
(wave-instructions) x 2 cycles (a wave64 VALU instruction occupies a SIMD-32 for 2 cycles) over
the SIMD-cycles of the launch (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs), per kernel.

usage: python tools/traffic.py gpurun_out/prof_<tag> profiles/<r>/traffic_<cfg>.json <round> [workload]"""
import collections
import csv
import glob
import json
import os
import sys


def per_dispatch(path, counter):
    vals = collections.defaultdict(float)
    names = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] != counter:
                    continue
                vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
                names[r["Dispatch_Id"]] = r["Kernel_Name"]
    return vals, names


def main():
    root, out, rnd = sys.argv[1], sys.argv[2], sys.argv[3]
    workload = sys.argv[4] if len(sys.argv) > 4 else "C2 avenger-proxy 1920x1080 Whitted d=5 (bench.py default)"
    fetch, fn = per_dispatch(os.path.join(root, "pmc_fetch"), "FETCH_SIZE")
    write, wn = per_dispatch(os.path.join(root, "pmc_write"), "WRITE_SIZE")

    def trace_ids(names):  # the uninstrumented closest-hit launches (COUNT=false variants)
        return [d for d, n in names.items() if "k_trace" in n and "<true" not in n]

    # a budgeted bounce-level packet launch is followed by k_trace8g<..., RESUME = true> over its
    # deferred rays: bench.py times the pair as ONE closest-hit launch (launch_trace), so their
    # bytes are summed and the pair counted once
    def is_resume(n):
        return "k_trace8g" in n and ", true>" in n.split("(")[0]

    fids, wids = trace_ids(fn), trace_ids(wn)
    f_n = max(1, sum(1 for d in fids if not is_resume(fn[d])))
    w_n = max(1, sum(1 for d in wids if not is_resume(wn[d])))
    f_kb = sum(fetch[d] for d in fids) / f_n
    w_kb = sum(write[d] for d in wids) / w_n
    res = {
        "workload": workload,
        "kernel": "closest-hit launches (k_trace, k_trace8g), every level + shadow queue",
        "source": f"{root}: rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE, separate passes",
        "correction": "gfx950: FETCH_SIZE x2 (MI355X_MICROARCH.md HBM section); WRITE_SIZE as reported; KB=1024 B",
        "launches_fetch_pass": f_n,
        "launches_write_pass": w_n,
        "resume_launches_fetch_pass": len(fids) - f_n,
        "fetch_kb_per_launch": round(f_kb, 1),
        "write_kb_per_launch": round(w_kb, 1),
        "bytes_per_launch": int(round((2 * f_kb + w_kb) * 1024)),
        "round": rnd,
    }
    valu, vn = per_dispatch(os.path.join(root, "pmc_valu"), "SQ_INSTS_VALU")
    gui, _ = per_dispatch(os.path.join(root, "pmc_valu"), "GRBM_GUI_ACTIVE")
    if valu:
        by = collections.defaultdict(lambda: [0.0, 0.0, 0])
        for d in trace_ids(vn):
            k = vn[d].split("(")[0].split("<")[0].strip()
            by[k][0] += valu[d]
            by[k][1] += gui.get(d, 0.0)
            by[k][2] += 1
        res["valu_issue"] = {
            k: {"launches": n, "valu_insts_per_launch": round(v / n), "frac": round(2 * v / (1024 * g / 8), 4) if g else None}
            for k, (v, g, n) in by.items()}
        res["valu_issue_note"] = ("frac = SQ_INSTS_VALU x 2 cyc / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): the fraction of "
                                  "the chip's VALU issue slots the launch used (1.0 = every SIMD issuing a wave64 "
                                  "VALU instruction every 2 cycles)")
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
