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


def frame_calls(names, calls=5):
    """Dispatch ids of the bench's profile=1 roofline calls: every call ends with ONE
    k_export_counters per pipeline slot (one slot with frames in flight); --roofline-only runs
    warm-up calls, `calls` profile=1 calls, then one profile=2 (instrumented) call -- the segments
    before the last one, the last `calls` of them."""
    ids = sorted(names, key=lambda d: int(d))
    segs, cur = [], []
    for d in ids:
        cur.append(d)
        if "k_export_counters" in names[d]:
            segs.append(cur)
            cur = []
    return segs[-1 - calls:-1] if len(segs) > calls else []


def frame_bytes(fetch, fn, write, wn, frames_per_call, calls=5):
    """Whole-frame DRAM bytes (every kernel of a call: traces, shades, combines, finish, counter
    export) per frame, from the profile=1 calls; the per-kind split too."""
    fsegs, wsegs = frame_calls(fn, calls), frame_calls(wn, calls)
    if not fsegs or not wsegs:
        return None
    kind = lambda n: n.split("(")[0].split("<")[0].replace("void pgrt::", "").strip()
    by = collections.defaultdict(float)
    tot_f = sum(fetch[d] for s in fsegs for d in s)
    tot_w = sum(write[d] for s in wsegs for d in s)
    for s in fsegs:
        for d in s:
            by[kind(fn[d])] += 2 * fetch[d]
    for s in wsegs:
        for d in s:
            by[kind(wn[d])] += write[d]
    frames = frames_per_call * len(fsegs)
    return {
        "bytes_per_frame": int(round((2 * tot_f / len(fsegs) + tot_w / len(wsegs)) * 1024 / frames_per_call)),
        "fetch_bytes_per_frame": int(round(2 * tot_f * 1024 / frames)),
        "write_bytes_per_frame": int(round(tot_w * 1024 * len(fsegs) / len(wsegs) / frames)),
        "calls": len(fsegs), "frames_per_call": frames_per_call,
        "by_kernel_bytes_per_frame": {k: int(round(v * 1024 / frames)) for k, v in sorted(by.items(), key=lambda x: -x[1])},
    }


def roofline_kernel_trace(root, calls, out):
    """The trace pass's closest-hit launches of exactly the profile=1 roofline calls: written to
    <out>_kernel_trace.csv (one row per launch as bench.py times it -- a budgeted packet launch and
    its k_trace8g<RESUME> deferral launch are one row, from the first's start to the second's
    end), their average duration beside the bench's own avg_launch_ms (HIP events, same run)."""
    files = glob.glob(os.path.join(root, "trace", "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        return None
    rows = {}
    with open(files[0]) as fh:
        for r in csv.DictReader(fh):
            rows[r["Dispatch_Id"]] = r
    names = {d: r["Kernel_Name"] for d, r in rows.items()}
    segs = frame_calls(names, calls)
    if not segs:
        return None
    is_trace = lambda n: ("k_trace" in n and "<true" not in n) or (
        "k_subtree" in n and n.split("(")[0].rstrip().endswith("false>"))
    is_resume = lambda n: "k_trace8g" in n and ", true>" in n.split("(")[0]
    launches = []
    for seg in segs:
        for d in sorted(seg, key=int):
            n = names[d]
            if not is_trace(n):
                continue
            t0, t1 = int(rows[d]["Start_Timestamp"]), int(rows[d]["End_Timestamp"])
            if is_resume(n) and launches:
                launches[-1]["end"] = t1  # the deferral launch of the packet launch before it
                launches[-1]["kernels"] += " + " + n.split("(")[0]
                continue
            launches.append({"dispatch": d, "kernels": n.split("(")[0], "start": t0, "end": t1})
    path = os.path.splitext(out)[0] + "_kernel_trace.csv"
    with open(path, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["dispatch", "kernels", "start_ns", "end_ns", "duration_us"])
        for l in launches:
            w.writerow([l["dispatch"], l["kernels"], l["start"], l["end"], round((l["end"] - l["start"]) / 1e3, 3)])
    avg_ms = sum(l["end"] - l["start"] for l in launches) / len(launches) / 1e6
    res = {"csv": os.path.basename(path), "calls": len(segs), "launches": len(launches),
           "launches_per_call": round(len(launches) / len(segs), 2), "avg_launch_ms": round(avg_ms, 4)}
    logp = os.path.join(root, "trace.log")
    if os.path.exists(logp):  # bench.py --roofline-only's own line in the same (traced) run
        for line in open(logp):
            if line.startswith('{"metric'):
                b = json.loads(line).get("roofline") or {}
                if b.get("avg_launch_ms"):
                    res["bench_avg_launch_ms_same_run"] = b["avg_launch_ms"]
                    res["rocprof_vs_bench"] = round(avg_ms / b["avg_launch_ms"], 4)
    return res


def main():
    root, out, rnd = sys.argv[1], sys.argv[2], sys.argv[3]
    workload = sys.argv[4] if len(sys.argv) > 4 else "C2 avenger-proxy 1920x1080 Whitted d=5 (bench.py default)"
    fetch, fn = per_dispatch(os.path.join(root, "pmc_fetch"), "FETCH_SIZE")
    write, wn = per_dispatch(os.path.join(root, "pmc_write"), "WRITE_SIZE")

    def trace_ids(names):  # the uninstrumented closest-hit launches (COUNT=false variants)
        # (k_subtree: the deep levels' closest hits + their shading in one launch, timed by
        # bench.py as a closest-hit launch; its <int, bool, false> variants are uninstrumented)
        return [d for d, n in names.items() if ("k_trace" in n and "<true" not in n)
                or ("k_subtree" in n and n.split("(")[0].rstrip().endswith("false>"))]

    # a budgeted bounce-level packet launch is followed by k_trace8g<..., RESUME = true> over its
    # deferred rays: bench.py times the pair as ONE closest-hit launch (launch_trace), so their
    # bytes are summed and the pair counted once
    def is_resume(n):
        return "k_trace8g" in n and ", true>" in n.split("(")[0]

    # only the bench's profile=1 roofline calls (the segments frame_calls picks), so the bytes
    # per launch describe exactly the launches bench.py's avg_launch_ms times
    calls = int(os.environ.get("ROOF_CALLS", "5"))
    in_calls = lambda names: {d for seg in frame_calls(names, calls) for d in seg}
    fsel, wsel = in_calls(fn), in_calls(wn)
    fids = [d for d in trace_ids(fn) if d in fsel]
    wids = [d for d in trace_ids(wn) if d in wsel]
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
        vsel = in_calls(vn)
        for d in [d for d in trace_ids(vn) if d in vsel]:
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
    # bench.py --roofline-only: F frames per call (8 for C2, 1 for C3-C5), 5 profile=1 calls for
    # C2 and 2 for the others (its `reps`)
    fpc = int(os.environ.get("FRAMES_PER_CALL", "8"))
    fr = frame_bytes(fetch, fn, write, wn, fpc, int(os.environ.get("ROOF_CALLS", "5")))
    if fr:
        res["frame"] = fr
        res["frame_note"] = ("every kernel of the profile=1 roofline calls (FETCH_SIZE x2 + WRITE_SIZE), per frame; "
                             "calls delimited by their k_export_counters dispatch")
    kt = roofline_kernel_trace(root, calls, out)
    if kt:
        res["kernel_trace"] = kt
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
