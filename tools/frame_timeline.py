"""Device-stamped launch timeline of C2 frames (pgrt_timeline_enable; no rocprof, no HIP events).

Two workloads, each measured with the timeline OFF (host wall clock) and ON (device stamps):
  sync : one synchronous frame at a time (pgrt_render_device), the reference's Producer loop
         (APP/simpleguidx11.cpp:95-124) -- the frame latency
  r20  : the driver's timed region, `bench.py --steps 20`: 20 distinct frames as calls of 8 + 8 + 4
         frames, 8 calls in flight, after the same set-up and 5 warm-up frames

usage: python tools/frame_timeline.py [--out FILE] [--reps N] [--cfg field=value ...]
Prints one JSON object per workload: the host-timed figures with the timeline off and on, the
device span, and per launch (ordered by start) kind / level / slot / start / end in microseconds
relative to the first launch of the region."""
import argparse
import json
import os
import statistics
import sys
import time
from collections import deque

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:  # as bench.py (before HIP initialises)
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

import scenes  # noqa: E402
from pgi_raytracing_amd import abi  # noqa: E402
from pgi_raytracing_amd.raytracer import Context, load_obj  # noqa: E402

W, H, D = 1920, 1080, 5


def rel(recs, t0):
    return [dict(kind=r["kind"], level=r["level"], slot=r["slot"], ticket=r["ticket"], waves=r["waves"],
                 wave_us=r["wave_us"], last_in_us=r["last_in_us"],
                 start_us=round(r["us_start"] - t0, 2), end_us=round(r["us_end"] - t0, 2),
                 dur_us=round(r["us_end"] - r["us_start"], 2)) for r in sorted(recs, key=lambda r: r["start"])]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--cfg", action="append", default=[])
    ap.add_argument("--host", action="store_true", help="also frames to page-locked host memory (sync and async)")
    a = ap.parse_args()
    sc = load_obj(scenes.AVENGER_OBJ)
    sc.set_environment(os.path.join(ROOT, "assets", "spherical_map_windows.jpg"))
    ctx = Context(0)
    for kv in a.cfg:
        k, v = kv.split("=", 1)
        ctx.configure(**{k: float(v) if "." in v else int(v)})
    ctx.set_scene(sc)
    ctx.set_camera(abi.default_camera(W, H))
    base = abi.make_params(spp_side=1, max_level=D, jitter=abi.PGRT_JITTER_HASH)
    F, IN_FLIGHT = 8, 8
    call_bytes = F * W * H * 16
    fb = ctx.alloc(IN_FLIGHT * call_bytes)
    results = {}

    # ---- sync: one frame at a time ----
    def sync_frames(n, on):
        ctx.set_frames_in_flight(1)
        ctx.timeline_enable(on)
        lat = []
        for k in range(n):
            p = abi.RenderParams.from_buffer_copy(base)
            p.frame = 1000 + k
            t = time.perf_counter()
            ctx.render_device(p, fb)
            lat.append((time.perf_counter() - t) * 1e3)
        return lat

    sync_frames(5, False)
    lat_off = sync_frames(a.reps, False)
    ctx.timeline_read()
    lat_on = sync_frames(a.reps, True)
    recs = ctx.timeline_read()
    ctx.timeline_enable(False)
    by_ticket = {}
    for r in recs:
        by_ticket.setdefault(r["ticket"], []).append(r)
    spans = {t: (max(r["us_end"] for r in rs) - min(r["us_start"] for r in rs)) for t, rs in by_ticket.items()}
    med_t = sorted(spans, key=lambda t: spans[t])[len(spans) // 2]
    t0 = min(r["us_start"] for r in by_ticket[med_t])
    results["sync"] = {
        "workload": "C2 1920x1080 d=5 1 spp, one synchronous frame at a time (pgrt_render_device)",
        "host_ms_median_timeline_off": round(statistics.median(lat_off), 4),
        "host_ms_median_timeline_on": round(statistics.median(lat_on), 4),
        "device_span_ms_median": round(spans[med_t] / 1e3, 4),
        "device_span_ms_min": round(min(spans.values()) / 1e3, 4),
        "frames": len(spans),
        "launches": rel(by_ticket[med_t], t0),
    }

    # ---- sync_host / async_host: frames to page-locked host memory (SURVEY §8(d)'s ms/frame) ----
    if a.host:
        hb = ctx.host_array((H, W, 4))

        def sync_host(n, on):
            ctx.set_frames_in_flight(1)
            ctx.timeline_enable(on)
            lat = []
            for k in range(n):
                p = abi.RenderParams.from_buffer_copy(base)
                p.frame = 2000 + k
                t = time.perf_counter()
                ctx.render(p, out=hb)
                lat.append((time.perf_counter() - t) * 1e3)
            return lat

        sync_host(3, False)
        h_off = sync_host(a.reps, False)
        ctx.timeline_read()
        h_on = sync_host(a.reps, True)
        recs = ctx.timeline_read()
        ctx.timeline_enable(False)
        ctx.host_free(hb)
        by_ticket = {}
        for r in recs:
            by_ticket.setdefault(r["ticket"], []).append(r)
        spans = {t: (max(r["us_end"] for r in rs) - min(r["us_start"] for r in rs)) for t, rs in by_ticket.items()}
        med_t = sorted(spans, key=lambda t: spans[t])[len(spans) // 2]
        t0 = min(r["us_start"] for r in by_ticket[med_t])
        results["sync_host"] = {
            "workload": "C2, one synchronous frame at a time into a page-locked host framebuffer (pgrt_render)",
            "host_ms_median_timeline_off": round(statistics.median(h_off), 4),
            "host_ms_median_timeline_on": round(statistics.median(h_on), 4),
            "device_span_ms_median": round(spans[med_t] / 1e3, 4),
            "frames": len(spans),
            "launches": rel(by_ticket[med_t], t0),
        }
        ring = 4
        bufs = [ctx.host_array((F, H, W, 4)) for _ in range(ring)]
        ctx.set_frames_in_flight(ring)

        def host_calls(n, on):
            ctx.timeline_enable(on)
            pend = deque()
            t = time.perf_counter()
            for k in range(n):
                p = abi.RenderParams.from_buffer_copy(base)
                p.frame = 3000 + k * F
                pend.append(ctx.render_frames_host_async(p, F, bufs[k % ring]))
                if len(pend) >= ring:
                    ctx.render_wait(pend.popleft())
            while pend:
                ctx.render_wait(pend.popleft())
            return (time.perf_counter() - t) * 1e3

        host_calls(ring, False)
        dt_off = host_calls(12, False)
        ctx.timeline_read()
        dt_on = host_calls(12, True)
        recs = ctx.timeline_read()
        ctx.timeline_enable(False)
        for b in bufs:
            ctx.host_free(b)
        t0 = min(r["us_start"] for r in recs)
        results["async_host"] = {
            "workload": f"C2, 12 calls of {F} frames to page-locked host memory, {ring} in flight (pgrt_render_frames_host_async)",
            "ms_per_frame_timeline_off": round(dt_off / (12 * F), 4),
            "ms_per_frame_timeline_on": round(dt_on / (12 * F), 4),
            "launches": [r for r in rel(recs, t0) if r["kind"] in ("host_export", "finish", "trace_pkt", "export")],
        }

    # ---- r20: the driver's timed region ----
    ctx.set_frames_in_flight(IN_FLIGHT)
    nxt = [0]

    def run(n):
        pend = deque()
        sizes = [F] * (n // F) + ([n % F] if n % F else [])
        for k, nf in enumerate(sizes):
            p = abi.RenderParams.from_buffer_copy(base)
            p.frame = nxt[0]
            nxt[0] += nf
            pend.append(ctx.render_frames_device_async(p, nf, fb + (k % IN_FLIGHT) * call_bytes))
            if len(pend) >= IN_FLIGHT:
                ctx.render_wait(pend.popleft())
        while pend:
            ctx.render_wait(pend.popleft())

    def region(on):
        ctx.timeline_enable(on)
        run(IN_FLIGHT * F)  # set-up (every frame set allocated), as bench.py
        run(5)              # warm-up
        ctx.timeline_read()
        ctx.synchronize()
        t = time.perf_counter()
        run(20)
        ctx.synchronize()
        dt = (time.perf_counter() - t) * 1e3
        return dt, ctx.timeline_read()

    offs, ons, regs = [], [], []
    for _ in range(max(3, a.reps // 3)):
        offs.append(region(False)[0])
        dt, rr = region(True)
        ons.append(dt)
        regs.append(rr)
    ctx.timeline_enable(False)
    spans = [(max(r["us_end"] for r in rr) - min(r["us_start"] for r in rr)) / 1e3 for rr in regs]
    mi = sorted(range(len(spans)), key=lambda i: spans[i])[len(spans) // 2]
    rr = regs[mi]
    t0 = min(r["us_start"] for r in rr)
    calls = {}
    for r in rr:
        c = calls.setdefault(r["ticket"], [1e30, 0])
        c[0] = min(c[0], r["us_start"] - t0)
        c[1] = max(c[1], r["us_end"] - t0)
    results["r20"] = {
        "workload": "C2, bench.py --steps 20: calls of 8 + 8 + 4 distinct frames, 8 in flight",
        "host_ms_timeline_off": [round(x, 4) for x in offs],
        "host_ms_timeline_on": [round(x, 4) for x in ons],
        "host_ms_per_frame_off_median": round(statistics.median(offs) / 20, 5),
        "device_span_ms": [round(x, 4) for x in spans],
        "device_span_ms_per_frame_median": round(statistics.median(spans) / 20, 5),
        "calls_us": {str(k): [round(v[0], 1), round(v[1], 1)] for k, v in sorted(calls.items())},
        "launches": rel(rr, t0),
    }
    txt = json.dumps(results, indent=1)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(txt)
    for k, v in results.items():
        print(k, json.dumps({kk: vv for kk, vv in v.items() if kk != "launches"}))
        for r in v["launches"]:
            print(f"   {r['start_us']:9.1f} {r['end_us']:9.1f} {r['dur_us']:8.1f}  t{r['ticket']} s{r['slot']} "
                  f"{r['kind']:<13} L{r['level']:<3} waves {r['waves']:6d}  wave p50/p90/max "
                  f"{r['wave_us'][0]:6.1f} {r['wave_us'][1]:6.1f} {r['wave_us'][2]:6.1f}  last in {r['last_in_us']:6.1f}")


if __name__ == "__main__":
    main()
