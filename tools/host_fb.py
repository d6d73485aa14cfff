"""Host-framebuffer figures of C2 (pgrt_render to the framebuffer in host memory):
synchronous frames into page-locked memory (median of --reps after 3 warm-ups) and the throughput
of pgrt_render_frames_host_async for each (frames per call, calls in flight) given.  A/B tool:
PGRT_LIB selects the library.

usage: python tools/host_fb.py [--reps 20] [--async 8x4 2x4 ...]"""
import argparse
import json
import os
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

W, H = 1920, 1080


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--async", dest="asy", nargs="*", default=["8x4"])
    ap.add_argument("--frames", type=int, default=96, help="frames per async measurement")
    ap.add_argument("--cfg", action="append", default=[], help="pgrt_config field=value")
    ap.add_argument("--modes", type=int, nargs="*", default=[], help="host_export values, one process")
    ap.add_argument("--rounds", type=int, default=1, help="passes over --modes")
    a = ap.parse_args()
    sc = load_obj(scenes.AVENGER_OBJ)
    sc.set_environment(os.path.join(ROOT, "assets", "spherical_map_windows.jpg"))
    ctx = Context(0)
    for kv in a.cfg:
        k, v = kv.split("=", 1)
        ctx.configure(**{k: int(v)})
    ctx.set_scene(sc)
    ctx.set_camera(abi.default_camera(W, H))
    p = abi.make_params(max_level=5)
    out = {"lib": os.environ.get("PGRT_LIB", "in-tree"), "cfg": a.cfg}
    # --modes: host_export values measured in THIS process, interleaved over --rounds (a process's
    # SDMA rate varies from run to run on the same box: 27 or 54 GB/s, profiles/r5/r5l)
    modes = a.modes if a.modes else [None]
    for rnd in range(a.rounds):
        for m in modes:
            key = "" if m is None else f"m{m}_"
            if m is not None:
                ctx.configure(host_export=m)
            hb = ctx.host_array((H, W, 4))
            ctx.set_frames_in_flight(1)
            for _ in range(3):
                ctx.render(p, out=hb)
            lat = []
            for _ in range(a.reps):
                t = time.perf_counter()
                ctx.render(p, out=hb)
                lat.append((time.perf_counter() - t) * 1e3)
            ctx.host_free(hb)
            out.setdefault(f"{key}sync_ms_median", []).append(round(sorted(lat)[len(lat) // 2], 4))
            for spec in a.asy:
                F, ring = map(int, spec.split("x"))
                bufs = [ctx.host_array((F, H, W, 4)) for _ in range(ring)]
                ctx.set_frames_in_flight(ring)

                def calls(n):
                    pend = deque()
                    for k in range(n):
                        pend.append(ctx.render_frames_host_async(p, F, bufs[k % ring]))
                        if len(pend) >= ring:
                            ctx.render_wait(pend.popleft())
                    while pend:
                        ctx.render_wait(pend.popleft())

                calls(ring)
                n = max(2 * ring, a.frames // F)
                t = time.perf_counter()
                calls(n)
                dt = time.perf_counter() - t
                for b in bufs:
                    ctx.host_free(b)
                out.setdefault(f"{key}async_{F}x{ring}_ms_per_frame", []).append(round(dt / (n * F) * 1e3, 4))
    for k, v in list(out.items()):
        if isinstance(v, list) and len(v) == 1 and k not in ("cfg",):
            out[k] = v[0]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
