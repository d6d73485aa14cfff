"""Frames-in-flight scan on one GPU: C2 throughput (ms/frame) for the whole frame and for one
rank's share of an N-GPU frame approximated by a 1080/N-row strip, at 1..4 frames in flight."""
import os
import sys
import time
from collections import deque

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
import scenes  # noqa: E402
from pgi_raytracing_amd import abi  # noqa: E402
from pgi_raytracing_amd.raytracer import Context, load_obj  # noqa: E402

sc = load_obj(scenes.AVENGER_OBJ)
sc.set_environment(os.path.join(ROOT, "assets", "spherical_map_windows.jpg"))
ctx = Context(0)
ctx.set_scene(sc)
W, H = 1920, 1080
ctx.set_camera(abi.default_camera(W, H))
fb = ctx.alloc(W * H * 16)
DS = [int(x) for x in os.environ.get("SCAN_DS", "1,2,3,4").split(",")]


def throughput(p, d, n=300):
    ctx.set_frames_in_flight(d)
    for rep in range(2):
        pend = deque()
        t = time.perf_counter()
        for _ in range(n if rep else 30):
            pend.append(ctx.render_device_async(p, fb))
            if len(pend) >= d:
                ctx.render_wait(pend.popleft())
        while pend:
            ctx.render_wait(pend.popleft())
        dt = time.perf_counter() - t
    return dt / n * 1e3


for n in (1, 2, 4, 8):
    rows = H // n
    p = abi.make_params(max_level=5, rect=(0, 0, W, rows) if n > 1 else (0, 0, 0, 0))
    print(f"share 1/{n}: " + " ".join(f"d{d} {throughput(p, d):.3f}" for d in DS), flush=True)

if os.environ.get("SCAN_SUBMIT"):  # host cost of one submission (no implicit waits: d frames)
    for n in (1, 8):
        rows = H // n
        p = abi.make_params(max_level=5, rect=(0, 0, W, rows) if n > 1 else (0, 0, 0, 0))
        ctx.set_frames_in_flight(4)
        sub, wt = [], []
        pend = deque()
        for i in range(200):
            t = time.perf_counter()
            pend.append(ctx.render_device_async(p, fb))
            sub.append(time.perf_counter() - t)
            if len(pend) >= 4:
                t = time.perf_counter()
                ctx.render_wait(pend.popleft())
                wt.append(time.perf_counter() - t)
        while pend:
            ctx.render_wait(pend.popleft())
        sub.sort()
        wt.sort()
        print(f"share 1/{n}: submit median {sub[100] * 1e3:.3f} ms, wait median {wt[len(wt) // 2] * 1e3:.3f} ms")
