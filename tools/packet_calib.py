"""Calibration of the automatic packet / one-lane choice per Whitted level (GPU).

For C2 (avenger-proxy 1920x1080 d=5, 8 frames per call) and C5 (10^6 random triangles, 4096^2,
d=8): every level traced as wave packets (packet_levels 16) vs only level 0 (packet_levels 1:
deeper levels one lane -- or 8 lanes -- per ray), per-level closest-hit ms (profile 1, median of
reps) and the packet utilisation of every level (FrameCounters::pkt, sampled blocks).
usage: python tools/packet_calib.py [C2|C5 ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]

import scenes  # noqa: E402
from pgi_raytracing_amd import abi  # noqa: E402
from pgi_raytracing_amd.raytracer import Context, load_obj  # noqa: E402


def run(cfg):
    env = os.path.join(ROOT, "assets", "spherical_map_windows.jpg")
    ctx = Context(0)
    if cfg == "C5":
        ctx.set_scene(scenes.random_scene(1_000_000, 42, env))
        W = H = 4096
        ctx.set_camera(abi.make_camera(W, H, abi.deg2rad(42.185), (-140.0, -175.0, 80.0), (0.0, 0.0, 0.0)))
        d, F = 8, 1
    else:
        sc = load_obj(scenes.AVENGER_OBJ)
        sc.set_environment(env)
        ctx.set_scene(sc)
        W, H = 1920, 1080
        ctx.set_camera(abi.default_camera(W, H))
        d, F = 5, 8
    fb = ctx.alloc(F * W * H * 16)
    med = lambda xs: sorted(xs)[len(xs) // 2]  # noqa: E731
    out = {"config": cfg}
    for name, pk in (("packets_all", 16), ("packets_l0", 1)):
        ctx.configure(packet_levels=pk)
        p = abi.make_params(max_level=d)
        ctx.render_frames_device(p, F, fb)
        p.profile = 1
        lv = []
        for _ in range(7):
            ctx.render_frames_device(p, F, fb)
            lv.append(ctx.frame_diag())
        p.profile = 0
        ctx.render_frames_device(p, F, fb)
        util = ctx.frame_diag()
        out[name] = [{"L": L, "rays": lv[0][L]["rays"], "trace_ms": round(med([x[L]["ms_trace"] for x in lv]), 4),
                      "util": round(util[L]["packet_steps_hit"] / util[L]["packet_steps_live"], 4)
                      if util[L]["packet_steps_live"] else None}
                     for L in range(d + 1) if lv[0][L]["rays"]]
    print(json.dumps(out), flush=True)
    ctx.free(fb)
    ctx.close()


if __name__ == "__main__":
    for c in sys.argv[1:] or ["C2", "C5"]:
        run(c)
