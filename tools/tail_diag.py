"""Persistent tail diagnostics (tail.hip, profile == 2 counters) of one C2 frame / call.

usage: DIAG_FRAMES=F python tools/tail_diag.py [W H d]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import scenes  # noqa: E402
from pgi_raytracing_amd import abi  # noqa: E402
from pgi_raytracing_amd.raytracer import Context, load_obj  # noqa: E402


def main():
    a = [int(x) for x in sys.argv[1:]] + [1920, 1080, 5][len(sys.argv) - 1:]
    W, H, d = a[:3]
    sc = load_obj(scenes.AVENGER_OBJ)
    sc.set_environment(os.path.join(ROOT, "assets", "spherical_map_windows.jpg"))
    ctx = Context(0)
    for kv in filter(None, os.environ.get("DIAG_CFG", "").split(",")):
        k, v = kv.split("=", 1)
        ctx.configure(**{k: int(v)})
    ctx.set_scene(sc)
    ctx.set_camera(abi.default_camera(W, H))
    F = int(os.environ.get("DIAG_FRAMES", "1"))
    buf = ctx.alloc(F * W * H * 16)
    p = abi.make_params(spp_side=1, max_level=d)
    for prof in (0, 1, 2):
        p.profile = prof
        st = ctx.render(p)[1] if F == 1 else ctx.render_frames_device(p, F, buf)
        print("profile", prof, "ms_total", round(st.ms_total, 3), "ms_trace", round(st.ms_trace, 3),
              "launches", st.trace_launches)
    for L, dd in enumerate(ctx.frame_diag()):
        lr = [dd[k] for k in ("lr_visits", "lr_tests", "lr_leaves", "lr_node_cyc64", "lr_leaf_cyc64", "lr_load_cyc64")]
        print(f"L{L}: rays {dd['rays']} trace_ms {dd['ms_trace']:.3f} | tail: iterations {lr[0]} idle {lr[1]} "
              f"flag polls x16 {lr[2]} kcycles pick {lr[3]} trace {lr[4]} shade {lr[5]}")


if __name__ == "__main__":
    main()
