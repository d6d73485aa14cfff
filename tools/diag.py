"""Per-level traversal diagnostics of one frame (GPU): rays, node visits and the worst ray.

usage: python tools/diag.py [W H d S dof]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import scenes  # noqa: E402
from pgi_raytracing_amd import abi  # noqa: E402
from pgi_raytracing_amd.raytracer import Context, load_obj  # noqa: E402


def main():
    a = [int(x) for x in sys.argv[1:]] + [1920, 1080, 5, 1, 0][len(sys.argv) - 1:]
    W, H, d, S, dof = a[:5]
    env = os.path.join(ROOT, "assets", "spherical_map_windows.jpg")
    c5 = os.environ.get("DIAG_SCENE") == "c5"  # BASELINE C5: 10^6 random triangles
    if c5:
        sc = scenes.random_scene(1_000_000, 42, env)
    else:
        sc = load_obj(scenes.AVENGER_OBJ)
        if not os.environ.get("DIAG_NOENV"):
            sc.set_environment(env)
    ctx = Context(0)
    for kv in filter(None, os.environ.get("DIAG_CFG", "").split(",")):  # e.g. DIAG_CFG=packet_budget=-1
        k, v = kv.split("=", 1)
        ctx.configure(**{k: float(v) if "." in v else int(v)})
    t = time.time()
    ctx.set_scene(sc)
    info = ctx.bvh_info()
    print(json.dumps({"bvh": {"builder": {1: "lbvh", 2: "ploc"}.get(info.builder, info.builder), "iters": info.build_iterations,
                              "tris": info.num_triangles, "nodes": info.num_nodes, "depth": info.max_depth,
                              "width": info.width, "refs": info.num_references, "split": round(info.split_beta, 3), "build_ms": round(info.build_ms, 3), "set_scene_s": round(time.time() - t, 3)}}))
    if c5:
        ctx.set_camera(abi.make_camera(W, H, abi.deg2rad(42.185), (-140.0, -175.0, 80.0), (0.0, 0.0, 0.0)))
    else:
        ctx.set_camera(abi.default_camera(W, H))
    p = abi.make_params(spp_side=S, max_level=d, dof=dof,
                        jitter=abi.PGRT_JITTER_HASH if S > 1 or dof else abi.PGRT_JITTER_NONE)
    F = int(os.environ.get("DIAG_FRAMES", "1"))  # frames per call (the bench's batched frames)
    buf = ctx.alloc(F * W * H * 16)

    def render(q):
        if F == 1:
            return ctx.render(q)
        return None, ctx.render_frames_device(q, F, buf)

    render(p)
    p.profile = 1
    reps = int(os.environ.get("DIAG_REPS", "9"))  # medians over repeated profiled frames
    stats, lvs = [], []
    for _ in range(reps):
        _, st = render(p)
        stats.append(st.as_dict())
        lvs.append([(dd["ms_trace"], dd["ms_shade"]) for dd in ctx.frame_diag()])
    med = lambda xs: sorted(xs)[len(xs) // 2]  # noqa: E731
    print(json.dumps({"stage_ms": {k: round(med([x[k] for x in stats]), 4) for k in stats[0] if k.startswith("ms_")},
                      "rays": st.rays(), "trace_launches": st.trace_launches, "reps": reps}))
    lv_ms = [(med([lv[L][0] for lv in lvs]), med([lv[L][1] for lv in lvs])) for L in range(len(lvs[0]))]
    p.profile = 2
    render(p)
    for L, dd in enumerate(ctx.frame_diag()):
        if dd["rays"] == 0 and dd["shadow_rays"] == 0:
            continue
        r = max(1, dd["rays"])
        s = max(1, dd["shadow_rays"])
        print(f"L{L}: rays {dd['rays']:9d} visits/ray {dd['visits'] / r:7.1f} max {dd['max_visits']:6d} "
              f"tests/ray {dd['tests'] / r:6.1f} max {dd['max_tests']:5d} | shadow {dd['shadow_rays']:8d} "
              f"visits/ray {dd['shadow_visits'] / s:6.1f} max {dd['shadow_max_visits']:5d} | wave iters "
              f"{dd['max_wave_iterations']:5d} ray {dd['max_ray_ticks'] / 100:6.1f} us spills {dd['stack_spills']:6d} "
              f"stack {dd['max_stack']:3d} | longest: vis {dd['lr_visits']} tests {dd['lr_tests']} leaves "
              f"{dd['lr_leaves']} node cyc/vis {dd['lr_node_cyc64'] * 64 / max(1, dd['lr_visits']):.0f} leaf cyc/leaf "
              f"{dd['lr_leaf_cyc64'] * 64 / max(1, dd['lr_leaves']):.0f} load cyc/vis "
              f"{dd['lr_load_cyc64'] * 64 / max(1, dd['lr_visits']):.0f} | trace {lv_ms[L][0] * 1e3:7.1f} us shade {lv_ms[L][1] * 1e3:6.1f} us")


if __name__ == "__main__":
    main()
