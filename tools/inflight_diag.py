"""Frames-in-flight diagnosis for a bench config: per-frame submit->complete time, rays and
overflow retries of every frame (bench.py's timed loop, one frame per call).
usage: python tools/inflight_diag.py <config> <in_flight> <frames>"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
os.environ["GPU_MAX_HW_QUEUES"] = "16"
import bench  # noqa: E402
import scenes  # noqa: E402
from pgi_raytracing_amd import abi  # noqa: E402
from pgi_raytracing_amd.raytracer import Context, load_obj  # noqa: E402


def main():
    cfg, inflight, frames = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    c = bench.CONFIGS[cfg]
    for k, v in c.get("env", {}).items():
        os.environ.setdefault(k, v)
    env = os.path.join(ROOT, "assets", "spherical_map_windows.jpg")
    if c["scene"] == "avenger":
        sc = load_obj(scenes.AVENGER_OBJ)
        sc.set_environment(env)
        cam = abi.default_camera(c["width"], c["height"])
    else:
        sc = scenes.random_scene(1_000_000, 42, env)
        cam = abi.make_camera(c["width"], c["height"], abi.deg2rad(42.185), (-140.0, -175.0, 80.0), (0.0, 0.0, 0.0))
    p = abi.make_params(spp_side=c["spp_side"], max_level=c["max_level"], dof=c["dof"],
                        jitter=abi.PGRT_JITTER_HASH if (c["spp_side"] > 1 or c["dof"]) else abi.PGRT_JITTER_NONE)
    ctx = Context(0)
    ctx.set_scene(sc)
    ctx.set_camera(cam)
    fb = ctx.alloc(c["width"] * c["height"] * 16)
    ctx.set_frames_in_flight(inflight)
    pend = []
    t0 = time.perf_counter()
    for f in range(frames):
        pend.append((f, time.perf_counter(), ctx.render_device_async(p, fb)))
        if len(pend) >= inflight:
            g, ts, t = pend.pop(0)
            st = ctx.render_wait(t)
            print(f"frame {g}: ms_total {st.ms_total:.2f} rays {st.rays()} retries {st.overflow_retries} "
                  f"t {1e3 * (time.perf_counter() - t0):.1f}", flush=True)
    while pend:
        g, ts, t = pend.pop(0)
        st = ctx.render_wait(t)
        print(f"frame {g}: ms_total {st.ms_total:.2f} rays {st.rays()} retries {st.overflow_retries} "
              f"t {1e3 * (time.perf_counter() - t0):.1f}", flush=True)


if __name__ == "__main__":
    main()
