"""Host-side submit cost of the driver-style C2 run: how long each pgrt_render_frames_device_async
call takes to return (host work before the GPU can start: slot setup, uploads, launches), and
when the last call's frames are done.  usage: python tools/submit_latency.py [calls] [frames]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
import scenes  # noqa: E402
from pgi_raytracing_amd import abi  # noqa: E402
from pgi_raytracing_amd.raytracer import Context, load_obj  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    F = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    if not os.path.exists(scenes.AVENGER_OBJ):
        scenes.write_avenger_proxy()
    scene = load_obj(scenes.AVENGER_OBJ)
    scene.set_environment(os.path.join(ROOT, "assets", "spherical_map_windows.jpg"))
    ctx = Context(0)
    ctx.set_scene(scene)
    ctx.set_camera(abi.default_camera(1920, 1080))
    params = abi.make_params(max_level=5)
    ctx.set_frames_in_flight(8)
    fb = ctx.alloc(F * 1920 * 1080 * 16)
    for rep in range(4):
        pend = [ctx.render_frames_device_async(params, F, fb) for _ in range(8)]
        for h in pend:
            ctx.render_wait(h)
        ctx.synchronize()
        t0 = time.perf_counter()
        marks, pend = [], []
        for _ in range(calls):
            pend.append(ctx.render_frames_device_async(params, F, fb))
            marks.append(time.perf_counter() - t0)
        for h in pend:
            ctx.render_wait(h)
        ctx.synchronize()
        done = time.perf_counter() - t0
        print(f"rep {rep}: submit returns at " + ", ".join(f"{m * 1e3:.3f}" for m in marks)
              + f" ms; all {calls * F} frames done at {done * 1e3:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
