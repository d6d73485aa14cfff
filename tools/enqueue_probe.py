"""Host-side cost of submitting frame calls (pgrt_render_frames_device_async) in bench.py's C2
setting: warm the frame sets like bench.py, then time each submission of K frames and the wait.
usage: python tools/enqueue_probe.py [K] [F]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
import scenes  # noqa: E402
from pgi_raytracing_amd import abi  # noqa: E402
from pgi_raytracing_amd.raytracer import Context, load_obj  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
F = int(sys.argv[2]) if len(sys.argv) > 2 else 8
scene = load_obj(scenes.AVENGER_OBJ)
scene.set_environment(os.path.join(ROOT, "assets", "spherical_map_windows.jpg"))
ctx = Context(0)
ctx.set_scene(scene)
ctx.set_camera(abi.default_camera(1920, 1080))
p = abi.make_params(spp_side=1, max_level=5)
fb = ctx.alloc(F * 1920 * 1080 * 16)
ctx.set_frames_in_flight(8)
for rep in range(4):
    ts = [ctx.render_frames_device_async(p, F, fb) for _ in range(8)]
    for t in ts:
        ctx.render_wait(t)
    ctx.synchronize()
    sub = []
    t0 = time.perf_counter()
    ts = []
    for f0 in range(0, K, F):
        a = time.perf_counter()
        ts.append(ctx.render_frames_device_async(p, min(F, K - f0), fb))
        sub.append((time.perf_counter() - a) * 1e3)
    t_sub = time.perf_counter()
    for t in ts:
        ctx.render_wait(t)
    ctx.synchronize()
    t1 = time.perf_counter()
    print(f"K={K} F={F}: submit ms {[round(x, 3) for x in sub]}, all submitted at {(t_sub - t0) * 1e3:.3f} ms, "
          f"done at {(t1 - t0) * 1e3:.3f} ms -> {(t1 - t0) * 1e3 / K:.4f} ms/frame", flush=True)
