"""N synchronous C2 frames through pgrt_render_device (the drop-in's one frame per call), for
rocprofv3 --hip-trace --kernel-trace: where the host time of one frame goes.
usage: python tools/sync_frames.py [frames]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import scenes  # noqa: E402
from pgi_raytracing_amd import abi  # noqa: E402
from pgi_raytracing_amd.raytracer import Context, load_obj  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
sc = load_obj(scenes.AVENGER_OBJ)
sc.set_environment(os.path.join(ROOT, "assets", "spherical_map_windows.jpg"))
ctx = Context(0)
for kv in filter(None, os.environ.get("DIAG_CFG", "").split(",")):
    k, v = kv.split("=", 1)
    ctx.configure(**{k: float(v) if "." in v else int(v)})
ctx.set_scene(sc)
ctx.set_camera(abi.default_camera(1920, 1080))
fb = ctx.alloc(1920 * 1080 * 16)
ms = []
for f in range(n):
    p = abi.make_params(max_level=5, jitter=abi.PGRT_JITTER_HASH, frame=f)
    t = time.perf_counter()
    ctx.render_device(p, fb)
    ms.append((time.perf_counter() - t) * 1e3)
print("frame ms:", " ".join(f"{x:.3f}" for x in ms))
