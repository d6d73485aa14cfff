"""Strong-scaling estimate on one GPU: each rank's share of an N-GPU C2 frame (64x64 tiles dealt
round-robin, pgrt_render_tiles_device) rendered alone; prints the median ms per rank and the max
over ranks (the gather is not included)."""
import os
import sys
import time

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
fb = ctx.alloc(W * H * 16 + (1 << 20) * 16)


def med_ms(p, rank=0, world=1, reps=40):
    for _ in range(5):
        ctx.render_tiles_device(p, rank, world, fb)
    ctx.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        ctx.render_tiles_device(p, rank, world, fb)
        ctx.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    return sorted(ts)[len(ts) // 2]


full = med_ms(abi.make_params(max_level=5))
print(f"full frame {full:.3f} ms")
for n in (2, 4, 8):
    ms = [med_ms(abi.make_params(max_level=5), r, n) for r in range(n)]
    print(f"N={n}: ranks {' '.join(f'{m:.3f}' for m in ms)} | max {max(ms):.3f} ms -> speedup {full / max(ms):.2f}")
