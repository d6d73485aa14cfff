"""Debug aid: closest hits of the multi-lane kernel vs the one-lane kernel on random rays."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import scenes  # noqa: E402
from pgi_raytracing_amd.raytracer import Context, load_obj  # noqa: E402
from test_gpu_parity import _random_rays  # noqa: E402

sc = load_obj(scenes.AVENGER_OBJ)
ctx = Context(0)
rays = _random_rays(sc, 20000, 11)
os.environ["PGRT_GROUP_MAX"] = "0"
ctx.set_scene(sc)
a = ctx.intersect(rays)
os.environ["PGRT_GROUP_MAX"] = "1000000000"
ctx.set_scene(sc)
b = ctx.intersect(rays)
eq = (a.view(np.int32) == b.view(np.int32)).all(1)
bad = np.argwhere(~eq).ravel()
print("mismatch", len(bad), "of", len(eq))
for i in bad[:12]:
    print(i, "one-lane", a[i], a[i, 3:].view(np.int32), "group", b[i], b[i, 3:].view(np.int32), "ray", rays[i])
