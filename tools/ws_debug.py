"""Debug run of the work-sharing subtree launch: one small avenger frame (96x64, d = 5) with the
subtree from level 2, compared with the oracle (PGRT_LIB: a PGRT_WS_DEBUG build prints the
watchdog state)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import pyoracle  # noqa: E402
import scenes  # noqa: E402
from pgi_raytracing_amd import abi  # noqa: E402
from pgi_raytracing_amd.raytracer import Context, load_obj  # noqa: E402

sc = load_obj(scenes.AVENGER_OBJ)
sc.set_environment(os.path.join(ROOT, "assets", "spherical_map_windows.jpg"))
ctx = Context(0)
ctx.configure(subtree_level=int(sys.argv[1]) if len(sys.argv) > 1 else 2)
ctx.set_scene(sc)
cam = abi.default_camera(96, 64)
ctx.set_camera(cam)
for d in (5, 4, 6):
    p = abi.make_params(max_level=d)
    img, st = ctx.render(p)
    ref, _ = pyoracle.OracleScene(sc).render(cam, p)
    same = (img == ref) | (np.isnan(img) & np.isnan(ref))
    print("d", d, "pixels differing:", int((~same).sum()), "rays", st.rays(), flush=True)
