"""Full-size C2 frame: the oracle built on pgrt_detmath.h (what the GPU matches bit for bit)
against the same oracle built on glibc's libm (ORACLE_LIBM) -- how far "bit-identical to the
restatement" is from a reference built on a platform libm.  Prints one JSON line.
usage: python tools/libm_parity.py [width height]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tools")]
import pyoracle  # noqa: E402  test infrastructure
import scenes  # noqa: E402
from pgi_raytracing_amd import abi  # noqa: E402
from pgi_raytracing_amd.raytracer import load_obj  # noqa: E402


def main(w=1920, h=1080):
    scene = load_obj(scenes.AVENGER_OBJ)
    scene.set_environment(os.path.join(ROOT, "assets", "spherical_map_windows.jpg"))
    cam = abi.default_camera(w, h)
    p = abi.make_params(spp_side=1, max_level=5)
    a, _ = pyoracle.OracleScene(scene, libm=False).render(cam, p, threads=os.cpu_count())
    b, _ = pyoracle.OracleScene(scene, libm=True).render(cam, p, threads=os.cpu_count())
    nan_a, nan_b = np.isnan(a), np.isnan(b)
    d = np.abs(np.where(nan_a, 0, a) - np.where(nan_b, 0, b))[..., :3].max(axis=2)
    nan_px = (nan_a != nan_b).any(axis=2)
    over = (d > 1e-4) | nan_px
    # where the differing pixels are: primary misses (environment only) vs pixels on the ship
    rays = []
    ys, xs = np.nonzero(over)
    for y, x in zip(ys[:4000], xs[:4000]):
        r = pyoracle.generate_ray(cam, float(x), float(y))
        rays.append([r[0], r[1], r[2], r[6], r[3], r[4], r[5], r[7]])
    on_ship = None
    if rays:
        hits = pyoracle.OracleScene(scene).intersect(np.array(rays, np.float32))
        on_ship = float((hits[:, 3].view(np.int32) >= 0).mean())
    print(json.dumps({"frame": f"C2 {w}x{h} d=5 1 spp", "pixels": int(w * h),
                      "frac_over_1e-4": float(over.mean()), "pixels_over_1e-4": int(over.sum()),
                      "frac_not_identical": float(((d > 0) | nan_px).mean()),
                      "max_abs_diff": float(d.max()), "nan_mismatch_pixels": int(nan_px.sum()),
                      "over_1e-4_on_ship_frac": on_ship}))


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:3]])
