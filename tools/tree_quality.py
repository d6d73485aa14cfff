"""C5 tree quality, CPU side: internal-node visits and triangle tests per ray of the oracle's
top-down 16-bin SAH BVH (oracle/oracle.c bvh_build; leaves <= 4 triangles; the same visit
semantics as libpgrt's one-lane traversal: one visit = one internal node fetched, both child
boxes tested) on every 64th row of the C5 frame.  Compare with the GPU PLOC tree's one-lane
counts: python bench.py --config C5 --roofline-only --packet-levels -1 (roofline.node_visits_per_ray).
usage: python tools/tree_quality.py [row_step]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tools")]
import pyoracle  # noqa: E402
import scenes  # noqa: E402
from pgi_raytracing_amd import abi  # noqa: E402


def main():
    step = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    env = os.path.join(ROOT, "assets", "spherical_map_windows.jpg")
    sc = scenes.random_scene(1_000_000, 42, env)
    t = time.time()
    osc = pyoracle.OracleScene(sc)
    print(f"oracle SAH build {time.time() - t:.1f} s", flush=True)
    cam = abi.make_camera(4096, 4096, abi.deg2rad(42.185), (-140.0, -175.0, 80.0), (0.0, 0.0, 0.0))
    p = abi.make_params(max_level=8)
    t = time.time()
    _, st = osc.render(cam, p, row_step=step)
    rays = st.rays_primary + st.rays_shadow + st.rays_reflect + st.rays_refract
    print(f"every {step}th row: {rays} rays in {time.time() - t:.1f} s; oracle SAH tree: "
          f"{st.node_visits / rays:.2f} node visits / ray, {st.tri_tests / rays:.2f} triangle tests / ray")


if __name__ == "__main__":
    main()
