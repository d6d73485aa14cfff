"""Render the same small frames with two builds of libpgrt.so (PGRT_LIB) and report the pixels
that differ (A/B debugging of a kernel change that should be bit-identical).

usage: python tools/diff_libs.py <libA> <libB> [W H d S dof]"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(out, W, H, d, S, dof):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import scenes  # noqa: F401
    from pgi_raytracing_amd import abi
    from pgi_raytracing_amd.raytracer import Context, load_obj
    sc = load_obj(scenes.AVENGER_OBJ)
    sc.set_environment(os.path.join(ROOT, "assets", "spherical_map_windows.jpg"))
    ctx = Context(0)
    ctx.set_scene(sc)
    ctx.set_camera(abi.default_camera(W, H))
    p = abi.make_params(spp_side=S, max_level=d, dof=dof,
                        jitter=abi.PGRT_JITTER_HASH if S > 1 or dof else abi.PGRT_JITTER_NONE)
    img, st = ctx.render(p)
    np.save(out, img)


def main():
    if sys.argv[1] == "--child":
        child(sys.argv[2], *[int(x) for x in sys.argv[3:8]])
        return
    a, b = sys.argv[1:3]
    args = [str(x) for x in ([int(x) for x in sys.argv[3:]] + [48, 36, 5, 1, 0][len(sys.argv) - 3:])]
    outs = []
    for k, lib in enumerate((a, b)):
        out = f"/tmp/diff_libs_{k}.npy"
        subprocess.run([sys.executable, __file__, "--child", out] + args, check=True,
                       env=dict(os.environ, PGRT_LIB=lib))
        outs.append(np.load(out))
    A, B = outs
    ne = (A.view(np.int32) != B.view(np.int32)).any(-1)
    print(f"{ne.sum()} of {ne.size} pixels differ")
    for y, x in list(zip(*np.nonzero(ne)))[:20]:
        print(f"  ({x},{y}) A {A[y, x]} B {B[y, x]}")


if __name__ == "__main__":
    main()
