"""Closest-hit launch duration against queue size (run under rocprofv3 --kernel-trace): random
secondary-like rays in the avenger proxy (origins on triangles, uniformly random directions),
traced through pgrt_intersect_closest at several sizes, one lane per ray (group_max -1) and 8
lanes per ray (group_max large).  Prints the order of the launches; pair them with the trace.
usage: python tools/latency_curve.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
import scenes  # noqa: E402
from pgi_raytracing_amd.raytracer import Context, load_obj  # noqa: E402

FLT_MAX = np.float32(3.402823466e38)


def rays(scene, n, seed):
    rng = np.random.default_rng(seed)
    p = scene.positions.reshape(-1, 3, 3)
    idx = rng.integers(0, p.shape[0], size=n)
    w = rng.dirichlet([1, 1, 1], size=n).astype(np.float32)
    org = np.einsum("nk,nkc->nc", w, p[idx]).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return np.concatenate([org, np.full((n, 1), 0.01, np.float32), d, np.full((n, 1), FLT_MAX, np.float32)], 1)


def main():
    sc = load_obj(scenes.AVENGER_OBJ)
    ctx = Context(0)
    ctx.set_scene(sc)
    for gm, label in ((-1, "one-lane"), (4_000_000, "8/4-lane groups")):
        ctx.configure(group_max=gm)
        for n in (256, 4096, 32768, 131072, 524288):
            r = rays(sc, n, n)
            for rep in range(3):
                h = ctx.intersect(r)
            print(f"{label} n={n} hit fraction {(h[:, 3].view(np.int32) >= 0).mean():.3f} (3 launches)", flush=True)


if __name__ == "__main__":
    main()
