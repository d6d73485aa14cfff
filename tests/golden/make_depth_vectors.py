"""Boundary vectors for Embree's triangle depth test (tests/golden/depth_test_vectors.npz).

Embree 3.11's Moeller-Trumbore intersector (kernels/geometry/triangle_intersector_moeller.h, not
vendored in the reference; rtcIntersect1 is called at APP/raytracer.cpp:146) tests the depth on
the SCALED distance, absDen*tnear < T <= absDen*tfar, and divides only afterwards (t = T /
absDen).  Near tnear / tfar that classifies hits differently from "t = T / absDen; tnear < t <=
tfar".  These vectors put the interval ends exactly on (and one ulp either side of) each ray's
divided hit distance, so the two forms disagree on many of them:

  * "near": tnear = t, tnear = t -/+ 1 ulp (tfar FLT_MAX)
  * "far":  tfar = t, tfar = t -/+ 1 ulp (tnear 0.001)
  * "shadow": LightSource::GenerateRay's form (APP/LightSource.cpp:11-32): origin the light
    (-500, -100, 500), direction an unnormalised position vector, tfar exactly the occluder's t

Expected hits come from an independent float32 restatement here (numpy, one rounding per
operation, the operation order of oracle/oracle.c tri_hit), brute force over every triangle,
closest t with ties to the smaller index.  tests/test_golden.py checks the oracle against them
(CPU) and the HIP kernels (GPU, pgrt_intersect_closest) bit for bit.

usage: python tests/golden/make_depth_vectors.py
"""
import os

import numpy as np

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "depth_test_vectors.npz")
F = np.float32
FLT_MAX = F(3.402823466e38)
LIGHT = np.array([-500.0, -100.0, 500.0], F)


def xorsign(a, s):
    return (a.view(np.uint32) ^ (s.view(np.uint32) & np.uint32(0x80000000))).view(F)


def embree_hits(pos, rays, scaled=True):
    """rtcIntersect1 over all triangles: (n, 4) {t, u, v, prim bits}.  scaled=False: the
    divide-first form (for counting how many vectors the two forms classify differently)."""
    tri = pos.reshape(-1, 3, 3).astype(F)
    v0, v1, v2 = tri[:, 0], tri[:, 1], tri[:, 2]
    e1, e2 = v0 - v1, v2 - v0
    ng = np.stack([e2[:, 1] * e1[:, 2] - e2[:, 2] * e1[:, 1], e2[:, 2] * e1[:, 0] - e2[:, 0] * e1[:, 2],
                   e2[:, 0] * e1[:, 1] - e2[:, 1] * e1[:, 0]], 1)
    n = rays.shape[0]
    out = np.zeros((n, 4), F)
    for i in range(n):
        o, tnear, d, tfar = rays[i, 0:3], rays[i, 3], rays[i, 4:7], rays[i, 7]
        c = v0 - o
        r = np.stack([c[:, 1] * d[2] - c[:, 2] * d[1], c[:, 2] * d[0] - c[:, 0] * d[2],
                      c[:, 0] * d[1] - c[:, 1] * d[0]], 1)
        den = (ng[:, 0] * d[0] + ng[:, 1] * d[1]) + ng[:, 2] * d[2]
        absden = np.abs(den)
        U = xorsign((r[:, 0] * e2[:, 0] + r[:, 1] * e2[:, 1]) + r[:, 2] * e2[:, 2], den)
        V = xorsign((r[:, 0] * e1[:, 0] + r[:, 1] * e1[:, 1]) + r[:, 2] * e1[:, 2], den)
        T = xorsign((ng[:, 0] * c[:, 0] + ng[:, 1] * c[:, 1]) + ng[:, 2] * c[:, 2], den)
        with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
            ok = (den != 0) & (U >= 0) & (V >= 0) & ((U + V) <= absden)
            t = T / absden
            if scaled:
                ok &= (absden * tnear < T) & (T <= absden * tfar)
            else:
                ok &= (t > tnear) & (t <= tfar)
            best = -1
            for k in np.nonzero(ok)[0]:
                if best < 0 or t[k] < t[best]:
                    best = k
            if best < 0:
                out[i] = (tfar, 0, 0, np.int32(-1).view(F))
            else:
                out[i] = (t[best], U[best] / absden[best], V[best] / absden[best], np.int32(best).view(F))
    return out


def main():
    rng = np.random.default_rng(20251018)
    K = 48  # triangles, each in its own 60-unit cell
    pos = np.zeros((K, 3, 3), F)
    centres = np.zeros((K, 3), F)
    rays = []
    kinds = []
    for k in range(K):
        centre = np.array([(k % 8) * 60.0 - 200.0, (k // 8) * 60.0 - 150.0, rng.uniform(-20, 20)], F)
        if k >= 32:  # shadow-style: the triangle straddles a point of the light's ray L + s * H
            H = rng.uniform(-120, 120, 3).astype(F)
            s = F(rng.uniform(0.3, 0.9))
            centre = (LIGHT + s * H).astype(F)
        centres[k] = centre
        a = rng.normal(size=3)
        b = rng.normal(size=3)
        pos[k] = (centre + rng.uniform(2, 6) * np.stack([a / np.linalg.norm(a), b / np.linalg.norm(b),
                                                           -(a + b) / np.linalg.norm(a + b)])).astype(F)
    flat = pos.reshape(-1)
    for k in range(K):
        for rep in range(6):
            w = rng.dirichlet([1, 1, 1])
            target = (w[0] * pos[k, 0].astype(np.float64) + w[1] * pos[k, 1] + w[2] * pos[k, 2])
            if k >= 32:
                o = LIGHT.copy()
                d = ((target - LIGHT) / rng.uniform(0.3, 0.9)).astype(F)  # an unnormalised position-like vector
            else:
                o = (centres[k] + rng.normal(size=3) * 25).astype(F)
                d = (target - o).astype(F)
                if rep % 2:
                    d = (d / np.linalg.norm(d.astype(np.float64))).astype(F)
            base = np.concatenate([o, [F(0.001)], d, [FLT_MAX]]).astype(F)
            t = embree_hits(flat, base[None, :])[0]
            if t[3].view(np.int32) < 0:
                continue
            tt = t[0]
            for kind, tn, tf in (("near", tt, FLT_MAX), ("near-", np.nextafter(tt, F(0)), FLT_MAX),
                                 ("near+", np.nextafter(tt, FLT_MAX), FLT_MAX),
                                 ("far", F(0.001), tt), ("far-", F(0.001), np.nextafter(tt, F(0))),
                                 ("far+", F(0.001), np.nextafter(tt, FLT_MAX))):
                r = base.copy()
                r[3], r[7] = tn, tf
                rays.append(r)
                kinds.append(("shadow-" if k >= 32 else "") + kind)
    rays = np.array(rays, F)
    hits = embree_hits(flat, rays)
    old = embree_hits(flat, rays, scaled=False)
    differ = (hits.view(np.int32) != old.view(np.int32)).any(1)
    np.savez_compressed(OUT, pos=flat, rays=rays, hits=hits, kinds=np.array(kinds), divide_first_differs=differ)
    print(f"{len(rays)} rays over {K} triangles; the divide-first form differs on {int(differ.sum())} "
          f"({', '.join(sorted(set(k for k, x in zip(kinds, differ) if x)))})")


if __name__ == "__main__":
    main()
