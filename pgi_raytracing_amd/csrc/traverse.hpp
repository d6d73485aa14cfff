// traverse.hpp -- the closest-hit building blocks shared by the traversal kernels (trace.hip) and
// the persistent tail kernel (tail.hip): slab tests against a BVH2 node's child boxes, Embree's
// triangle test, and one lane's complete closest-hit traversal with its stack in LDS.
// Reference: rtcIntersect1 (APP/raytracer.cpp:130-148 get_ray_hit; rtcore_scene.h:96).
#pragma once

#include "shade_ops.hpp"
#include "trace.hpp"

namespace pgrt {

constexpr int kSentinel = 0x7fffffff;  // bottom of every stack: "traversal finished"

__device__ __forceinline__ bool box_hit(float lox, float hix, float loy, float hiy, float loz,
                                        float hiz, float idx, float idy, float idz, float oix,
                                        float oiy, float oiz, float tmax, float& tent) {
    const float tx0 = fmaf(lox, idx, -oix), tx1 = fmaf(hix, idx, -oix);
    const float ty0 = fmaf(loy, idy, -oiy), ty1 = fmaf(hiy, idy, -oiy);
    const float tz0 = fmaf(loz, idz, -oiz), tz1 = fmaf(hiz, idz, -oiz);
    const float t0 = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
    const float t1 = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tmax));
    tent = t0;
    return t0 <= t1 * 1.000001f;  // conservative: rounding never culls a box a hit lies in
}
// the same test with each axis's near and far planes already chosen from the sign of the ray's
// inverse direction: fma is monotonic, so the near plane's t IS the fminf above (and the far's
// the fmaxf) -- identical t0 / t1 without the 6 min / max that order them
__device__ __forceinline__ bool box_hit_nf(float nx, float fx, float ny, float fy, float nz, float fz, float idx,
                                           float idy, float idz, float oix, float oiy, float oiz, float tmax,
                                           float& tent) {
    const float txn = fmaf(nx, idx, -oix), txf = fmaf(fx, idx, -oix);
    const float tyn = fmaf(ny, idy, -oiy), tyf = fmaf(fy, idy, -oiy);
    const float tzn = fmaf(nz, idz, -oiz), tzf = fmaf(fz, idz, -oiz);
    const float t0 = fmaxf(fmaxf(txn, tyn), fmaxf(tzn, 0.0f));
    const float t1 = fminf(fminf(txf, tyf), fminf(tzf, tmax));
    tent = t0;
    return t0 <= t1 * 1.000001f;
}

// Moeller-Trumbore as Embree's closest-hit path evaluates it (see oracle/oracle.c): e1 = v0 - v1,
// e2 = v2 - v0 (precomputed), Ng = e2 x e1, scaled edge tests, IEEE divisions.  Closest hit in
// (tnear, tfar]; ties in t go to the smaller original triangle index.
// ng: the triangle's Ng = e2 x e1 (tri_normal, precomputed per reference with the same float ops)
__device__ __forceinline__ void tri_test_ng(float4 q0, float4 q1, float4 q2, float4 ng, float ox, float oy, float oz,
                                            float dx, float dy, float dz, float tnear, float tfar, float& best_t,
                                            float& best_u, float& best_v, int& best_prim) {
    const float e1x = q1.x, e1y = q1.y, e1z = q1.z;
    const float e2x = q2.x, e2y = q2.y, e2z = q2.z;
    const float ngx = ng.x, ngy = ng.y, ngz = ng.z;
    const float cx = q0.x - ox, cy = q0.y - oy, cz = q0.z - oz;
    const float rx = cy * dz - cz * dy;
    const float ry = cz * dx - cx * dz;
    const float rz = cx * dy - cy * dx;
    const float den = ngx * dx + ngy * dy + ngz * dz;
    const float absden = fabsf(den);
    const float U = xorsign(rx * e2x + ry * e2y + rz * e2z, den);
    const float V = xorsign(rx * e1x + ry * e1y + rz * e1z, den);
    if (den != 0.0f && U >= 0.0f && V >= 0.0f && U + V <= absden) {
        const float T = xorsign(ngx * cx + ngy * cy + ngz * cz, den);
        const float t = T / absden;
        if (t > tnear && t <= tfar) {
            const int prim = __float_as_int(q0.w);
            if (best_prim < 0 || t < best_t || (t == best_t && prim < best_prim)) {
                best_t = t;
                best_u = U / absden;
                best_v = V / absden;
                best_prim = prim;
            }
        }
    }
}

__device__ __forceinline__ void tri_test(float4 q0, float4 q1, float4 q2, float ox, float oy, float oz, float dx,
                                         float dy, float dz, float tnear, float tfar, float& best_t, float& best_u,
                                         float& best_v, int& best_prim) {
    tri_test_ng(q0, q1, q2, tri_normal(q1, q2), ox, oy, oz, dx, dy, dz, tnear, tfar, best_t, best_u, best_v,
                best_prim);
}

// One lane's closest hit over the binary BVH (the one-lane kernel's while-while loop with
// postponed leaves, Aila & Laine 2009), the stack in LDS: lstack[entry * stride + slot], depth + 2
// entries (the caller sizes it).  o4 = org | tnear, d4 = dir | tfar; tfar < 0 (padding) -> no
// hit.  Returns (t, u, v, prim bits); prim -1 = no hit (t = tfar).
__device__ __forceinline__ float4 trace_closest_lds(const SceneView& s, float4 o4, float4 d4, int* lstack, int stride,
                                                    int slot) {
    const float ox = o4.x, oy = o4.y, oz = o4.z, tnear = o4.w;
    const float dx = d4.x, dy = d4.y, dz = d4.z, tfar = d4.w;
    const float sdx = fabsf(dx) < 1e-30f ? copysignf(1e-30f, dx) : dx;
    const float sdy = fabsf(dy) < 1e-30f ? copysignf(1e-30f, dy) : dy;
    const float sdz = fabsf(dz) < 1e-30f ? copysignf(1e-30f, dz) : dz;
    const float idx = __builtin_amdgcn_rcpf(sdx), idy = __builtin_amdgcn_rcpf(sdy), idz = __builtin_amdgcn_rcpf(sdz);
    const float oix = ox * idx, oiy = oy * idy, oiz = oz * idz;
    float best_t = tfar, best_u = 0.0f, best_v = 0.0f;
    int best_prim = -1;
    int sp = 0;
    lstack[slot] = kSentinel;  // stack[0]
    int node = s.root;
    int leaf = 0;  // postponed leaf (negative code) or 0
    if (node < 0) {
        leaf = node;
        node = kSentinel;
    }
    if (!(tfar >= 0.0f)) {
        node = kSentinel;
        leaf = 0;
    }
    while (node != kSentinel || leaf < 0) {
        const float bt = __builtin_canonicalizef(best_t);
        while ((unsigned)node < (unsigned)kSentinel) {
            const int top = lstack[sp * stride + slot];
            const BvhNode* nd = s.nodes + node;
            const float4 a = nd->a, b = nd->b, c = nd->c;
            const int4 d = nd->d;
            float t0, t1;
            const bool h0 = box_hit(a.x, a.y, a.z, a.w, c.x, c.y, idx, idy, idz, oix, oiy, oiz, bt, t0);
            const bool h1 = box_hit(b.x, b.y, b.z, b.w, c.z, c.w, idx, idy, idz, oix, oiy, oiz, bt, t1);
            const bool any = h0 || h1;
            const bool first0 = h0 && (!h1 || t0 <= t1);
            const bool both = h0 && h1;
            lstack[(sp + 1) * stride + slot] = first0 ? d.y : d.x;  // above the top: free either way
            node = any ? (first0 ? d.x : d.y) : top;
            sp += both ? 1 : (any ? 0 : -1);
            if (node < 0 && leaf == 0) {  // first leaf: park it and keep descending
                leaf = node;
                node = lstack[sp * stride + slot];
                --sp;
            }
            if (!__any(leaf == 0)) break;
        }
        while (leaf < 0) {
            const int first = leaf_first(leaf), end = first + leaf_count(leaf);
            float4 p0 = s.tri[3 * first], p1 = s.tri[3 * first + 1], p2 = s.tri[3 * first + 2];
            for (int k = first; k < end; ++k) {
                const float4 q0 = p0, q1 = p1, q2 = p2;
                if (k + 1 < end) {
                    p0 = s.tri[3 * k + 3];
                    p1 = s.tri[3 * k + 4];
                    p2 = s.tri[3 * k + 5];
                }
                tri_test(q0, q1, q2, ox, oy, oz, dx, dy, dz, tnear, tfar, best_t, best_u, best_v, best_prim);
            }
            leaf = 0;
            if (node < 0) {  // the node popped after parking is a leaf too: test it now
                leaf = node;
                node = lstack[sp * stride + slot];
                --sp;
            }
        }
    }
    return make_float4(best_t, best_u, best_v, __int_as_float(best_prim));
}

}  // namespace pgrt
