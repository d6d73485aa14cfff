// traverse.hpp -- the closest-hit building blocks of the traversal kernels (trace.hip): slab tests
// against a BVH2 node's child boxes and Embree's triangle test.
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

// Moeller-Trumbore as Embree's closest-hit path evaluates it (see oracle/oracle.c tri_hit): e1 =
// v0 - v1, e2 = v2 - v0 (precomputed), Ng = e2 x e1, scaled edge tests, the depth test on the
// scaled distance (absDen * tnear < T <= absDen * tfar, Embree 3.11 triangle_intersector_moeller.h)
// before t = T / absDen (IEEE division; Embree: rcp).  Closest hit in the ray's (tnear, tfar];
// ties in t go to the smaller original triangle index.
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
        if (absden * tnear < T && T <= absden * tfar) {
            const float t = T / absden;
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

__device__ __forceinline__ float qb(unsigned w, int j) { return (float)((w >> (8 * j)) & 0xffu); }

// ---- 8 lanes per ray, 8-wide BVH
//
// For small queues (the deep Whitted levels: tens of thousands of rays on 1024 SIMDs) a level
// takes as long as its slowest ray, and a one-lane traversal of that ray is a chain of ~100
// dependent node fetches.  Here 8 lanes trace one ray: every lane tests one child box of the
// current 8-wide node (lane k takes slot k ^ octant, so the group's ballot byte is already in
// near-to-far order), and the triangles of the node's hit leaves are tested 8 at a time.  The
// chain shrinks to one fetch per 8-wide node (about a third of the binary depth) plus one per
// leaf batch.  All 8 lanes hold identical traversal state (ballot / DPP reductions), so the
// group's control flow is uniform; the node-group stack lives in LDS, one per group.
constexpr int kGroupStack = 32;  // node groups per ray: >= 8-wide depth + 1

// reduce over the 8 lanes of a group: xor 1, xor 2 (quad DPP), then lane i <-> 7 - i (row
// half mirror), so every lane ends with the group value
#ifdef PGRT_GROUP_SHFL  // debugging aid: the same reductions through ds_bpermute
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
    return __shfl_xor(v, CTRL == 0xB1 ? 1 : (CTRL == 0x4E ? 2 : 7), 64);
}
#else
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, false);
}
#endif
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(dpp_i<CTRL>(__float_as_int(v)));
}
constexpr int kDppXor1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141;  // row_half_mirror

template <int CTRL>
__device__ __forceinline__ void merge_hit_step(float& t, float& u, float& v, int& prim) {
    const float ot = dpp_f<CTRL>(t), ou = dpp_f<CTRL>(u), ov = dpp_f<CTRL>(v);
    const int op = dpp_i<CTRL>(prim);
    if (op >= 0 && (prim < 0 || ot < t || (ot == t && op < prim))) {
        t = ot;
        u = ou;
        v = ov;
        prim = op;
    }
}

// group reductions: G = 8 uses xor 1, xor 2 and the half-row mirror; G = 4 the two quad steps
template <int G>
__device__ __forceinline__ int group_or(int v) {
    v |= dpp_i<kDppXor1>(v);
    v |= dpp_i<kDppXor2>(v);
    if constexpr (G == 8) v |= dpp_i<kDppHalfMirror>(v);
    return v;
}
template <int G>
__device__ __forceinline__ void group_merge_hit(float& t, float& u, float& v, int& prim) {
    merge_hit_step<kDppXor1>(t, u, v, prim);
    merge_hit_step<kDppXor2>(t, u, v, prim);
    if constexpr (G == 8) merge_hit_step<kDppHalfMirror>(t, u, v, prim);
}

// one child slot of a wide node against the ray (conservative quantized slab test)
struct SlotTest {
    bool hit, inner;
    unsigned meta;
};
__device__ __forceinline__ SlotTest test_slot(unsigned slot, const uint4& m, const uint4& qx, const uint4& qy,
                                              const uint4& qz, unsigned imask, float ax, float ay, float az,
                                              float bx, float by, float bz, bool px, bool py, bool pz,
                                              float best_t) {
    const int j = (int)(slot & 3u);
    const bool hi_half = slot >= 4u;
    const unsigned lxw = hi_half ? qx.y : qx.x, hxw = hi_half ? qx.w : qx.z;
    const unsigned lyw = hi_half ? qy.y : qy.x, hyw = hi_half ? qy.w : qy.z;
    const unsigned lzw = hi_half ? qz.y : qz.x, hzw = hi_half ? qz.w : qz.z;
    const float lx = qb(lxw, j), hx = qb(hxw, j), ly = qb(lyw, j), hy = qb(hyw, j);
    const float lz = qb(lzw, j), hz = qb(hzw, j);
    const float t0 = fmaxf(fmaxf(fmaf(px ? lx : hx, ax, bx), fmaf(py ? ly : hy, ay, by)),
                           fmaxf(fmaf(pz ? lz : hz, az, bz), 0.0f));
    const float t1 = fminf(fminf(fmaf(px ? hx : lx, ax, bx), fmaf(py ? hy : ly, ay, by)),
                           fminf(fmaf(pz ? hz : lz, az, bz), best_t));
    SlotTest r;
    r.meta = ((hi_half ? m.w : m.z) >> (8 * j)) & 0xffu;
    r.hit = r.meta != 0u && t0 <= t1 * 1.000001f;
    r.inner = ((imask >> slot) & 1u) != 0u;
    return r;
}


// Diagnostics build only (-DPGRT_STEP_PROFILE=1, tools/step_profile.py): the dependent steps of
// one traced ray on the shader clock (s_memtime cycles) -- each 8-wide node step and each triangle
// round, and inside them the wait from issuing the step's loads to their first use.  The product
// build compiles none of it.
#ifndef PGRT_STEP_PROFILE
#define PGRT_STEP_PROFILE 0
#endif
struct StepProf {
    unsigned long long node_cyc, node_wait, tri_cyc, tri_wait;
    unsigned nodes, tris;
};

// One ray traced by a group of G lanes (k = lane in the group, gshift = the group's first lane in
// the wave) over the 8-wide BVH; stk[sp * stride] is the group's node-group stack (kGroupStack
// entries, LDS).  Every lane of the group ends with the closest hit in best_* (in: the bound to
// start from -- tfar and no hit, or a hit found earlier).  o4 = org | tnear, d4 = dir | tfar;
// tfar < 0 (padding) -> nothing is traversed.
template <int G, bool COUNT>
__device__ __forceinline__ void trace8_group(const SceneView& s, float4 o4, float4 d4, int k, int gshift, uint2* stk,
                                             int stride, float& best_t, float& best_u, float& best_v, int& best_prim,
                                             unsigned& rvis, unsigned& rtest, StepProf* prof = nullptr) {
    (void)prof;
    const float ox = o4.x, oy = o4.y, oz = o4.z, tnear = o4.w;
    const float dx = d4.x, dy = d4.y, dz = d4.z, tfar = d4.w;
    const float sdx = fabsf(dx) < 1e-30f ? copysignf(1e-30f, dx) : dx;
    const float sdy = fabsf(dy) < 1e-30f ? copysignf(1e-30f, dy) : dy;
    const float sdz = fabsf(dz) < 1e-30f ? copysignf(1e-30f, dz) : dz;
    const float idx = __builtin_amdgcn_rcpf(sdx), idy = __builtin_amdgcn_rcpf(sdy), idz = __builtin_amdgcn_rcpf(sdz);
    const bool px = idx >= 0.0f, py = idy >= 0.0f, pz = idz >= 0.0f;
    const unsigned oct = (dx > 0.0f ? 1u : 0u) | (dy > 0.0f ? 2u : 0u) | (dz > 0.0f ? 4u : 0u);
    int sp = 0;
    unsigned gbase = 0, gbits = (1u << (24 + oct)) | 1u;  // the root: slot 0 of a virtual parent
    if (!(tfar >= 0.0f)) gbits = 0;
    unsigned tbase = 0, tbits = 0;
    for (;;) {
        while (tbits == 0u) {  // ---- node phase (group-uniform) ----
            long long pc0 = 0;
            if constexpr (PGRT_STEP_PROFILE) pc0 = clock64();  // (prof NULL: callers without a record)
            if (gbits <= 0x00ffffffu) {
                if (sp == 0) break;
                --sp;
                const uint2 g = stk[sp * stride];
                gbase = g.x;
                gbits = g.y;
            }
            const int pb = 31 - __clz((int)gbits);
            gbits &= ~(1u << pb);
            const unsigned slot = (unsigned)(pb - 24) ^ oct;
            const int child = (int)gbase + __popc(gbits & 0xffu & ((1u << slot) - 1u));
            if (gbits > 0x00ffffffu) {
                stk[sp * stride] = make_uint2(gbase, gbits);  // same value from all lanes of the group
                ++sp;
            }
            const Bvh8Node* nd = at_bytes(s.nodes8, (unsigned)child * (unsigned)sizeof(Bvh8Node));
            long long pc1 = 0;
            if constexpr (PGRT_STEP_PROFILE) pc1 = clock64();
            const float4 p = nd->p;
            const uint4 m = nd->m, qx = nd->qx, qy = nd->qy, qz = nd->qz;
            if constexpr (PGRT_STEP_PROFILE) {  // the node's loads have landed
                asm volatile("" ::"v"(p.w), "v"(m.z), "v"(qx.x), "v"(qy.x), "v"(qz.x));
                if (prof) prof->node_wait += (unsigned long long)(clock64() - pc1);
            }
            if (COUNT) ++rvis;
            const unsigned eb = __float_as_uint(p.w);
            const unsigned imask = eb >> 24;
            const float ax = __uint_as_float((eb & 0xffu) << 23) * idx;
            const float ay = __uint_as_float(((eb >> 8) & 0xffu) << 23) * idy;
            const float az = __uint_as_float(((eb >> 16) & 0xffu) << 23) * idz;
            const float bx = (p.x - ox) * idx, by = (p.y - oy) * idy, bz = (p.z - oz) * idz;
            // lane k tests the slot at near-to-far position k (slot k ^ oct) and, for G = 4, also
            // position k + 4; the ballots then give the group's near-to-far hit byte
            const SlotTest s0 =
                test_slot((unsigned)k ^ oct, m, qx, qy, qz, imask, ax, ay, az, bx, by, bz, px, py, pz, best_t);
            int tb = (s0.hit && !s0.inner) ? (int)wide_leaf_bits(s0.meta) : 0;
            unsigned nb = (unsigned)(__ballot(s0.hit && s0.inner) >> gshift) & ((1u << G) - 1u);
            if constexpr (G == 4) {
                const SlotTest s1 = test_slot((unsigned)(k + 4) ^ oct, m, qx, qy, qz, imask, ax, ay, az, bx, by, bz,
                                              px, py, pz, best_t);
                if (s1.hit && !s1.inner) tb |= (int)wide_leaf_bits(s1.meta);
                nb |= ((unsigned)(__ballot(s1.hit && s1.inner) >> gshift) & 0xfu) << 4;
            }
            tb = group_or<G>(tb);
            gbase = m.x;
            gbits = (nb << 24) | imask;
            tbase = m.y;
            tbits = (unsigned)tb;
            if constexpr (PGRT_STEP_PROFILE) {
                asm volatile("" ::"v"(tbits), "v"(gbits));
                if (prof) {
                    prof->node_cyc += (unsigned long long)(clock64() - pc0);
                    ++prof->nodes;
                }
            }
        }
        if (tbits == 0u) break;
        // ---- triangle phase: G triangles per round, then the group's closest hit ----
        while (tbits != 0u) {
            long long pc0 = 0;
            if constexpr (PGRT_STEP_PROFILE) pc0 = clock64();
            // this lane's set bit: the lowest k cleared, branch-free (k is the lane in the group)
            unsigned mine = tbits;
#pragma unroll
            for (int q = 0; q < G - 1; ++q) mine = q < k ? mine & (mine - 1u) : mine;
            if (mine != 0u) {
                const int tr = (int)tbase + __ffs((int)mine) - 1;
                const float4* q = at_bytes(s.tri8, (unsigned)tr * 48u);
                long long pc1 = 0;
                if constexpr (PGRT_STEP_PROFILE) pc1 = clock64();
                const float4 q0 = q[0], q1 = q[1], q2 = q[2];
                if constexpr (PGRT_STEP_PROFILE) {
                    asm volatile("" ::"v"(q0.x), "v"(q1.x), "v"(q2.x));
                    if (prof && k == 0) prof->tri_wait += (unsigned long long)(clock64() - pc1);
                }
                tri_test(q0, q1, q2, ox, oy, oz, dx, dy, dz, tnear, tfar, best_t, best_u, best_v, best_prim);
            }
            if (COUNT) rtest += (unsigned)min(__popc(tbits), G);
            for (int q = 0; q < G; ++q) tbits &= tbits - 1u;
            group_merge_hit<G>(best_t, best_u, best_v, best_prim);
            if constexpr (PGRT_STEP_PROFILE) {
                asm volatile("" ::"v"(best_t), "v"(best_prim));
                if (prof) {
                    prof->tri_cyc += (unsigned long long)(clock64() - pc0);
                    ++prof->tris;
                }
            }
        }
    }
}

}  // namespace pgrt
