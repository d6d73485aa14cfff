// trace.hip -- closest-hit BVH traversal: the replacement for Embree's rtcIntersect1
// (APP/raytracer.cpp:130-148 get_ray_hit; rtcore_scene.h:96).
//
// One lane = one ray of a SoA queue (ro = {org, tnear}, rd = {dir, tfar}; 16-B coalesced
// loads), BVH2 with both child boxes in the parent node (64 B per node, one cache line per
// visit), per-lane traversal stack in LDS laid out [depth][lane] (bank = lane % 32 for every
// depth: conflict-free), spilling to a per-thread global region past kLdsStack entries.
//
// Loop structure (Aila & Laine's "while-while" with postponed leaves): a lane keeps descending
// internal nodes and parks the first leaf it meets; the wave switches to triangle tests only
// when every active lane holds a leaf, so internal-node and leaf work are not serialised
// against each other inside a wave.  Persistent waves pull 64 rays at a time from a work
// counter (one atomic per wave), so the grid is sized to the machine, not to the queue.
//
// Results do not depend on the traversal order: every triangle the conservative box test lets
// through is tested with the same arithmetic as the oracle, and ties in t go to the smaller
// original triangle index -- so the hit record is bit-identical to the CPU restatement.
#include "shade_ops.hpp"
#include <string>

#include <hip/hip_ext.h>

#include "trace.hpp"
#include "traverse.hpp"
#include "camera_ops.hpp"
#include "stamps.hpp"
#include "cache_ops.hpp"

namespace pgrt {

constexpr int kTraceBlock = 256;
__device__ __forceinline__ int ray_count(const int* count_dev, int count_terms, int count_host, int cap) {
    if (!count_dev) return count_host;
    int n = 0;
    for (int k = 0; k < count_terms; ++k) n += count_dev[2 * k];  // stride 2: FrameCounters::alloc words
    return min(n, cap);
}

// While-while schedule (Aila & Laine 2009): a lane descends until it parks a leaf, the wave
// tests triangles once every active lane has one (r1 A/B, profiles/r1/trace_variants.txt: the
// fastest of {grid-stride, persistent fetch} x {while-while, one step per iteration}).
// SPILL: stack entries past kLdsStack go to a per-thread global region.  Without SPILL the
// whole stack is in LDS (dynamic size = BVH depth + 2 entries per lane, chosen at launch):
// every push/pop is a ds_write/ds_read instead of a flat access that must wait on vmcnt too.
// the rare spill accesses as out-of-line calls, so the LDS push/pop stays a plain ds access
// (a select between an LDS and a global pointer would become a flat access on every pop)
__device__ __noinline__ void spill_store(int* p, int v) { *p = v; }
__device__ __noinline__ int spill_load(const int* p) { return *p; }

// SFIN: the shadow queue of a ShadowFinal batch (its own instance: the completion code's registers
// stay out of the deep levels' traversal kernel)
template <bool COUNT, bool SPILL, bool SFIN>
__global__ __launch_bounds__(kTraceBlock) void k_trace(SceneView s, const float4* __restrict__ ro,
                                                       const float4* __restrict__ rd,
                                                       float4* __restrict__ hits,
                                                       const int* __restrict__ count_dev, int count_terms,
                                                       int count_host, int cap, int* __restrict__ gstack,
                                                       unsigned long long* __restrict__ counters,
                                                       float4 const_org, unsigned char* __restrict__ lit,
                                                       ShadowFinal sf) {
    PGRT_STAMP_BEGIN(s.stamps);
    extern __shared__ int lstack[];  // [entries][kTraceBlock]
    const int n0 = SFIN ? *sf.n0 : 0;  // level-0 shadow rays (ShadowFinal)
    const int tid = threadIdx.x;
    const int lane = __lane_id();
    const int n = ray_count(count_dev, count_terms, count_host, cap);
    int* gst = gstack + (size_t)(blockIdx.x * kTraceBlock + tid) * kGlobalStack;
    unsigned long long nvis = 0, ntest = 0, mvis = 0, mtest = 0;
#define PUSH(v)                                                       \
    do {                                                              \
        ++sp;                                                         \
        if (COUNT && sp > msp) msp = sp;                              \
        if (!SPILL || __builtin_expect(sp < kLdsStack, 1)) lstack[sp * kTraceBlock + tid] = (v); \
        else {                                                        \
            if (COUNT) ++nspill;                                      \
            spill_store(gst + (sp - kLdsStack), (v));                 \
        }                                                             \
    } while (0)
#define POP() pop_entry(sp)
    auto pop_entry = [&](int& spr) -> int {
        int v;
        if (!SPILL || __builtin_expect(spr < kLdsStack, 1)) v = lstack[spr * kTraceBlock + tid];
        else v = spill_load(gst + (spr - kLdsStack));
        --spr;
        return v;
    };
    const int wstride = gridDim.x * kTraceBlock;
    int stride_i = ((blockIdx.x * kTraceBlock + tid) >> 6) * 64 + lane - wstride;
    unsigned long long witer = 0, nspill = 0, mclk = 0, mray[6] = {0, 0, 0, 0, 0, 0};
    int msp = 0;
    for (;;) {
        stride_i += wstride;
        if (stride_i >= n) break;
        const int i = stride_i;
        const float4 o4 = ro ? ld_stream(ro + i) : const_org;
        const float4 d4 = ld_stream(rd + i);
        const float ox = o4.x, oy = o4.y, oz = o4.z, tnear = o4.w;
        const float dx = d4.x, dy = d4.y, dz = d4.z, tfar = d4.w;
        const float sdx = fabsf(dx) < 1e-30f ? copysignf(1e-30f, dx) : dx;
        const float sdy = fabsf(dy) < 1e-30f ? copysignf(1e-30f, dy) : dy;
        const float sdz = fabsf(dz) < 1e-30f ? copysignf(1e-30f, dz) : dz;
        const float idx = __builtin_amdgcn_rcpf(sdx), idy = __builtin_amdgcn_rcpf(sdy),
                    idz = __builtin_amdgcn_rcpf(sdz);
        const float oix = ox * idx, oiy = oy * idy, oiz = oz * idz;
        float best_t = tfar, best_u = 0.0f, best_v = 0.0f;
        int best_prim = -1;
        unsigned rvis = 0, rtest = 0;
        long long t_start = 0;
        unsigned long long rcyc_node = 0, rcyc_leaf = 0, rleaf = 0, rcyc_load = 0;
        if (COUNT) t_start = wall_clock64();
        int sp = 0;
        lstack[tid] = kSentinel;  // stack[0]
        int node = s.root;
        int leaf = 0;  // postponed leaf (negative code) or 0
        if (node < 0) {
            leaf = node;
            node = kSentinel;
        }
        if (!(tfar >= 0.0f)) {  // padding slots / empty segments: no traversal
            node = kSentinel;
            leaf = 0;
        }
        while (node != kSentinel || leaf < 0) {
            // ---- descend internal nodes until every active lane has parked a leaf ----
            long long tn0 = 0;
            if (COUNT) tn0 = clock64();
            // best_t only changes in the leaf phase: canonicalised once per descent, not per step
            const float bt = __builtin_canonicalizef(best_t);
            while ((unsigned)node < (unsigned)kSentinel) {
                if (COUNT) ++witer;
                // the stack top (the pop target when neither child is hit) is read before the node
                // fetch, so its LDS latency hides behind the global loads
                const int top = SPILL ? 0 : lstack[sp * kTraceBlock + tid];
                const BvhNode* nd = at_bytes(s.nodes, (unsigned)node << 6);
                long long tq0 = 0;
                if (COUNT) tq0 = clock64();
                const float4 a = nd->a, b = nd->b, c = nd->c;
                const int4 d = nd->d;
                if (COUNT) {
                    ++rvis;
                    // node-load round trip (instrumented variant only): wait for the data here
                    asm volatile("" ::"v"(a.x), "v"(b.x), "v"(c.x), "v"(d.x));
                    rcyc_load += (unsigned long long)(clock64() - tq0);
                }
                float t0, t1;
                const bool h0 = box_hit(a.x, a.y, a.z, a.w, c.x, c.y, idx, idy, idz, oix, oiy, oiz, bt, t0);
                const bool h1 = box_hit(b.x, b.y, b.z, b.w, c.z, c.w, idx, idy, idz, oix, oiy, oiz, bt, t1);
                if constexpr (!SPILL) {
                    // branch-free form: the far child is written above the top whether or not it is
                    // pushed (that slot is free), the stack pointer moves by selects
                    const bool any = h0 || h1;
                    const bool first0 = h0 && (!h1 || t0 <= t1);
                    const bool both = h0 && h1;
                    lstack[(sp + 1) * kTraceBlock + tid] = first0 ? d.y : d.x;
                    if (COUNT && both && sp + 1 > msp) msp = sp + 1;
                    node = any ? (first0 ? d.x : d.y) : top;
                    sp += both ? 1 : (any ? 0 : -1);
                } else {
                    if (!h0 && !h1) {
                        node = POP();
                    } else {
                        const bool first0 = h0 && (!h1 || t0 <= t1);
                        node = first0 ? d.x : d.y;
                        if (h0 && h1) PUSH(first0 ? d.y : d.x);
                    }
                }
                if (node < 0 && leaf == 0) {  // first leaf: park it and keep descending
                    leaf = node;
                    node = POP();
                }
                if (!__any(leaf == 0)) break;
            }
            long long tl0 = 0;
            if (COUNT) {
                tl0 = clock64();
                rcyc_node += (unsigned long long)(tl0 - tn0);
            }
            // ---- triangle tests for the parked leaves ----
            while (leaf < 0) {
                if (COUNT) {
                    ++witer;
                    ++rleaf;
                }
                const int first = leaf_first(leaf), end = first + leaf_count(leaf);
                // software-pipelined: the next triangle's loads are in flight while this one is
                // tested, so a leaf costs about one memory latency instead of one per triangle
                const float4* pt = at_bytes(s.tri, (unsigned)first * 48u);
                float4 p0 = pt[0], p1 = pt[1], p2 = pt[2];
                for (int k = first; k < end; ++k) {
                    if (COUNT) ++rtest;
                    const float4 q0 = p0, q1 = p1, q2 = p2;
                    if (k + 1 < end) {
                        const float4* pn = at_bytes(s.tri, (unsigned)(k + 1) * 48u);
                        p0 = pn[0];
                        p1 = pn[1];
                        p2 = pn[2];
                    }
                    tri_test(q0, q1, q2, ox, oy, oz, dx, dy, dz, tnear, tfar, best_t, best_u, best_v, best_prim);
                }
                leaf = 0;
                if (node < 0) {  // the node popped after parking is a leaf too: test it now
                    leaf = node;
                    node = POP();
                }
            }
            if (COUNT) rcyc_leaf += (unsigned long long)(clock64() - tl0);
        }
        if (lit) {  // is_illuminated (raytracer.cpp:163-173): no hit, or the occluder is dielectric
            const bool lv = best_prim < 0 || *at_bytes(s.prim_glass, (unsigned)best_prim) != 0;
            st_stream_nt(lit + i, (unsigned char)(lv ? 1 : 0));
            if constexpr (SFIN) {  // ShadowFinal: the ray's owner is complete with this verdict
                const float4 c = ld_stream(sf.contrib + i);
                // opaque_color's sum over the one light (from 0: 0 + x)
                const float4 v = lv ? make_float4(0.0f + c.x, 0.0f + c.y, 0.0f + c.z, 1.0f)
                                    : make_float4(0.0f, 0.0f, 0.0f, 1.0f);
                const int owner = __float_as_int(c.w);
                if (i < n0) {  // a level-0 pixel: get_pixel's sum and gamma, to the framebuffer
                    store_final_1spp(sf.fp, sf.tiles, sf.fo, owner, v);
                } else if (sf.colors[1]) {  // a deeper node: its colour (the queue is level-major)
                    int base = n0;
                    float4* dst = nullptr;
                    for (int L = 1; L < kMaxLevels; ++L) {
                        if (L >= sf.levels) break;
                        const int cnt = sf.n0[2 * L];
                        if (!dst && i < base + cnt) dst = sf.colors[L];
                        base += cnt;
                    }
                    if (dst) st_stream(dst + owner, v);
                }
            }
        } else
            st_stream(hits + i, make_float4(best_t, best_u, best_v, __int_as_float(best_prim)));
        if (COUNT) {
            const unsigned long long dt = (unsigned long long)(wall_clock64() - t_start);
            if (dt > mclk) {  // the longest ray's profile
                mclk = dt;
                mray[0] = (dt << 24) | min(rvis, 0xffffffu);
                mray[1] = (dt << 24) | min(rtest, 0xffffffu);
                mray[2] = (dt << 24) | min(rleaf, 0xffffffull);
                mray[3] = (dt << 24) | min(rcyc_node >> 6, 0xffffffull);
                mray[4] = (dt << 24) | min(rcyc_leaf >> 6, 0xffffffull);
                mray[5] = (dt << 24) | min(rcyc_load >> 6, 0xffffffull);
            }
            nvis += rvis;
            ntest += rtest;
            mvis = rvis > mvis ? rvis : mvis;
            mtest = rtest > mtest ? rtest : mtest;
        }
    }
#undef PUSH
#undef POP
    if (COUNT) {
        atomicAdd(&counters[0], nvis);
        atomicAdd(&counters[1], ntest);
        atomicMax(&counters[2], mvis);
        atomicMax(&counters[3], mtest);
        // wave loop iterations (node steps + leaf rounds): every active lane counts the same
        // iterations of its wave's loops only while it is inside them, so the max over lanes
        // is a lower bound of the wave's iteration count
        atomicMax(&counters[4], witer);
        atomicMax(&counters[5], mclk);  // longest ray, wall_clock64 ticks (100 MHz)
        atomicAdd(&counters[6], nspill);  // stack pushes past the LDS part
        atomicMax(&counters[7], (unsigned long long)msp);
        // the longest ray: (ticks << 24 | x) for x = visits, tests, leaf rounds, node-phase
        // cycles / 64, leaf-phase cycles / 64 (max picks the longest ray's record)
        for (int k = 0; k < 6; ++k) atomicMax(&counters[8 + k], mray[k]);
    }
    PGRT_STAMP_END(s.stamps);
}

// ---------------------------------------------------------------- 8-wide traversal
//
// Stack entries are node groups (child_base, hit bits << 24 | imask): the children of one wide
// node still to visit.  Hit bits sit at 24 + (slot ^ oct) with oct = the ray's direction octant,
// so taking the highest bit first visits children on the side the ray comes from first
// (slot bit k = child on the + side of axis k).  A visited node's leaf triangles are tested
// right away; its internal hits become the current group.
constexpr int kLdsStack8 = 8;  // 8-B groups: 8 x 8 B x 256 lanes = 16 KB per block


template <bool COUNT>
__global__ __launch_bounds__(kTraceBlock) void k_trace8(SceneView s, const float4* __restrict__ ro,
                                                        const float4* __restrict__ rd, float4* __restrict__ hits,
                                                        const int* __restrict__ count_dev, int count_terms,
                                                        int count_host, int cap, int* __restrict__ gstack,
                                                        unsigned long long* __restrict__ counters) {
    PGRT_STAMP_BEGIN(s.stamps);
    __shared__ uint2 lstack[kLdsStack8 * kTraceBlock];
    const int tid = threadIdx.x;
    const int n = ray_count(count_dev, count_terms, count_host, cap);
    uint2* gst = reinterpret_cast<uint2*>(gstack + (size_t)(blockIdx.x * kTraceBlock + tid) * kGlobalStack);
    unsigned long long nvis = 0, ntest = 0, mvis = 0, mtest = 0;
    for (int i = blockIdx.x * kTraceBlock + tid; i < n; i += gridDim.x * kTraceBlock) {
        const float4 o4 = ld_stream(ro + i);
        const float4 d4 = ld_stream(rd + i);
        const float ox = o4.x, oy = o4.y, oz = o4.z, tnear = o4.w;
        const float dx = d4.x, dy = d4.y, dz = d4.z, tfar = d4.w;
        const float sdx = fabsf(dx) < 1e-30f ? copysignf(1e-30f, dx) : dx;
        const float sdy = fabsf(dy) < 1e-30f ? copysignf(1e-30f, dy) : dy;
        const float sdz = fabsf(dz) < 1e-30f ? copysignf(1e-30f, dz) : dz;
        const float idx = __builtin_amdgcn_rcpf(sdx), idy = __builtin_amdgcn_rcpf(sdy),
                    idz = __builtin_amdgcn_rcpf(sdz);
        const bool px = idx >= 0.0f, py = idy >= 0.0f, pz = idz >= 0.0f;
        const unsigned oct = (dx > 0.0f ? 1u : 0u) | (dy > 0.0f ? 2u : 0u) | (dz > 0.0f ? 4u : 0u);
        float best_t = tfar, best_u = 0.0f, best_v = 0.0f;
        int best_prim = -1;
        unsigned rvis = 0, rtest = 0;
        int sp = 0;
        // current node group: the root alone (slot 0 of a virtual parent with child_base 0)
        unsigned gbase = 0, gbits = (1u << (24 + oct)) | 1u;
        if (!(tfar >= 0.0f)) gbits = 0;  // padding slots / empty segments
        unsigned tbase = 0, tbits = 0;
        for (;;) {
            // ---- node phase: lanes without pending triangles descend until every lane of the
            // wave holds a triangle group or is finished ("while-while", Aila & Laine 2009) ----
            while (tbits == 0u) {
                if (gbits <= 0x00ffffffu) {
                    if (sp == 0) break;  // traversal finished
                    --sp;
                    const uint2 g = sp < kLdsStack8 ? lstack[sp * kTraceBlock + tid] : gst[sp - kLdsStack8];
                    gbase = g.x;
                    gbits = g.y;
                }
                const int pb = 31 - __clz((int)gbits);
                gbits &= ~(1u << pb);
                const unsigned slot = (unsigned)(pb - 24) ^ oct;
                const int child = (int)gbase + __popc(gbits & 0xffu & ((1u << slot) - 1u));
                if (gbits > 0x00ffffffu) {  // siblings left: save the group
                    if (sp < kLdsStack8) lstack[sp * kTraceBlock + tid] = make_uint2(gbase, gbits);
                    else gst[sp - kLdsStack8] = make_uint2(gbase, gbits);
                    ++sp;
                }
                const Bvh8Node* nd = at_bytes(s.nodes8, (unsigned)child * (unsigned)sizeof(Bvh8Node));
                const float4 p = nd->p;
                const uint4 m = nd->m, qx = nd->qx, qy = nd->qy, qz = nd->qz;
                if (COUNT) ++rvis;
                const unsigned eb = __float_as_uint(p.w);
                const float ax = __uint_as_float((eb & 0xffu) << 23) * idx;
                const float ay = __uint_as_float(((eb >> 8) & 0xffu) << 23) * idy;
                const float az = __uint_as_float(((eb >> 16) & 0xffu) << 23) * idz;
                const float bx = (p.x - ox) * idx, by = (p.y - oy) * idy, bz = (p.z - oz) * idz;
                const unsigned imask = eb >> 24;
                // near / far planes by the ray's sign per axis
                const unsigned nx0 = px ? qx.x : qx.z, nx1 = px ? qx.y : qx.w;
                const unsigned fx0 = px ? qx.z : qx.x, fx1 = px ? qx.w : qx.y;
                const unsigned ny0 = py ? qy.x : qy.z, ny1 = py ? qy.y : qy.w;
                const unsigned fy0 = py ? qy.z : qy.x, fy1 = py ? qy.w : qy.y;
                const unsigned nz0 = pz ? qz.x : qz.z, nz1 = pz ? qz.y : qz.w;
                const unsigned fz0 = pz ? qz.z : qz.x, fz1 = pz ? qz.w : qz.y;
                unsigned nbits = 0, tb = 0;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int j = k & 3;
                    const unsigned wnx = k < 4 ? nx0 : nx1, wfx = k < 4 ? fx0 : fx1;
                    const unsigned wny = k < 4 ? ny0 : ny1, wfy = k < 4 ? fy0 : fy1;
                    const unsigned wnz = k < 4 ? nz0 : nz1, wfz = k < 4 ? fz0 : fz1;
                    const float t0 = fmaxf(fmaxf(fmaf(qb(wnx, j), ax, bx), fmaf(qb(wny, j), ay, by)),
                                           fmaxf(fmaf(qb(wnz, j), az, bz), 0.0f));
                    const float t1 = fminf(fminf(fmaf(qb(wfx, j), ax, bx), fmaf(qb(wfy, j), ay, by)),
                                           fminf(fmaf(qb(wfz, j), az, bz), best_t));
                    const unsigned meta = ((k < 4 ? m.z : m.w) >> (8 * j)) & 0xffu;
                    if (meta != 0u && t0 <= t1 * 1.000001f) {
                        if ((imask >> k) & 1u) nbits |= 1u << (24 + (k ^ oct));
                        else tb |= wide_leaf_bits(meta);
                    }
                }
                gbase = m.x;
                gbits = nbits | imask;
                tbase = m.y;
                tbits = tb;
            }
            if (tbits == 0u) break;  // no triangles pending and no nodes left
            // ---- triangle phase: loads of the next triangle overlap the current test ----
            int k = (int)tbase + __ffs((int)tbits) - 1;
            tbits &= tbits - 1u;
            float4 p0 = s.tri8[3 * k], p1 = s.tri8[3 * k + 1], p2 = s.tri8[3 * k + 2];
            for (;;) {
                const float4 q0 = p0, q1 = p1, q2 = p2;
                const bool more = tbits != 0u;
                if (more) {
                    k = (int)tbase + __ffs((int)tbits) - 1;
                    tbits &= tbits - 1u;
                    p0 = s.tri8[3 * k];
                    p1 = s.tri8[3 * k + 1];
                    p2 = s.tri8[3 * k + 2];
                }
                if (COUNT) ++rtest;
                tri_test(q0, q1, q2, ox, oy, oz, dx, dy, dz, tnear, tfar, best_t, best_u, best_v, best_prim);
                if (!more) break;
            }
        }
        st_stream(hits + i, make_float4(best_t, best_u, best_v, __int_as_float(best_prim)));
        if (COUNT) {
            nvis += rvis;
            ntest += rtest;
            mvis = rvis > mvis ? rvis : mvis;
            mtest = rtest > mtest ? rtest : mtest;
        }
    }
    if (COUNT) {
        atomicAdd(&counters[14], nvis);  // 80-B wide-node visits
        atomicAdd(&counters[1], ntest);
        atomicMax(&counters[2], mvis);
        atomicMax(&counters[3], mtest);
    }
    PGRT_STAMP_END(s.stamps);
}


// ---------------------------------------------------------------- 8 lanes per ray, 8-wide BVH
//
// (the group traversal itself is trace8_group, traverse.hpp)

// RESUME: the rays are a budgeted packet launch's deferred rays (perm = the defer list): each
// starts from the closest hit the packet found so far (hits[i]), which bounds its traversal
template <bool COUNT, int G, bool RESUME = false>
__global__ __launch_bounds__(kTraceBlock) void k_trace8g(SceneView s, const float4* __restrict__ ro,
                                                         const float4* __restrict__ rd, float4* __restrict__ hits,
                                                         const int* __restrict__ count_dev, int count_terms,
                                                         int count_host, int cap,
                                                         unsigned long long* __restrict__ counters,
                                                         const int* __restrict__ perm) {
    static_assert(G == 4 || G == 8, "lanes per ray");
    PGRT_STAMP_BEGIN(s.stamps);
    constexpr int kGroups = kTraceBlock / G;
    __shared__ uint2 gstk[kGroupStack][kGroups];
    const int tid = threadIdx.x;
    const int k = tid & (G - 1);  // lane within the group
    const int gib = tid / G;      // group within the block
    const int gshift = __lane_id() & ~(G - 1);
    const int n = ray_count(count_dev, count_terms, count_host, cap);
    unsigned long long nvis = 0, ntest = 0, mvis = 0, mtest = 0;
    for (int slot_i = blockIdx.x * kGroups + gib; slot_i < n; slot_i += gridDim.x * kGroups) {
        const int i = perm ? ld_stream_nt(perm + slot_i) : slot_i;  // RESUME: the deferred ray of this slot
        const float4 o4 = ld_stream(ro + i);
        const float4 d4 = ld_stream(rd + i);
        float best_t = d4.w, best_u = 0.0f, best_v = 0.0f;
        int best_prim = -1;
        if constexpr (RESUME) {  // the packet's closest hit so far (its t is <= tfar)
            const float4 h = ld_stream(hits + i);
            best_t = h.x;
            best_u = h.y;
            best_v = h.z;
            best_prim = __float_as_int(h.w);
        }
        unsigned rvis = 0, rtest = 0;
        trace8_group<G, COUNT>(s, o4, d4, k, gshift, &gstk[0][gib], kGroups, best_t, best_u, best_v, best_prim, rvis,
                               rtest);
        if (k == 0) st_stream(hits + i, make_float4(best_t, best_u, best_v, __int_as_float(best_prim)));
        if (COUNT && k == 0) {
            nvis += rvis;
            ntest += rtest;
            mvis = rvis > mvis ? rvis : mvis;
            mtest = rtest > mtest ? rtest : mtest;
        }
    }
    if (COUNT && k == 0) {
        atomicAdd(&counters[14], nvis);  // 80-B wide-node visits
        atomicAdd(&counters[1], ntest);
        atomicMax(&counters[2], mvis);
        atomicMax(&counters[3], mtest);
    }
    PGRT_STAMP_END(s.stamps);
}


// ---------------------------------------------------------------- wave packets (primary rays)
//
// Level 0 holds coherent rays: one wave = one 8x8 pixel block (or one pixel's samples).  Here the
// wave traverses the binary BVH as one packet: a single wave-uniform node stream (the union of
// its rays' paths), every node and triangle fetched ONCE per wave by scalar loads into SGPRs
// (constant address space), each lane testing its own ray against them.  A child is entered
// when any lane's ray hits it (ballot), nearer-first by majority vote; each lane keeps its own
// closest hit, so results are the one-lane kernel's.  No per-lane gathers go through the
// texture path, and the per-lane state is small (no node data in VGPRs).
typedef const __attribute__((address_space(4))) float* cfloat_ptr;
__device__ __forceinline__ float4 cload4(cfloat_ptr p) { return make_float4(p[0], p[1], p[2], p[3]); }
constexpr int kPktStack = 64;  // wave-uniform stack entries (>= BVH depth + 2)

// The packet's internal-node loop: from `node` down to the next leaf (returned) or kSentinel.
// SGN 0-7: every live ray's direction has sign bits SGN (1 = x < 0, 2 = y, 4 = z), so each
// axis's near / far plane is a fixed operand (box_hit_nf); SGN 8: mixed signs (box_hit).
// BUDGET: stop with kDefer once `steps` (wave-uniform, counted across calls) exceeds `budget`
constexpr int kDefer = 0x7ffffffe;  // pkt_nodes result: the wave ran out of steps (not a node index)
template <int SGN, bool COUNT, bool SAMPLE, bool BUDGET>
__device__ __forceinline__ int pkt_nodes(const cfloat_ptr nodes, int node, int& sp, int* wstk, float bt, float idx,
                                         float idy, float idz, float oix, float oiy, float oiz, bool live,
                                         unsigned& rvis, unsigned& useful, unsigned& live_steps, int& steps,
                                         int budget) {
    while ((unsigned)node < (unsigned)kSentinel) {
        if constexpr (BUDGET) {
            if (++steps > budget) return kDefer;
        }
        // the pop target, read before the node loads (wstk[0] holds kSentinel): one wait for both
        const int top = __builtin_amdgcn_readfirstlane(wstk[sp]);
        // base + zero-extended 32-bit byte offset: the scalar loads take it as their offset operand
        const cfloat_ptr nd = (cfloat_ptr)((const __attribute__((address_space(4))) char*)nodes +
                                           (unsigned long long)((unsigned)node << 6));
        const float4 a = cload4(nd), b = cload4(nd + 4), c = cload4(nd + 8);
        const int4 d = make_int4(__float_as_int(nd[12]), __float_as_int(nd[13]), __float_as_int(nd[14]),
                                 __float_as_int(nd[15]));
        // the child indices with the boxes, in one scalar-load wait (not a second one after the
        // box tests)
        asm volatile("" ::"s"(d.x), "s"(d.y));
        if (COUNT) ++rvis;
        float t0, t1;
        bool h0, h1;
        if constexpr (SGN < 8) {
            constexpr bool nx = SGN & 1, ny = SGN & 2, nz = SGN & 4;
            h0 = box_hit_nf(nx ? a.y : a.x, nx ? a.x : a.y, ny ? a.w : a.z, ny ? a.z : a.w, nz ? c.y : c.x,
                            nz ? c.x : c.y, idx, idy, idz, oix, oiy, oiz, bt, t0);
            h1 = box_hit_nf(nx ? b.y : b.x, nx ? b.x : b.y, ny ? b.w : b.z, ny ? b.z : b.w, nz ? c.w : c.z,
                            nz ? c.z : c.w, idx, idy, idz, oix, oiy, oiz, bt, t1);
        } else {
            h0 = box_hit(a.x, a.y, a.z, a.w, c.x, c.y, idx, idy, idz, oix, oiy, oiz, bt, t0);
            h1 = box_hit(b.x, b.y, b.z, b.w, c.z, c.w, idx, idy, idz, oix, oiy, oiz, bt, t1);
        }
        if (SAMPLE && live) {
            ++live_steps;
            useful += (h0 || h1) ? 1u : 0u;
        }
        const unsigned long long b0 = __ballot(h0), b1 = __ballot(h1);
        if (b0 == 0ull && b1 == 0ull) {
            node = top;  // kSentinel at sp == 0: the traversal is over (sp -1 is never read)
            --sp;
        } else if (b0 != 0ull && b1 != 0ull) {
            // nearer first, by majority of the lanes that hit both
            const unsigned long long near0 = __ballot(h0 && h1 && t0 <= t1);
            const unsigned long long both = b0 & b1;
            const bool first0 = 2 * __popcll(near0) >= __popcll(both);
            wstk[++sp] = first0 ? d.y : d.x;
            node = first0 ? d.x : d.y;
        } else {
            node = b0 != 0ull ? d.x : d.y;
        }
    }
    return node;
}

// SAMPLE: this block measures packet utilisation (a block-uniform choice; the loop without the
// counters is a separate copy, so unsampled blocks pay nothing for them)
// BUDGET (bounce levels): a wave that has taken `budget` node / triangle steps stops; its live
// rays keep the closest hit found so far and go to defer_list (k_trace8g<RESUME> finishes them)
template <bool COUNT, bool GEN, bool SAMPLE, bool BUDGET>
__device__ __forceinline__ void pkt_trace(const SceneView& s, const float4* __restrict__ ro,
                                          const float4* __restrict__ rd, float4* __restrict__ hits, int n,
                                          unsigned long long* __restrict__ counters, const PrimaryGen& gen,
                                          unsigned long long* __restrict__ util, int (*wstack)[kPktStack],
                                          int budget, int* __restrict__ defer_list,
                                          int* __restrict__ defer_count) {
    static_assert(!(GEN && BUDGET), "level 0 has no step budget");
    const int wib = threadIdx.x >> 6;
    const int lane = __lane_id();
    const cfloat_ptr nodes = (cfloat_ptr)(const void*)s.nodes;  // 16 floats per node
    const cfloat_ptr tris = (cfloat_ptr)(const void*)s.tri;     // 12 floats per triangle
    unsigned long long nvis = 0, ntest = 0;
    // packet utilisation (sampled: every 8th block): internal-node steps at which this lane's ray
    // hit a child box, and steps it spent live -- their ratio is the fraction of the wave's node
    // stream the ray needed (pgrt_config.packet_levels AUTO decides per level from it)
    constexpr bool sample = SAMPLE;
    unsigned useful = 0, live_steps = 0;
    if (lane == 0) wstack[wib][0] = kSentinel;  // the bottom entry: entries are wstack[wib][1..sp]
    for (int base = (blockIdx.x * kTraceBlock) + wib * 64; base < n; base += gridDim.x * kTraceBlock) {
        const int slot_i = base + lane;
        const bool valid = slot_i < n;
        const int i = slot_i;
        float4 o4 = make_float4(0, 0, 0, 0), d4 = make_float4(0, 0, 1, -1.0f);
        bool pv = false;
        if (valid) {
            if constexpr (GEN) {
                pv = primary_ray(gen.cam, gen.fp, gen.tiles, i, o4, d4);  // level 0: no ray queue read
                // the level-0 shade reads the rays back; pinhole rays share origin, tnear and
                // medium (store_ro / store_time NULL: the shade takes them from the camera)
                st_stream(gen.store_rd + i, d4);
                if (gen.store_ro) {
                    st_stream(gen.store_ro + i, o4);
                    st_stream_nt(gen.store_time + i, pv ? PGRT_IOR_AIR : 0.0f);
                }
            } else {
                o4 = ld_stream(ro + i);
                d4 = ld_stream(rd + i);
            }
        }
        const float ox = o4.x, oy = o4.y, oz = o4.z, tnear = o4.w;
        const float dx = d4.x, dy = d4.y, dz = d4.z, tfar = d4.w;
        const float sdx = fabsf(dx) < 1e-30f ? copysignf(1e-30f, dx) : dx;
        const float sdy = fabsf(dy) < 1e-30f ? copysignf(1e-30f, dy) : dy;
        const float sdz = fabsf(dz) < 1e-30f ? copysignf(1e-30f, dz) : dz;
        const float idx = __builtin_amdgcn_rcpf(sdx), idy = __builtin_amdgcn_rcpf(sdy),
                    idz = __builtin_amdgcn_rcpf(sdz);
        const float oix = ox * idx, oiy = oy * idy, oiz = oz * idz;
        const bool live = valid && tfar >= 0.0f;  // padding slots / empty segments never hit
        float best_t = live ? tfar : -1.0f;       // a dead lane's boxes all miss (t1 < 0 <= t0)
        float best_u = 0.0f, best_v = 0.0f;
        int best_prim = -1;
        int sp = 0;
        int node = s.root;
        const unsigned long long lmask = __ballot(live);
        if (lmask == 0ull) node = kSentinel;
        // direction signs shared by every live ray of the packet (coherent waves: nearly always)
        // -> a copy of the node loop with each axis's near / far plane fixed at compile time;
        // mixed signs (sgn 8) take the min / max form
        const unsigned long long negx = __ballot(live && idx < 0.0f), negy = __ballot(live && idy < 0.0f),
                                 negz = __ballot(live && idz < 0.0f);
        const bool uni = (negx == 0ull || negx == lmask) && (negy == 0ull || negy == lmask) &&
                         (negz == 0ull || negz == lmask);
        const int sgn = __builtin_amdgcn_readfirstlane(
            uni ? (negx != 0ull ? 1 : 0) | (negy != 0ull ? 2 : 0) | (negz != 0ull ? 4 : 0) : 8);
        unsigned rvis = 0, rtest = 0;
        int steps = 0;
        node = __builtin_amdgcn_readfirstlane(node);  // wave-uniform by construction
        for (;;) {
            // internal nodes (0 <= node < kSentinel) in a loop of their own: the leaf code, which
            // updates the closest hits, stays out of it (no register copies of them per step)
            // best_t is constant over this loop: canonicalised once (IEEE min/max would re-quiet it
            // every step)
            const float bt = __builtin_canonicalizef(best_t);
#define PGRT_PKT_NODES(S)                                                                                      \
    node = pkt_nodes<S, COUNT, SAMPLE, BUDGET>(nodes, node, sp, wstack[wib], bt, idx, idy, idz, oix, oiy, oiz, live, \
                                               rvis, useful, live_steps, steps, budget)
            switch (sgn) {
                case 0: PGRT_PKT_NODES(0); break;
                case 1: PGRT_PKT_NODES(1); break;
                case 2: PGRT_PKT_NODES(2); break;
                case 3: PGRT_PKT_NODES(3); break;
                case 4: PGRT_PKT_NODES(4); break;
                case 5: PGRT_PKT_NODES(5); break;
                case 6: PGRT_PKT_NODES(6); break;
                case 7: PGRT_PKT_NODES(7); break;
                default: PGRT_PKT_NODES(8); break;
            }
#undef PGRT_PKT_NODES
            if (node == kSentinel || (BUDGET && node == kDefer)) break;
            // leaf: its triangles against every lane's ray
            const int first = leaf_first(node), end = first + leaf_count(node);
            if constexpr (BUDGET) steps += end - first;
            for (int k = first; k < end; ++k) {
                // base + zero-extended 32-bit byte offsets (scalar-load offset operands, as the nodes)
                const cfloat_ptr q = (cfloat_ptr)((const __attribute__((address_space(4))) char*)tris +
                                                  (unsigned long long)((unsigned)k * 48u));
                const float4 q0 = cload4(q), q1 = cload4(q + 4), q2 = cload4(q + 8);
                if (COUNT) ++rtest;
                const float4 ng = cload4((cfloat_ptr)((const __attribute__((address_space(4))) char*)s.tri_ng +
                                                      (unsigned long long)((unsigned)k << 4)));  // precomputed Ng
                // whole records, in one wait: the unused words keep the loads at full width (3 + 1
                // scalar loads instead of 7 narrowed ones)
                asm volatile("" ::"s"(q0.w), "s"(q1.w), "s"(q2.w), "s"(ng.w));
                if (live)
                    tri_test_ng(q0, q1, q2, ng, ox, oy, oz, dx, dy, dz, tnear, tfar, best_t, best_u, best_v,
                                best_prim);
            }
            node = __builtin_amdgcn_readfirstlane(wstack[wib][sp]);  // wstack[wib][0]: kSentinel
            sp -= sp > 0 ? 1 : 0;
        }
        if constexpr (GEN) {
            if (gen.hitmask) {  // 1-spp level 0 (L0Final): hit records of the hits only + the wave's mask
                const bool hit = live && best_prim >= 0;
                const unsigned long long hm = __ballot(hit);
                if (hit) st_stream(hits + i, make_float4(best_t, best_u, best_v, __int_as_float(best_prim)));
                if (lane == 0) st_stream_nt(gen.hitmask + (base >> 6), hm);
                if (COUNT && lane == 0) {
                    nvis += rvis;
                    ntest += rtest;
                }
                continue;
            }
        }
        if (valid) st_stream(hits + i, make_float4(live ? best_t : tfar, best_u, best_v, __int_as_float(best_prim)));
        if constexpr (BUDGET) {
            if (node == kDefer) {  // out of steps: the live rays to the 8-lanes-per-ray kernel
                const unsigned long long dm = __ballot(live);
                int b = 0;
                if (lane == 0) b = atomicAdd(defer_count, (int)__popcll(dm));
                b = __builtin_amdgcn_readfirstlane(b);
                if (live)
                    defer_list[b + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(dm >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((unsigned)dm, 0u))] = i;
            }
        }
        if (COUNT && lane == 0) {
            nvis += rvis;
            ntest += rtest;
        }
    }
    if (sample) {  // wave sums, one atomic pair per wave of the sampled blocks
        unsigned long long u = useful, l = live_steps;
        for (int off = 32; off >= 1; off >>= 1) {
            u += __shfl_xor(u, off, 64);
            l += __shfl_xor(l, off, 64);
        }
        if (lane == 0 && l > 0) {
            atomicAdd(&util[0], u);
            atomicAdd(&util[1], l);
        }
    }
    if (COUNT && lane == 0) {  // per-wave counts (one packet step = one node visit)
        atomicAdd(&counters[0], nvis);
        atomicAdd(&counters[1], ntest);
    }
}

// MINW: minimum waves per SIMD the register allocation must allow (launch bound).  The level-0
// kernel (GEN) uses 67 VGPRs -> 7 waves; big scenes (BVH + triangles far beyond the L2, fetches
// that wait on the MALL / HBM) take the 8-wave build (59 VGPRs, more SGPR spills): C5 19.6 ->
// 19.1 ms/frame; since the lighter r4 ray generation the avenger proxy's level 0 gains too (r4z A/B,
// profiles/r4/ab_r4z_shade_block_l0_waves.txt: C2 400 frames 0.1525 -> 0.1496 ms/frame)
template <bool COUNT, bool GEN, int MINW, bool BUDGET = false>
__global__ __launch_bounds__(kTraceBlock, MINW) void k_trace_pkt(SceneView s, const float4* __restrict__ ro,
                                                           const float4* __restrict__ rd, float4* __restrict__ hits,
                                                           const int* __restrict__ count_dev, int count_terms,
                                                           int count_host, int cap,
                                                           unsigned long long* __restrict__ counters, PrimaryGen gen,
                                                           unsigned long long* __restrict__ util, int budget,
                                                           int* __restrict__ defer_list, int* __restrict__ defer_count) {
    PGRT_STAMP_BEGIN(s.stamps);
    __shared__ int wstack[kTraceBlock / 64][kPktStack];
    const int n = ray_count(count_dev, count_terms, count_host, cap);
    if constexpr (GEN) {
        if (gen.store_count && blockIdx.x == 0 && threadIdx.x == 0) *gen.store_count = n;
        // level 0 is always traced as packets: its utilisation is never sampled
        pkt_trace<COUNT, GEN, false, false>(s, ro, rd, hits, n, counters, gen, util, wstack, 0, nullptr, nullptr);
    } else {
        // packet utilisation sampled in every 8th block (pgrt_config.packet_levels AUTO)
        if (util != nullptr && (blockIdx.x & 7) == 0)
            pkt_trace<COUNT, GEN, true, BUDGET>(s, ro, rd, hits, n, counters, gen, util, wstack, budget, defer_list,
                                                defer_count);
        else
            pkt_trace<COUNT, GEN, false, BUDGET>(s, ro, rd, hits, n, counters, gen, util, wstack, budget, defer_list,
                                                 defer_count);
    }
    PGRT_STAMP_END(s.stamps);
}

// Kernel-exact launch timing (profile frames): the closest-hit launch records the caller's
// events itself (hipExtLaunchKernel: taken by the packet processor at kernel start / end, the
// same clock rocprofv3's kernel trace reads), instead of event records queued around it.
namespace {
thread_local hipEvent_t t_ev_start = nullptr, t_ev_stop = nullptr;
}
void set_trace_events(hipEvent_t start, hipEvent_t stop) {
    t_ev_start = start;
    t_ev_stop = stop;
}
#define PGRT_TLAUNCH(kernel, grid, block, lds, stream, ...) \
    hipExtLaunchKernelGGL(kernel, grid, block, lds, stream, t_ev_start, t_ev_stop, 0, __VA_ARGS__)

bool trace_packets_available(const SceneView& s) {
    return !s.wide && s.root >= 0 && s.depth + 2 <= kPktStack;
}

// 4 lanes per ray (two child slots each) above this many rays, 8 at or below it (r1 A/B)
constexpr int kGroup8Max = 150000;

bool launch_trace(const SceneView& s_in, const TraceLaunch& t, hipStream_t stream) {
    SceneView s = s_in;  // s.stamps: this launch's timeline slots (stamps.hpp)
    const int max_count = t.max_count;
    if (max_count <= 0) return false;
    PGRT_REQUIRE((t.ro && !t.lit) || (!s.wide && !t.packets && !t.gen && !t.allow_group), PGRT_ERR_INVALID_ARGUMENT,
                 "compact shadow queues are traced by the one-lane binary kernel only");
    const int ex = t.expect > 0 && t.expect < max_count ? t.expect : max_count;  // grid sizing only
    if (s.wide) {
        int grid = ceil_div(ex, kTraceBlock);
        if (grid > t.gstack_threads / kTraceBlock) grid = t.gstack_threads / kTraceBlock;
        s.stamps = stamp_next(t.lit || !t.allow_group ? kStampTraceShadow : kStampTrace, t.level, grid, kTraceBlock);
        if (t.count)
            PGRT_TLAUNCH((k_trace8<true>), dim3(grid), dim3(kTraceBlock), 0, stream, s, t.ro, t.rd, t.hits,
                         t.count_dev, t.count_terms, t.count_host, max_count, t.gstack, t.counters);
        else
            PGRT_TLAUNCH((k_trace8<false>), dim3(grid), dim3(kTraceBlock), 0, stream, s, t.ro, t.rd, t.hits,
                         t.count_dev, t.count_terms, t.count_host, max_count, t.gstack, t.counters);
        return true;
    }
    // coherent waves (level 0's 8x8-pixel blocks, the coherent bounce levels): packet traversal
    if ((t.packets || t.gen) && trace_packets_available(s)) {
        int grid = ceil_div(ex, kTraceBlock);
        if (grid > 16384) grid = 16384;
        const PrimaryGen g = t.gen ? *t.gen : PrimaryGen{};
        // a step budget on a bounce level: the waves out of steps hand their rays to k_trace8g
        const bool budget = !t.gen && t.budget > 0 && t.defer_list && t.defer_count && s.depth8 + 1 <= kGroupStack;
        hipEvent_t ev_stop = budget && t.resume ? nullptr : t_ev_stop;  // profile timing spans both launches
#define PGRT_LAUNCH_P(C, G, W, B)                                                                              \
    hipExtLaunchKernelGGL((k_trace_pkt<C, G, W, B>), dim3(grid), dim3(kTraceBlock), 0, stream, t_ev_start, ev_stop, \
                          0, s, t.ro, t.rd, t.hits, t.count_dev, t.count_terms, t.count_host, max_count, t.counters, \
                          g, t.pkt_util, t.budget, t.defer_list, t.defer_count)
        s.stamps = stamp_next(kStampTracePkt, t.level, grid, kTraceBlock);
        if (t.count) {
            if (t.gen) PGRT_LAUNCH_P(true, true, 1, false);
            else if (budget) PGRT_LAUNCH_P(true, false, 1, true);
            else PGRT_LAUNCH_P(true, false, 1, false);
        } else if (t.gen) {
            PGRT_LAUNCH_P(false, true, 8, false);  // every scene (r4z: the avenger too)
        } else if (budget) {
            PGRT_LAUNCH_P(false, false, 1, true);
        } else {
            PGRT_LAUNCH_P(false, false, 1, false);
        }
#undef PGRT_LAUNCH_P
        if (budget && t.resume) {  // the deferred rays: 8 lanes per ray, from the packet's closest hits
            // grid from the previous deferral count; with none known (a level's first packet frame,
            // e.g. AUTO's start or probe on an incoherent scene, where most waves run out of steps),
            // from the level's rays -- a 1024-ray grid striding over millions of deferred rays made
            // single launches of 0.1-0.4 s on C5 (profiles/r3/c5_kernel_stats_r3fin.csv)
            const int dex = std::max(t.defer_expect > 0 ? t.defer_expect : ex, 1024);
            const int g8 = std::min(16384, ceil_div(dex, kTraceBlock / 8));
            s.stamps = stamp_next(kStampTraceResume, t.level, g8, kTraceBlock);
            if (t.count)
                hipExtLaunchKernelGGL((k_trace8g<true, 8, true>), dim3(g8), dim3(kTraceBlock), 0, stream, nullptr,
                                      t_ev_stop, 0, s, t.ro, t.rd, t.hits, t.defer_count, 1, 0, max_count, t.counters,
                                      t.defer_list);
            else
                hipExtLaunchKernelGGL((k_trace8g<false, 8, true>), dim3(g8), dim3(kTraceBlock), 0, stream, nullptr,
                                      t_ev_stop, 0, s, t.ro, t.rd, t.hits, t.defer_count, 1, 0, max_count, t.counters,
                                      t.defer_list);
        }
        return true;
    }
    if (t.allow_group && ex <= s.group_max && s.depth8 + 1 <= kGroupStack) {
        // 8 lanes per ray for the smallest queues (the latency floor of the slowest ray),
        // 4 lanes (two child slots each) when there are enough rays to fill the machine
        const bool g4 = ex > kGroup8Max;
        s.stamps = stamp_next(kStampTrace8g, t.level, std::min(16384, ceil_div(ex, kTraceBlock / (g4 ? 4 : 8))),
                              kTraceBlock);
#define PGRT_LAUNCH_G(C, G)                                                                                       \
    PGRT_TLAUNCH((k_trace8g<C, G>), dim3(std::min(16384, ceil_div(ex, kTraceBlock / G))), dim3(kTraceBlock), 0, \
                 stream, s, t.ro, t.rd, t.hits, t.count_dev, t.count_terms, t.count_host, max_count, t.counters, nullptr)
        if (t.count) {
            if (g4) PGRT_LAUNCH_G(true, 4); else PGRT_LAUNCH_G(true, 8);
        } else {
            if (g4) PGRT_LAUNCH_G(false, 4); else PGRT_LAUNCH_G(false, 8);
        }
#undef PGRT_LAUNCH_G
        return true;
    }
    int grid = ceil_div(ex, kTraceBlock);
    if (grid > t.gstack_threads / kTraceBlock) grid = t.gstack_threads / kTraceBlock;
    // all-LDS stack when the BVH depth fits (depth + 2 entries per lane, <= 64 KB per block)
    const int entries = s.depth + 2;
    const bool spill = entries * kTraceBlock * 4 > 65536;
    const size_t lds = (size_t)(spill ? kLdsStack : entries) * kTraceBlock * sizeof(int);
    s.stamps = stamp_next(t.lit || !t.allow_group ? kStampTraceShadow : kStampTrace, t.level, grid, kTraceBlock);
#define PGRT_LAUNCH(C, S, F)                                                                                      \
    PGRT_TLAUNCH((k_trace<C, S, F>), dim3(grid), dim3(kTraceBlock), lds, stream, s, t.ro, t.rd, t.hits, t.count_dev, \
                 t.count_terms, t.count_host, max_count, t.gstack, t.counters, t.const_org, t.lit, t.sfin)
    if (t.sfin.contrib && t.lit) {  // ShadowFinal: the compact shadow queue's own instance
        if (t.count) {
            if (spill) PGRT_LAUNCH(true, true, true); else PGRT_LAUNCH(true, false, true);
        } else {
            if (spill) PGRT_LAUNCH(false, true, true); else PGRT_LAUNCH(false, false, true);
        }
    } else if (t.count) {
        if (spill) PGRT_LAUNCH(true, true, false); else PGRT_LAUNCH(true, false, false);
    } else {
        if (spill) PGRT_LAUNCH(false, true, false); else PGRT_LAUNCH(false, false, false);
    }
#undef PGRT_LAUNCH
    return true;
}


// ---------------------------------------------------------------- any hit (rtcOccluded1)
//
// Embree's occlusion query (rtcore_scene.h: rtcOccluded1): is there ANY triangle hit with t in
// (tnear, tfar]?  One lane per ray over the binary BVH, LDS stack sized to the tree depth,
// nearer child first, and the traversal stops at the first accepted triangle.  The per-triangle
// acceptance is the closest-hit kernel's (tri_test), so occluded == (closest hit exists).
__global__ __launch_bounds__(kTraceBlock) void k_occluded(SceneView s, const float4* __restrict__ ro,
                                                          const float4* __restrict__ rd, int n,
                                                          int* __restrict__ occluded) {
    extern __shared__ int lstack[];  // [depth + 2][kTraceBlock]
    const int tid = threadIdx.x;
    for (int i = blockIdx.x * kTraceBlock + tid; i < n; i += gridDim.x * kTraceBlock) {
            const float4 o4 = ro[i];
        const float4 d4 = rd[i];
        const float ox = o4.x, oy = o4.y, oz = o4.z, tnear = o4.w;
        const float dx = d4.x, dy = d4.y, dz = d4.z, tfar = d4.w;
        const float sdx = fabsf(dx) < 1e-30f ? copysignf(1e-30f, dx) : dx;
        const float sdy = fabsf(dy) < 1e-30f ? copysignf(1e-30f, dy) : dy;
        const float sdz = fabsf(dz) < 1e-30f ? copysignf(1e-30f, dz) : dz;
        const float idx = __builtin_amdgcn_rcpf(sdx), idy = __builtin_amdgcn_rcpf(sdy),
                    idz = __builtin_amdgcn_rcpf(sdz);
        const float oix = ox * idx, oiy = oy * idy, oiz = oz * idz;
        int hit = 0;
        int sp = 0;
        lstack[tid] = kSentinel;
        int node = (tfar >= 0.0f) ? s.root : kSentinel;
        while (node != kSentinel && !hit) {
            if (node >= 0) {
                const BvhNode* nd = s.nodes + node;
                const float4 a = nd->a, b = nd->b, c = nd->c;
                const int4 d = nd->d;
                float t0, t1;
                const bool h0 = box_hit(a.x, a.y, a.z, a.w, c.x, c.y, idx, idy, idz, oix, oiy, oiz, tfar, t0);
                const bool h1 = box_hit(b.x, b.y, b.z, b.w, c.z, c.w, idx, idy, idz, oix, oiy, oiz, tfar, t1);
                if (h0 && h1) {
                    const bool first0 = t0 <= t1;
                    lstack[++sp * kTraceBlock + tid] = first0 ? d.y : d.x;
                    node = first0 ? d.x : d.y;
                } else if (h0 || h1) {
                    node = h0 ? d.x : d.y;
                } else {
                    node = lstack[(sp--) * kTraceBlock + tid];
                }
            } else {
                const int first = leaf_first(node), end = first + leaf_count(node);
                for (int k = first; k < end && !hit; ++k) {
                    float bt = tfar, bu = 0.0f, bv = 0.0f;
                    int bp = -1;
                    tri_test(s.tri[3 * k], s.tri[3 * k + 1], s.tri[3 * k + 2], ox, oy, oz, dx, dy, dz, tnear, tfar,
                             bt, bu, bv, bp);
                    hit = bp >= 0;
                }
                node = lstack[(sp--) * kTraceBlock + tid];
            }
        }
        occluded[i] = hit;
    }
}

void launch_occluded(const SceneView& s, const float4* ro, const float4* rd, int n, int* occluded,
                     hipStream_t stream) {
    if (n <= 0) return;
    PGRT_REQUIRE(s.depth + 2 <= 64, PGRT_ERR_INVALID_ARGUMENT, "BVH too deep for the any-hit stack");
    int grid = ceil_div(n, kTraceBlock);
    if (grid > 16384) grid = 16384;
    const size_t lds = (size_t)(s.depth + 2) * kTraceBlock * sizeof(int);
    hipLaunchKernelGGL(k_occluded, dim3(grid), dim3(kTraceBlock), lds, stream, s, ro, rd, n, occluded);
}

int trace_block_size() { return kTraceBlock; }

}  // namespace pgrt
