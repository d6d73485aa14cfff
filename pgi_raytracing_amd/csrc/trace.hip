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
#include "trace.hpp"

namespace pgrt {

constexpr int kTraceBlock = 256;
constexpr int kLdsStack = 32;
constexpr int kSentinel = 0x7fffffff;  // bottom of every stack: "traversal finished"
constexpr int kResidentBlocks = 256 * 5;  // 32 KB LDS per block -> 5 blocks per CU

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

// PERSIST: waves pull 64-ray batches from `fetch` (else: static grid-stride assignment).
// WW: while-while descent until every lane parked a leaf (else: one node step per iteration,
// internal-node and leaf work interleaved).  Both are schedule choices: results are identical.
template <bool COUNT, bool PERSIST, bool WW>
__global__ __launch_bounds__(kTraceBlock) void k_trace(SceneView s, const float4* __restrict__ ro,
                                                       const float4* __restrict__ rd,
                                                       float4* __restrict__ hits,
                                                       const int* __restrict__ count_dev, int count_terms,
                                                       int count_host, int cap, int* __restrict__ fetch,
                                                       int* __restrict__ gstack,
                                                       unsigned long long* __restrict__ counters) {
    __shared__ int lstack[kLdsStack * kTraceBlock];
    const int tid = threadIdx.x;
    const int lane = __lane_id();
    int n = count_host;
    if (count_dev) {
        n = 0;
        for (int k = 0; k < count_terms; ++k) n += count_dev[k];
        n = min(n, cap);
    }
    int* gst = gstack + (size_t)(blockIdx.x * kTraceBlock + tid) * kGlobalStack;
    unsigned long long nvis = 0, ntest = 0, mvis = 0, mtest = 0;
#define PUSH(v)                                                  \
    do {                                                         \
        ++sp;                                                    \
        if (sp < kLdsStack) lstack[sp * kTraceBlock + tid] = (v); \
        else gst[sp - kLdsStack] = (v);                          \
    } while (0)
#define POP() ((sp < kLdsStack) ? lstack[(sp--) * kTraceBlock + tid] : gst[(sp--) - kLdsStack])
    int stride_i = blockIdx.x * kTraceBlock + tid - gridDim.x * kTraceBlock;
    for (;;) {
        int i;
        if constexpr (PERSIST) {
            int base = 0;
            if (lane == 0) base = atomicAdd(fetch, 64);
            base = __shfl(base, 0, 64);
            if (base >= n) break;
            i = base + lane;
            if (i >= n) continue;  // tail of the last batch (whole wave then fetches past n and exits)
        } else {
            stride_i += gridDim.x * kTraceBlock;
            i = stride_i;
            if (i >= n) break;
        }
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
        float best_t = tfar, best_u = 0.0f, best_v = 0.0f;
        int best_prim = -1;
        unsigned rvis = 0, rtest = 0;
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
            while ((unsigned)node < (unsigned)kSentinel) {
                const BvhNode* nd = s.nodes + node;
                const float4 a = nd->a, b = nd->b, c = nd->c;
                const int4 d = nd->d;
                if (COUNT) ++rvis;
                float t0, t1;
                const bool h0 = box_hit(a.x, a.y, a.z, a.w, c.x, c.y, idx, idy, idz, oix, oiy, oiz, best_t, t0);
                const bool h1 = box_hit(b.x, b.y, b.z, b.w, c.z, c.w, idx, idy, idz, oix, oiy, oiz, best_t, t1);
                if (!h0 && !h1) {
                    node = POP();
                } else {
                    const bool first0 = h0 && (!h1 || t0 <= t1);
                    node = first0 ? d.x : d.y;
                    if (h0 && h1) PUSH(first0 ? d.y : d.x);
                }
                if (node < 0 && leaf == 0) {  // first leaf: park it and keep descending
                    leaf = node;
                    node = POP();
                }
                if constexpr (WW) {
                    if (!__any(leaf == 0)) break;
                } else {
                    break;
                }
            }
            // ---- triangle tests for the parked leaves ----
            while (leaf < 0) {
                const int first = leaf_first(leaf), cnt = leaf_count(leaf);
                for (int k = first; k < first + cnt; ++k) {
                    if (COUNT) ++rtest;
                    const float4 q0 = s.tri[3 * k], q1 = s.tri[3 * k + 1], q2 = s.tri[3 * k + 2];
                    // e1 = v0 - v1, e2 = v2 - v0 (precomputed), Ng = e2 x e1
                    const float e1x = q1.x, e1y = q1.y, e1z = q1.z;
                    const float e2x = q2.x, e2y = q2.y, e2z = q2.z;
                    const float ngx = e2y * e1z - e2z * e1y;
                    const float ngy = e2z * e1x - e2x * e1z;
                    const float ngz = e2x * e1y - e2y * e1x;
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
                leaf = 0;
                if (node < 0) {  // the node popped after parking is a leaf too: test it now
                    leaf = node;
                    node = POP();
                }
            }
        }
        hits[i] = make_float4(best_t, best_u, best_v, __int_as_float(best_prim));
        if (COUNT) {
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
    }
}

void launch_trace(const SceneView& s, const float4* ro, const float4* rd, float4* hits, const int* count_dev,
                  int count_host, int max_count, int* fetch, int* gstack, int gstack_threads,
                  unsigned long long* counters, bool count, hipStream_t stream, int expect, int count_terms) {
    if (max_count <= 0) return;
    // schedule A/B switch (PGRT_TRACE_VARIANT = bit0 persistent fetch | bit1 while-while).
    // Measured on the C2 frame (r1, profiles/r1/trace_variants.txt): 2 = grid-stride +
    // while-while is fastest (1.31 ms vs 1.64-2.10 ms for the others), so it is the default.
    static const int variant = [] {
        const char* e = getenv("PGRT_TRACE_VARIANT");
        return e ? atoi(e) : 2;
    }();
    const bool persist = variant & 1, ww = variant & 2;
    // size the grid to the expected count; persistent waves need no more than the machine
    // keeps resident; never more than the global overflow stacks cover
    int grid = ceil_div(expect > 0 && expect < max_count ? expect : max_count, kTraceBlock);
    if (persist && grid > kResidentBlocks) grid = kResidentBlocks;
    if (grid > gstack_threads / kTraceBlock) grid = gstack_threads / kTraceBlock;
#define PGRT_LAUNCH(C, P, W)                                                                               \
    hipLaunchKernelGGL((k_trace<C, P, W>), dim3(grid), dim3(kTraceBlock), 0, stream, s, ro, rd, hits, count_dev, \
                       count_terms, count_host, max_count, fetch, gstack, counters)
    if (count) {
        if (persist) { if (ww) PGRT_LAUNCH(true, true, true); else PGRT_LAUNCH(true, true, false); }
        else { if (ww) PGRT_LAUNCH(true, false, true); else PGRT_LAUNCH(true, false, false); }
    } else {
        if (persist) { if (ww) PGRT_LAUNCH(false, true, true); else PGRT_LAUNCH(false, true, false); }
        else { if (ww) PGRT_LAUNCH(false, false, true); else PGRT_LAUNCH(false, false, false); }
    }
#undef PGRT_LAUNCH
}

int trace_block_size() { return kTraceBlock; }

}  // namespace pgrt
