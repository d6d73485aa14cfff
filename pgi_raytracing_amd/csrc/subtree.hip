// subtree.hip -- the deep Whitted levels as ONE launch: every ray of level L_t evaluates its whole
// ray tree depth first, the way the reference's recursive Raytracer::trace does
// (APP/raytracer.cpp:237-394: trace the ray, shade the hit, recurse into the reflection and then
// the refraction child, mix_srgb the two and attenuate, :294-323; an opaque hit's shadow rays,
// is_illuminated :150-176, and Phong sum, :325-385; a miss samples the environment, :390-393).
//
// Why: below a few hundred thousand rays a level of the wavefront pipeline takes as long as its
// slowest ray (tens of node fetches in a dependent chain), so the deep levels' launches cost the
// SUM over levels of each level's slowest ray, plus a trace, a shade and a combine launch per
// level.  Here a group of G lanes owns one level-L_t ray and walks its subtree with an explicit
// stack in LDS (one frame per pending dielectric node: attenuation / R, the reflection's colour,
// the refraction ray), tracing every ray of the subtree -- reflection, refraction and shadow rays
// -- with trace8_group (8 / 4 lanes per ray over the 8-wide BVH).  The launch takes as long as
// the longest SUBTREE, and levels L_t.. need no queues, no node records, no combine.
//
// Bit-exactness: the hit is order-independent (closest hit, ties to the smaller triangle index),
// the shading is shade_eval / phong_term (the same functions k_shade runs), the shadow verdict is
// is_illuminated's (no hit, or a dielectric occluder), the lit Phong terms are summed in light
// order from 0 (opaque_color), and a dielectric node's colour is node_color's mix_srgb + attenuate
// -- so the level-L_t colours written here are the ones the per-level launches + k_combine give.
#include "cache_ops.hpp"
#include "shade_ops.hpp"
#include "shade_ray.hpp"
#include "stamps.hpp"
#include "trace.hpp"
#include "traverse.hpp"

namespace pgrt {

constexpr int kSubtreeBlock = 256;

// per-block statistics of the subtree levels (the counters k_shade keeps per level: children
// | shadow rays << 32 on alloc[L], refractions on refract[L + 1]), flushed once per block
struct SubtreeStats {
    unsigned long long alloc[kMaxLevels];
    int refract[kMaxLevels];
    unsigned long long trav_vis, trav_test, shadow_vis, shadow_test, hits, textured;
};

// one pending dielectric node of a group's subtree (frame j <-> the node of level L_t + j)
struct SubFrameRef {
    float4* att;   // (att.r, att.g, att.b, R)
    float4* refl;  // the reflection child's colour, once known
    float4* org;   // the children's origin (hit point, tnear 0.01)
    float4* rdir;  // the refraction direction, medium n2 in w
    int* info;     // nchild | phase << 4 (phase 1: the refraction child is being evaluated)
};

template <int G, bool LDS_TABLES, bool COUNT>
__global__ __launch_bounds__(kSubtreeBlock) void k_subtree(SceneView s, FrameParams fp, int level, Queue q,
                                                           LevelNodes nodes, FrameCounters* fc, int frames) {
    PGRT_STAMP_BEGIN(s.stamps);
    constexpr int kGroups = kSubtreeBlock / G;
    __shared__ uint2 gstk[kGroupStack][kGroups];
    __shared__ float lut255[256];
    __shared__ DevMaterial smat[LDS_TABLES ? kLdsMats : 1];
    __shared__ DevTexture stex[LDS_TABLES ? kLdsTex : 1];
    __shared__ SubtreeStats bst;
    extern __shared__ float4 fstore[];  // frames: att, refl, org, rdir [frames][kGroups] each, then info
    if constexpr (LDS_TABLES) {
        for (int k = threadIdx.x; k < s.nmat; k += kSubtreeBlock) smat[k] = s.mats[k];
        for (int k = threadIdx.x; k < s.ntex; k += kSubtreeBlock) stex[k] = s.tex[k];
        s.tex = stex;  // env_texel / tex_texel read descriptors through s.tex
    }
    for (int k = threadIdx.x; k < kMaxLevels; k += kSubtreeBlock) {
        bst.alloc[k] = 0;
        bst.refract[k] = 0;
    }
    if (threadIdx.x == 0) bst.trav_vis = bst.trav_test = bst.shadow_vis = bst.shadow_test = bst.hits = bst.textured = 0;
    const DevMaterial* mats = LDS_TABLES ? smat : s.mats;
    fill_byte_lut(lut255);  // ends with __syncthreads: the tables above are visible too
    const int tid = threadIdx.x;
    const int k = tid & (G - 1);  // lane within the group
    const int gib = tid / G;      // group within the block
    const int gshift = __lane_id() & ~(G - 1);
    const int fs = frames * kGroups;
    SubFrameRef F{fstore + gib, fstore + fs + gib, fstore + 2 * fs + gib, fstore + 3 * fs + gib,
                  reinterpret_cast<int*>(fstore + 4 * fs) + gib};
    const int n = min(fc_count(*fc, level), q.cap);
    const float4 no_hit_h = make_float4(0.0f, 0.0f, 0.0f, __int_as_float(-1));
    (void)no_hit_h;
    for (int i = blockIdx.x * kGroups + gib; i < n; i += gridDim.x * kGroups) {
        float4 o4 = ld_stream(q.ro + i), d4 = ld_stream(q.rd + i);
        float rtime = ld_stream_nt(q.time + i);
        int sp = 0;  // pending dielectric frames; the ray being evaluated is of level `level + sp`
        float4 val = make_float4(0, 0, 0, 1);
        for (;;) {
            // ---- evaluate one ray: its closest hit, then trace()'s body for it ----
            const int L = level + sp;
            float bt = d4.w, bu = 0.0f, bv = 0.0f;
            int bp = -1;
            unsigned rvis = 0, rtest = 0;
            trace8_group<G, COUNT>(s, o4, d4, k, gshift, &gstk[0][gib], kGroups, bt, bu, bv, bp, rvis, rtest);
            ShadeOut r;
            shade_eval(s, mats, lut255, L, fp.max_level, true, o4, d4, rtime, make_float4(bt, bu, bv, __int_as_float(bp)),
                       r);
            if (COUNT && k == 0) {
                atomicAdd(&bst.trav_vis, (unsigned long long)rvis);
                atomicAdd(&bst.trav_test, (unsigned long long)rtest);
                if (bp >= 0) {
                    atomicAdd(&bst.hits, 1ull);
                    if (r.kind == 2 && mats[r.mid].tex >= 0) atomicAdd(&bst.textured, 1ull);
                }
            }
            if (r.kind == 1) {  // dielectric: a frame for the node, then its reflection child
                if (k == 0) {
                    atomicAdd(&bst.alloc[L], (unsigned long long)r.nchild);
                    if (r.nchild == 2 && L + 1 < kMaxLevels) atomicAdd(&bst.refract[L + 1], 1);
                }
                const int fi = sp * kGroups;
                F.att[fi] = r.att;
                F.org[fi] = child_org(r);
                F.rdir[fi] = make_float4(r.refr_dir.x, r.refr_dir.y, r.refr_dir.z, r.n2);
                F.info[fi] = r.nchild;
                ++sp;
                o4 = child_org(r);
                d4 = child_dir(r.refl_dir);
                rtime = r.n1;
                continue;
            }
            if (r.kind == 2 && r.nshadow > 0) {  // opaque: is_illuminated per light, the lit Phong terms
                if (k == 0) atomicAdd(&bst.alloc[L], (unsigned long long)r.nshadow << 32);
                const DevMaterial& m = mats[r.mid];
                float blue = 0, green = 0, red = 0;
                for (int li = 0; li < s.nlight; ++li) {
                    const DevLight& Lt = s.lights[li];
                    const V3 lp = v3(Lt.pos[0], Lt.pos[1], Lt.pos[2]);
                    if (dot(r.nrm, lp) < 0) continue;  // raytracer.cpp:155
                    // LightSource::GenerateRay(hit): org = the light, dir = the hit position vector
                    const float4 so = make_float4(lp.x, lp.y, lp.z, 0.01f);
                    const float4 sd = make_float4(r.hitp.x, r.hitp.y, r.hitp.z,
                                                  length(v3(lp.x - r.hitp.x, lp.y - r.hitp.y, lp.z - r.hitp.z)));
                    float st = sd.w, su = 0.0f, sv = 0.0f;
                    int sprim = -1;
                    unsigned svis = 0, stest = 0;
                    trace8_group<G, COUNT>(s, so, sd, k, gshift, &gstk[0][gib], kGroups, st, su, sv, sprim, svis,
                                           stest);
                    if (COUNT && k == 0) {
                        atomicAdd(&bst.shadow_vis, (unsigned long long)svis);
                        atomicAdd(&bst.shadow_test, (unsigned long long)stest);
                    }
                    if (sprim < 0 || s.prim_glass[sprim] != 0) {  // raytracer.cpp:163-173
                        const float4 c = phong_term(m, Lt, r);
                        blue += c.x;
                        green += c.y;
                        red += c.z;
                    }
                }
                val = make_float4(blue, green, red, 1.0f);
            } else {
                val = r.color;  // a miss (environment), a hit at max_level, an opaque hit with no lit candidate
            }
            // ---- return up the stack: settle every frame whose children are done ----
            bool descend = false;
            while (sp > 0) {
                const int fi = (sp - 1) * kGroups;
                const int info = F.info[fi];
                const float4 att = F.att[fi];
                float4 c;
                if ((info >> 4) == 0) {  // the reflection child returned
                    if ((info & 15) == 2) {  // now the refraction child (raytracer.cpp:308-310)
                        F.refl[fi] = val;
                        F.info[fi] = info | (1 << 4);
                        o4 = F.org[fi];
                        const float4 rd4 = F.rdir[fi];
                        d4 = make_float4(rd4.x, rd4.y, rd4.z, 3.402823466e+38f);
                        rtime = rd4.w;
                        descend = true;
                        break;
                    }
                    c = val;  // total internal reflection (raytracer.cpp:321)
                } else {
                    c = mix_srgb(F.refl[fi], val, att.w);  // raytracer.cpp:318-319
                }
                val = make_float4(c.x * att.x, c.y * att.y, c.z * att.z, 1);
                --sp;
            }
            if (!descend) break;
        }
        if (k == 0) {  // the level-L_t node is final: k_combine(L_t - 1) reads its colour
            st_stream(nodes.color + i, val);
            st_stream(nodes.link + i, make_int4(-1, -1, -1, 0));
        }
    }
    __syncthreads();
    for (int L = tid; L < kMaxLevels; L += kSubtreeBlock) {
        if (bst.alloc[L]) atomicAdd(&fc->alloc[L], bst.alloc[L]);
        if (bst.refract[L]) atomicAdd(&fc->refract[L], bst.refract[L]);
    }
    if (COUNT && tid == 0) {
        atomicAdd(&fc->trav[level][14], bst.trav_vis);  // 80-B wide-node visits
        atomicAdd(&fc->trav[level][1], bst.trav_test);
        atomicAdd(&fc->trav[kMaxLevels][14], bst.shadow_vis);
        atomicAdd(&fc->trav[kMaxLevels][1], bst.shadow_test);
        atomicAdd(&fc->shade[level][0], bst.hits);
        atomicAdd(&fc->shade[level][1], bst.textured);
    }
    PGRT_STAMP_END(s.stamps);
}

// ---- work-sharing form (subtrees of at most kWsMaxDepth levels below the launch level) ----
//
// In k_subtree a group walks its ray's whole tree alone, so a launch lasts as long as the largest
// tree: one synchronous C2 frame's level-3 launch had a slowest wave of 158 us against a median of
// 41 (profiles/r5/r5a/timeline_r5a.txt), the frame's critical path.  Here the pending dielectric
// nodes of a block's trees live in LDS, heap-numbered per tree (node p's children are positions
// 2p + 1 and 2p + 2), and a node's REFRACTION child is published as a task that any idle group of
// the block takes, while the group that hit the dielectric continues with the reflection child.
// A child that settles stores its colour in its parent's node and decrements the node's pending
// count; whoever settles the last child combines the node (mix_srgb + attenuation, exactly
// node_color's) and settles it in turn, up to the tree's root, whose colour is the level-L_t node
// colour k_combine reads.  The combine's inputs and order are the same whichever group ran a child,
// so the colours are bit-identical to k_subtree's and to the per-level launches.
//   Progress: no group ever waits for another -- a group with nothing to do re-polls the task bits
// (s_sleep between polls) until every group of the block has run out of home rays and no tree is
// in progress -- so the divergent groups of one wave cannot deadlock each other.
constexpr int kWsMaxDepth = 3;  // max_level - launch level: <= 7 node positions per tree

struct WsNode {       // one pending dielectric node (96 B)
    float4 att;       // (att.r, att.g, att.b, R)
    float4 refl, refr;  // the children's colours, once settled
    float4 org;       // the children's origin (hit point, tnear 0.01)
    float4 rdir;      // the refraction direction, medium n2 in w
    int pending;      // children not yet settled
    int nchild;       // 2, or 1 at total internal reflection
    int pad[2];
};

__device__ __forceinline__ int lds_load(const int* p) { return __atomic_load_n(p, __ATOMIC_RELAXED); }
__device__ __forceinline__ unsigned lds_load(const unsigned* p) { return __atomic_load_n(p, __ATOMIC_RELAXED); }

// claim one published task bit (lane 0 of a group), scanning from a per-group start word; -1: none
__device__ __forceinline__ int ws_take_task(unsigned* bits, int words, int start) {
    for (int w = 0; w < words; ++w) {
        const int idx = (start + w) % words;
        unsigned m = lds_load(bits + idx);
        while (m) {
            const int b = __ffs((int)m) - 1;
            const unsigned old = atomicAnd(bits + idx, ~(1u << b));
            if (old & (1u << b)) return idx * 32 + b;
            m = old & ~(1u << b);
        }
    }
    return -1;
}

template <int G, bool LDS_TABLES, bool COUNT>
__global__ __launch_bounds__(kSubtreeBlock) void k_subtree_ws(SceneView s, FrameParams fp, int level, Queue q,
                                                              LevelNodes nodes, FrameCounters* fc, int npr) {
    PGRT_STAMP_BEGIN(s.stamps);
    constexpr int kGroups = kSubtreeBlock / G;
    constexpr int kTaskWords = (kGroups * ((1 << kWsMaxDepth) - 1) + 31) / 32;
    __shared__ uint2 gstk[kGroupStack][kGroups];
    __shared__ float lut255[256];
    __shared__ DevMaterial smat[LDS_TABLES ? kLdsMats : 1];
    __shared__ DevTexture stex[LDS_TABLES ? kLdsTex : 1];
    __shared__ SubtreeStats bst;
    __shared__ unsigned task_bits[kTaskWords];
    __shared__ int home_root[kGroups];  // the queue index of each group's current home ray
    __shared__ int home_busy[kGroups];  // 1 while that ray's tree is unsettled
    __shared__ int live_trees, exhausted;
    extern __shared__ WsNode wsn[];     // [kGroups][npr]
    if constexpr (LDS_TABLES) {
        for (int k = threadIdx.x; k < s.nmat; k += kSubtreeBlock) smat[k] = s.mats[k];
        for (int k = threadIdx.x; k < s.ntex; k += kSubtreeBlock) stex[k] = s.tex[k];
        s.tex = stex;
    }
    for (int k = threadIdx.x; k < kMaxLevels; k += kSubtreeBlock) {
        bst.alloc[k] = 0;
        bst.refract[k] = 0;
    }
    for (int k = threadIdx.x; k < kTaskWords; k += kSubtreeBlock) task_bits[k] = 0u;
    for (int k = threadIdx.x; k < kGroups; k += kSubtreeBlock) home_busy[k] = 0;
    if (threadIdx.x == 0) {
        bst.trav_vis = bst.trav_test = bst.shadow_vis = bst.shadow_test = bst.hits = bst.textured = 0;
        live_trees = 0;
        exhausted = 0;
    }
    const DevMaterial* mats = LDS_TABLES ? smat : s.mats;
    fill_byte_lut(lut255);  // ends with __syncthreads: the tables and the task state are visible too
    const int tid = threadIdx.x;
    const int k = tid & (G - 1);
    const int gib = tid / G;
    const int gshift = __lane_id() & ~(G - 1);
    const int n = min(fc_count(*fc, level), q.cap);
    const int stride = gridDim.x * kGroups;
    const int words = (kGroups * npr + 31) / 32;
    int next_home = blockIdx.x * kGroups + gib;
    bool have = false, out_of_rays = false;
    float4 o4 = make_float4(0, 0, 0, 0), d4 = make_float4(0, 0, 0, -1.0f);
    float rtime = 0.0f;
    int L = level, h = 0, tg = gib;
    unsigned idle_polls = 0;
    for (;;) {
        if (!have) {
            // (a) a published refraction child of any tree of the block
            int t = k == 0 ? ws_take_task(task_bits, words, (gib * words) / kGroups) : -1;
            t = __shfl(t, gshift);
            if (t >= 0) {
                tg = t / npr;
                const int p = t - tg * npr;
                const WsNode& nd = wsn[t];
                o4 = nd.org;
                const float4 rd4 = nd.rdir;
                d4 = make_float4(rd4.x, rd4.y, rd4.z, 3.402823466e+38f);
                rtime = rd4.w;
                h = 2 * p + 2;
                L = level + (31 - __clz(h + 1));
                have = true;
            } else if (!out_of_rays && lds_load(&home_busy[gib]) == 0) {
                // (b) the group's next home ray, once its previous tree is settled
                if (next_home < n) {
                    o4 = ld_stream(q.ro + next_home);
                    d4 = ld_stream(q.rd + next_home);
                    rtime = ld_stream_nt(q.time + next_home);
                    tg = gib;
                    h = 0;
                    L = level;
                    have = true;
                    if (k == 0) {
                        home_root[gib] = next_home;
                        home_busy[gib] = 1;
                        atomicAdd(&live_trees, 1);
                    }
                    next_home += stride;
                } else {
                    out_of_rays = true;
                    if (k == 0) atomicAdd(&exhausted, 1);
                }
            }
        }
        // Only a WHOLE idle wave polls / sleeps / leaves (a wave-uniform branch): were the idle
        // groups' polling a divergent path, the compiler may turn it into an inner loop that runs
        // with the busy groups of the same wave masked off -- and a busy group can be the very one
        // whose refraction task or root an idle group waits for (measured: a deadlock, r5g)
        if (__ballot(have) == 0ull) {
            if (lds_load(&exhausted) == kGroups && lds_load(&live_trees) == 0) break;
            // safety net: the block's trees settle within microseconds of the last ray; a wave
            // still polling after ~2^22 sleeps (> 0.1 s) reports it and leaves (the frame fails
            // loudly instead of hanging the GPU)
            if (++idle_polls > (1u << 22)) {
                if (k == 0) atomicOr(&fc->watchdog, 1);
#ifdef PGRT_WS_DEBUG
                if (k == 0 && blockIdx.x < 2)
                    printf("ws watchdog blk %d grp %d out %d busy %d live %d exh %d n %d next %d bits %08x %08x\n",
                           blockIdx.x, gib, (int)out_of_rays, home_busy[gib], live_trees, exhausted, n, next_home,
                           task_bits[0], task_bits[1 % kTaskWords]);
#endif
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        if (!have) continue;  // this group idles while others of its wave work (no inner loop)
        // ---- one ray: its closest hit, then trace()'s body for it ----
        float bt = d4.w, bu = 0.0f, bv = 0.0f;
        int bp = -1;
        unsigned rvis = 0, rtest = 0;
        trace8_group<G, COUNT>(s, o4, d4, k, gshift, &gstk[0][gib], kGroups, bt, bu, bv, bp, rvis, rtest);
        ShadeOut r;
        shade_eval(s, mats, lut255, L, fp.max_level, true, o4, d4, rtime, make_float4(bt, bu, bv, __int_as_float(bp)), r);
        if (COUNT && k == 0) {
            atomicAdd(&bst.trav_vis, (unsigned long long)rvis);
            atomicAdd(&bst.trav_test, (unsigned long long)rtest);
            if (bp >= 0) {
                atomicAdd(&bst.hits, 1ull);
                if (r.kind == 2 && mats[r.mid].tex >= 0) atomicAdd(&bst.textured, 1ull);
            }
        }
        if (r.kind == 1) {  // dielectric (level < max_level, so h < npr): its node, the refraction task
            const int ni = tg * npr + h;
            if (k == 0) {
                atomicAdd(&bst.alloc[L], (unsigned long long)r.nchild);
                if (r.nchild == 2 && L + 1 < kMaxLevels) atomicAdd(&bst.refract[L + 1], 1);
                WsNode& nd = wsn[ni];
                nd.att = r.att;
                nd.org = child_org(r);
                nd.rdir = make_float4(r.refr_dir.x, r.refr_dir.y, r.refr_dir.z, r.n2);
                nd.pending = r.nchild;
                nd.nchild = r.nchild;
                __threadfence_block();  // the node before its task bit
                if (r.nchild == 2) atomicOr(&task_bits[ni >> 5], 1u << (ni & 31));
            }
            o4 = child_org(r);  // this group continues with the reflection child
            d4 = child_dir(r.refl_dir);
            rtime = r.n1;
            h = 2 * h + 1;
            ++L;
            continue;
        }
        float4 val;
        if (r.kind == 2 && r.nshadow > 0) {  // opaque: is_illuminated per light, the lit Phong terms
            if (k == 0) atomicAdd(&bst.alloc[L], (unsigned long long)r.nshadow << 32);
            const DevMaterial& m = mats[r.mid];
            float blue = 0, green = 0, red = 0;
            for (int li = 0; li < s.nlight; ++li) {
                const DevLight& Lt = s.lights[li];
                const V3 lp = v3(Lt.pos[0], Lt.pos[1], Lt.pos[2]);
                if (dot(r.nrm, lp) < 0) continue;  // raytracer.cpp:155
                const float4 so = make_float4(lp.x, lp.y, lp.z, 0.01f);
                const float4 sd = make_float4(r.hitp.x, r.hitp.y, r.hitp.z,
                                              length(v3(lp.x - r.hitp.x, lp.y - r.hitp.y, lp.z - r.hitp.z)));
                float st = sd.w, su = 0.0f, sv = 0.0f;
                int sprim = -1;
                unsigned svis = 0, stest = 0;
                trace8_group<G, COUNT>(s, so, sd, k, gshift, &gstk[0][gib], kGroups, st, su, sv, sprim, svis, stest);
                if (COUNT && k == 0) {
                    atomicAdd(&bst.shadow_vis, (unsigned long long)svis);
                    atomicAdd(&bst.shadow_test, (unsigned long long)stest);
                }
                if (sprim < 0 || s.prim_glass[sprim] != 0) {  // raytracer.cpp:163-173
                    const float4 c = phong_term(m, Lt, r);
                    blue += c.x;
                    green += c.y;
                    red += c.z;
                }
            }
            val = make_float4(blue, green, red, 1.0f);
        } else {
            val = r.color;
        }
        // ---- settle up the tree: the last child of a node combines it ----
        for (;;) {
            if (h == 0) {  // the tree's root: the level-L_t node colour
                if (k == 0) {
                    const int i = home_root[tg];
                    st_stream(nodes.color + i, val);
                    st_stream(nodes.link + i, make_int4(-1, -1, -1, 0));
                    home_busy[tg] = 0;
                    atomicSub(&live_trees, 1);
                }
                break;
            }
            const int p = (h - 1) >> 1;
            WsNode& nd = wsn[tg * npr + p];
            int old = 0;
            if (k == 0) {
                if (h & 1) nd.refl = val;  // odd positions are reflection children
                else nd.refr = val;
                __threadfence_block();  // the colour before the count
                old = atomicSub(&nd.pending, 1);
            }
            old = __shfl(old, gshift);
            if (old != 1) break;  // the sibling is still running: it settles the node
            __threadfence_block();
            const float4 att = nd.att;
            // raytracer.cpp:318-319 (refraction present) or :321 (total internal reflection)
            const float4 c = nd.nchild == 2 ? mix_srgb(nd.refl, nd.refr, att.w) : nd.refl;
            val = make_float4(c.x * att.x, c.y * att.y, c.z * att.z, 1);
            h = p;
        }
        have = false;
    }
    __syncthreads();
    for (int LL = tid; LL < kMaxLevels; LL += kSubtreeBlock) {
        if (bst.alloc[LL]) atomicAdd(&fc->alloc[LL], bst.alloc[LL]);
        if (bst.refract[LL]) atomicAdd(&fc->refract[LL], bst.refract[LL]);
    }
    if (COUNT && tid == 0) {
        atomicAdd(&fc->trav[level][14], bst.trav_vis);
        atomicAdd(&fc->trav[level][1], bst.trav_test);
        atomicAdd(&fc->trav[kMaxLevels][14], bst.shadow_vis);
        atomicAdd(&fc->trav[kMaxLevels][1], bst.shadow_test);
        atomicAdd(&fc->shade[level][0], bst.hits);
        atomicAdd(&fc->shade[level][1], bst.textured);
    }
    PGRT_STAMP_END(s.stamps);
}

bool subtree_available(const SceneView& s) { return s.depth8 + 1 <= kGroupStack; }

void launch_subtree(const SceneView& s_in, const FrameParams& fp, int level, Queue q, LevelNodes nodes,
                    FrameCounters* fc, int max_count, int expect, bool count, hipStream_t stream) {
    if (max_count <= 0) return;
    const int ex = expect > 0 && expect < max_count ? expect : max_count;
    const bool g4 = ex > kSubtreeGroup8Max;
    const int groups = kSubtreeBlock / (g4 ? 4 : 8);
    const int grid = std::max(1, std::min(16384, ceil_div(ex, groups)));
    const int frames = std::max(1, fp.max_level - level);
    const size_t lds = (size_t)frames * groups * (4 * sizeof(float4) + sizeof(int));
    SceneView s = s_in;
    s.stamps = stamp_next(kStampSubtree, level, grid, kSubtreeBlock);
    const bool tables = s.nmat <= kLdsMats && s.ntex <= kLdsTex;
    if (frames <= kWsMaxDepth) {  // shallow trees: the work-sharing form
        const int npr = (1 << frames) - 1;
        const size_t wlds = (size_t)groups * npr * sizeof(WsNode);
#define PGRT_LAUNCH_WS(G, T, C)                                                                                     \
    hipLaunchKernelGGL((k_subtree_ws<G, T, C>), dim3(grid), dim3(kSubtreeBlock), wlds, stream, s, fp, level, q, nodes, \
                       fc, npr)
        if (count) {
            if (g4) { if (tables) PGRT_LAUNCH_WS(4, true, true); else PGRT_LAUNCH_WS(4, false, true); }
            else { if (tables) PGRT_LAUNCH_WS(8, true, true); else PGRT_LAUNCH_WS(8, false, true); }
        } else {
            if (g4) { if (tables) PGRT_LAUNCH_WS(4, true, false); else PGRT_LAUNCH_WS(4, false, false); }
            else { if (tables) PGRT_LAUNCH_WS(8, true, false); else PGRT_LAUNCH_WS(8, false, false); }
        }
#undef PGRT_LAUNCH_WS
        return;
    }
#define PGRT_LAUNCH_SUB(G, T, C)                                                                                       \
    hipLaunchKernelGGL((k_subtree<G, T, C>), dim3(grid), dim3(kSubtreeBlock), lds, stream, s, fp, level, q, nodes, fc, \
                       frames)
    if (count) {
        if (g4) { if (tables) PGRT_LAUNCH_SUB(4, true, true); else PGRT_LAUNCH_SUB(4, false, true); }
        else { if (tables) PGRT_LAUNCH_SUB(8, true, true); else PGRT_LAUNCH_SUB(8, false, true); }
    } else {
        if (g4) { if (tables) PGRT_LAUNCH_SUB(4, true, false); else PGRT_LAUNCH_SUB(4, false, false); }
        else { if (tables) PGRT_LAUNCH_SUB(8, true, false); else PGRT_LAUNCH_SUB(8, false, false); }
    }
#undef PGRT_LAUNCH_SUB
}

}  // namespace pgrt
