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

#if PGRT_STEP_PROFILE
// diagnostics build only: one record per evaluated ray tree (tools/step_profile.py)
constexpr int kStepRecs = 1 << 18;
constexpr int kStepWords = 12;
__device__ unsigned long long g_step_rec[kStepRecs][kStepWords];
__device__ unsigned g_step_count;
#endif

#ifndef PGRT_SUBTREE_SPREAD
#define PGRT_SUBTREE_SPREAD 0
#endif

template <int G, bool LDS_TABLES, bool COUNT>
#ifndef PGRT_SUBTREE_WAVES
#define PGRT_SUBTREE_WAVES 1
#endif
__global__ __launch_bounds__(kSubtreeBlock, PGRT_SUBTREE_WAVES) void k_subtree(SceneView s, FrameParams fp, int level, Queue q,
                                                           LevelNodes nodes, FrameCounters* fc, int frames) {
    PGRT_STAMP_BEGIN(s.stamps);
    chain_priority();
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
    // PGRT_SUBTREE_SPREAD: tree i -> group i / grid of block i % grid, so the trees of a wave lie grid
    // apart in the queue instead of adjacent (neighbouring pixels' trees are alike: a cluster of heavy
    // trees no longer lands in one wave, whose groups run one after another where they diverge)
    const int first = PGRT_SUBTREE_SPREAD ? gib * (int)gridDim.x + (int)blockIdx.x : (int)blockIdx.x * kGroups + gib;
    for (int i = first; i < n; i += gridDim.x * kGroups) {
        float4 o4 = ld_stream(q.ro + i), d4 = ld_stream(q.rd + i);
        float rtime = ld_stream_nt(q.time + i);
        int sp = 0;  // pending dielectric frames; the ray being evaluated is of level `level + sp`
        float4 val = make_float4(0, 0, 0, 1);
        StepProf prof{};
        StepProf* pp = nullptr;
        (void)prof;
#if PGRT_STEP_PROFILE
        pp = &prof;
        const long long tw0 = wall_clock64(), tc0 = clock64();
        unsigned long long shade_cyc = 0;
        unsigned ntrace = 0, maxsp = 0;
#endif
        for (;;) {
            // ---- evaluate one ray: its closest hit, then trace()'s body for it ----
            const int L = level + sp;
            float bt = d4.w, bu = 0.0f, bv = 0.0f;
            int bp = -1;
            unsigned rvis = 0, rtest = 0;
            trace8_group<G, COUNT>(s, o4, d4, k, gshift, &gstk[0][gib], kGroups, bt, bu, bv, bp, rvis, rtest, pp);
            ShadeOut r;
#if PGRT_STEP_PROFILE
            ++ntrace;
            maxsp = max(maxsp, (unsigned)sp);
            const long long sc0 = clock64();
#endif
            shade_eval(s, mats, lut255, L, fp.max_level, true, o4, d4, rtime, make_float4(bt, bu, bv, __int_as_float(bp)),
                       r);
#if PGRT_STEP_PROFILE
            asm volatile("" ::"v"(r.kind), "v"(r.color.x));
            shade_cyc += (unsigned long long)(clock64() - sc0);
#endif
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
                                           stest, pp);
#if PGRT_STEP_PROFILE
                    ++ntrace;
#endif
                    if (COUNT && k == 0) {
                        atomicAdd(&bst.shadow_vis, (unsigned long long)svis);
                        atomicAdd(&bst.shadow_test, (unsigned long long)stest);
                    }
                    if (sprim < 0 || *at_bytes(s.prim_glass, (unsigned)sprim) != 0) {  // raytracer.cpp:163-173
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
#if PGRT_STEP_PROFILE
        if (k == 0) {
            const long long tc1 = clock64(), tw1 = wall_clock64();
            const unsigned slot = atomicAdd(&g_step_count, 1u);
            if (slot < (unsigned)kStepRecs) {
                unsigned long long* rec = g_step_rec[slot];
                const unsigned wave = (blockIdx.x * kSubtreeBlock + tid) >> 6;
                rec[0] = (unsigned long long)tw0;
                rec[1] = (unsigned long long)tw1;
                rec[2] = (unsigned long long)(tc1 - tc0);
                rec[3] = prof.node_cyc;
                rec[4] = prof.node_wait;
                rec[5] = prof.tri_cyc;
                rec[6] = prof.tri_wait;
                rec[7] = shade_cyc;
                rec[8] = (unsigned long long)prof.nodes | ((unsigned long long)prof.tris << 32);
                rec[9] = (unsigned long long)ntrace | ((unsigned long long)maxsp << 16) | ((unsigned long long)level << 24) |
                         ((unsigned long long)G << 32) | ((unsigned long long)(gib % (64 / G)) << 40);
                rec[10] = (unsigned long long)wave | ((unsigned long long)(unsigned)i << 32);
                rec[11] = (unsigned long long)(size_t)q.ro;
            }
        }
#endif
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

// ---- cooperative ray trees ---------------------------------------------------------------------
// k_subtree evaluates each tree in ONE lane group, so a launch lasts as long as its largest tree: a
// canopy pixel's tree is 11-13 traces in series (r5zh, profiles/r6/r6c: the slowest wave's eight
// trees hold 5-13 traces each).  Here the groups of a block share their trees.  A dielectric node's
// refraction child becomes a task that any idle group of the block takes, while the group that met
// the node goes on with the reflection child; an idle group takes a waiting task first and starts a
// new root only when none waits.  A node's frame sits at its heap position in its tree's slot
// (children of heap index h at 2h+1 = reflection, 2h+2 = refraction), and the two children join on
// an LDS counter: the group that delivers a frame's last child mixes and attenuates
// (raytracer.cpp:318-321) and carries the colour on up.  Every node's arithmetic is the one k_subtree
// runs (shade_eval, is_illuminated's shadow rays, mix_srgb, attenuation), so the colours are
// bit-identical; only which group evaluates which ray, and when, changes.  Trees with at most
// kCoopMaxDepth levels below the first (2^D - 1 frames per tree slot, one slot per group).
//
// Lock-free: a waiting task is a bit of an LDS mask (claimed by atomicAnd), a tree slot a bit of
// another (claimed the same way), roots are claimed by atomicAdd, and s_busy counts the groups that
// hold a ray.  No group ever waits for another: an idle group retries once per iteration, and a
// wave leaves when all its groups are idle, no group of the block holds a ray (only a busy group can
// make a task), no task waits and no root is left.
#ifndef PGRT_COOP_WATCHDOG
#define PGRT_COOP_WATCHDOG 0
#endif
// PGRT_COOP_UNIFIED: one trace call site for the reflection / refraction rays and the shadow rays
#ifndef PGRT_COOP_UNIFIED
#define PGRT_COOP_UNIFIED 1
#endif
constexpr int kCoopMaxDepth = 4;
constexpr int kCoopTaskWords = 16;  // task bits: tree slots x frames <= 1024
constexpr int kCoopFrameBytes = 5 * (int)sizeof(float4) + 2 * (int)sizeof(int);  // att c0 c1 org rdir | cnt nch

template <int G, bool LDS_TABLES, bool COUNT>
__global__ __launch_bounds__(kSubtreeBlock, PGRT_SUBTREE_WAVES) void k_subtree_coop(SceneView s, FrameParams fp, int level,
                                                                                Queue q, LevelNodes nodes,
                                                                                FrameCounters* fc, int depth) {
    PGRT_STAMP_BEGIN(s.stamps);
    constexpr int kGroups = kSubtreeBlock / G;
    static_assert(kGroups <= 64, "tree slots are the bits of one 64-bit mask");
    __shared__ uint2 gstk[kGroupStack][kGroups];
    __shared__ float lut255[256];
    __shared__ DevMaterial smat[LDS_TABLES ? kLdsMats : 1];
    __shared__ DevTexture stex[LDS_TABLES ? kLdsTex : 1];
    __shared__ SubtreeStats bst;
    __shared__ int root_i[kGroups];                        // queue index of the root ray of tree slot t
    __shared__ unsigned long long s_task[kCoopTaskWords];  // frame fi's refraction child waits: bit fi
    __shared__ unsigned long long s_free;                  // free tree slots
    __shared__ int s_root_next, s_busy, s_tasks;
#if PGRT_COOP_UNIFIED
    // an opaque hit whose shadow rays are being traced: what phong_term needs (per group)
    __shared__ float4 g_nrm[kGroups], g_hitp[kGroups], g_org[kGroups], g_dir[kGroups], g_md[kGroups];
#endif
    extern __shared__ float4 cstore[];
    const int NF = (1 << depth) - 1;  // frames per tree: the dielectric nodes of levels level .. level + depth - 1
    const int nfr = kGroups * NF;
    const int ntw = (nfr + 63) >> 6;
    float4* f_att = cstore;            // (att.r, att.g, att.b, R)
    float4* f_c0 = cstore + nfr;       // the reflection child's colour
    float4* f_c1 = cstore + 2 * nfr;   // the refraction child's colour
    float4* f_org = cstore + 3 * nfr;  // the children's origin (hit point, tnear 0.01)
    float4* f_rdir = cstore + 4 * nfr; // the refraction direction, medium n2 in w
    int* f_cnt = reinterpret_cast<int*>(cstore + 5 * nfr);  // children delivered
    int* f_nch = f_cnt + nfr;                              // children (1: total internal reflection)
    const int tid = threadIdx.x;
    if constexpr (LDS_TABLES) {
        for (int k = tid; k < s.nmat; k += kSubtreeBlock) smat[k] = s.mats[k];
        for (int k = tid; k < s.ntex; k += kSubtreeBlock) stex[k] = s.tex[k];
        s.tex = stex;
    }
    for (int k = tid; k < kMaxLevels; k += kSubtreeBlock) {
        bst.alloc[k] = 0;
        bst.refract[k] = 0;
    }
    for (int k = tid; k < kCoopTaskWords; k += kSubtreeBlock) s_task[k] = 0ull;
    if (tid == 0) {
        bst.trav_vis = bst.trav_test = bst.shadow_vis = bst.shadow_test = bst.hits = bst.textured = 0;
        s_root_next = s_busy = s_tasks = 0;
        s_free = kGroups == 64 ? ~0ull : ((1ull << kGroups) - 1ull);
    }
    const DevMaterial* mats = LDS_TABLES ? smat : s.mats;
    fill_byte_lut(lut255);  // ends with __syncthreads
    const int k = tid & (G - 1);
    const int gib = tid / G;
    const int gshift = __lane_id() & ~(G - 1);
    const bool lead = k == 0;
    const int n = min(fc_count(*fc, level), q.cap);
    // the block's roots: the grid-stride sequence k_subtree's groups take (increasing in r)
    auto root_index = [&](int r) { return blockIdx.x * kGroups + (r % kGroups) + (r / kGroups) * gridDim.x * kGroups; };
    // claim one set bit of *m (a task or a free slot): -1 when none is left
    auto claim = [](unsigned long long* m) {
        unsigned long long v = *m;
        while (v != 0ull) {
            const unsigned long long bit = v & (~v + 1ull);
            const unsigned long long old = atomicAnd(m, ~bit);
            if (old & bit) return __ffsll((long long)bit) - 1;
            v = old & ~bit;
        }
        return -1;
    };
    bool have = false;
    int t = 0, h = 0, L = level;
    float4 o4 = make_float4(0, 0, 0, 0), d4 = o4;
    float rtime = 0.0f;
#if PGRT_COOP_UNIFIED
    int sh = -1;                                  // the light whose shadow ray is traced next (-1: o4 / d4's ray)
    float acc_b = 0.0f, acc_g = 0.0f, acc_r = 0.0f;  // the opaque hit's lit Phong terms so far, in light order
    // the first light at or after li that passes is_illuminated's N.L test (raytracer.cpp:155), or -1
    auto next_light = [&](int li, float4 nrm4) {
        for (; li < s.nlight; ++li) {
            const DevLight& Lt = s.lights[li];
            if (!(dot(v3(nrm4.x, nrm4.y, nrm4.z), v3(Lt.pos[0], Lt.pos[1], Lt.pos[2])) < 0)) return li;
        }
        return -1;
    };
#endif
#if PGRT_COOP_WATCHDOG
    unsigned iters = 0;
#endif
    for (;;) {
#if PGRT_COOP_WATCHDOG
        if (++iters > (1u << 20)) {  // diagnostics: a wave that never finishes reports its block's state
            if (__lane_id() == 0)
                printf("coop watchdog: block %d wave %d level %d n %d tasks %d busy %d root_next %d next_root_index %d "
                       "free %llx have %llx\n",
                       (int)blockIdx.x, (int)(tid >> 6), level, n, s_tasks, s_busy, s_root_next,
                       root_index(s_root_next), s_free, (unsigned long long)__ballot(lead && have));
            atomicOr(&fc->overflow, 8);
            break;
        }
#endif
        // ---- an idle group takes a waiting refraction child, else starts a root in a free slot ----
        if (!have) {
            int got = -1, got_root = -1, got_slot = -1;
            if (lead) {
                if (atomicAdd(&s_tasks, 0) > 0)
                    for (int w = 0; w < ntw && got < 0; ++w) {
                        const int b = claim(&s_task[w]);
                        if (b >= 0) got = (w << 6) + b;
                    }
                if (got >= 0) {
                    atomicSub(&s_tasks, 1);
                } else if (root_index(atomicAdd(&s_root_next, 0)) < n) {
                    got_slot = claim(&s_free);
                    if (got_slot >= 0) {
                        const int idx = root_index(atomicAdd(&s_root_next, 1));
                        if (idx < n) {
                            got_root = idx;
                            root_i[got_slot] = idx;
                        } else {  // the roots ran out meanwhile: the slot goes back
                            atomicOr(&s_free, 1ull << got_slot);
                            got_slot = -1;
                        }
                    }
                }
                if (got >= 0 || got_root >= 0) atomicAdd(&s_busy, 1);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            }
            got = __shfl(got, gshift, 64);
            got_root = __shfl(got_root, gshift, 64);
            got_slot = __shfl(got_slot, gshift, 64);
            if (got >= 0) {  // a refraction child: frame got holds its origin, direction and medium
                t = got / NF;
                const int p = got - t * NF;
                o4 = f_org[got];
                const float4 rd4 = f_rdir[got];
                d4 = make_float4(rd4.x, rd4.y, rd4.z, 3.402823466e+38f);
                rtime = rd4.w;
                h = 2 * p + 2;
                L = level + (31 - __clz(h + 1));
                have = true;
            } else if (got_root >= 0) {
                t = got_slot;
                h = 0;
                L = level;
                o4 = ld_stream(q.ro + got_root);
                d4 = ld_stream(q.rd + got_root);
                rtime = ld_stream_nt(q.time + got_root);
                have = true;
            }
        }
        if (__ballot(have) == 0ull) {  // the whole wave is idle: done, or wait for work
            int quit = 0;
            if (__lane_id() == 0)  // busy first: with no group holding a ray no task can appear later
                quit = atomicAdd(&s_busy, 0) == 0 && atomicAdd(&s_tasks, 0) == 0 &&
                       root_index(atomicAdd(&s_root_next, 0)) >= n;
            if (__shfl(quit, 0, 64)) break;
            __builtin_amdgcn_s_sleep(4);
            continue;
        }
        if (!have) continue;
#if PGRT_COOP_WATCHDOG
        if (lead && !(d4.x == d4.x && d4.y == d4.y && d4.z == d4.z && o4.x == o4.x && o4.y == o4.y && o4.z == o4.z))
            printf("coop watchdog: block %d group %d non-finite ray t %d h %d L %d o %f %f %f d %f %f %f %f\n",
                   (int)blockIdx.x, gib, t, h, L, o4.x, o4.y, o4.z, d4.x, d4.y, d4.z, d4.w);
#endif
#if PGRT_COOP_UNIFIED
        // ---- one ray -- o4 / d4's ray, or the next shadow ray of an opaque hit -- through ONE trace call
        // site, so groups of a wave in different phases of their trees still trace together ----
        float4 to4 = o4, td4 = d4;
        if (sh >= 0) {  // LightSource::GenerateRay(hit): from the light along the hit position vector
            const DevLight& Lt = s.lights[sh];
            const float4 hp = g_hitp[gib];
            to4 = make_float4(Lt.pos[0], Lt.pos[1], Lt.pos[2], 0.01f);
            td4 = make_float4(hp.x, hp.y, hp.z, length(v3(Lt.pos[0] - hp.x, Lt.pos[1] - hp.y, Lt.pos[2] - hp.z)));
        }
        float bt = td4.w, bu = 0.0f, bv = 0.0f;
        int bp = -1;
        unsigned rvis = 0, rtest = 0;
        trace8_group<G, COUNT>(s, to4, td4, k, gshift, &gstk[0][gib], kGroups, bt, bu, bv, bp, rvis, rtest);
        float4 val;
        if (sh >= 0) {  // a shadow ray: is_illuminated (raytracer.cpp:163-173), then the next light
            if (COUNT && lead) {
                atomicAdd(&bst.shadow_vis, (unsigned long long)rvis);
                atomicAdd(&bst.shadow_test, (unsigned long long)rtest);
            }
            const float4 nrm4 = g_nrm[gib];
            if (bp < 0 || *at_bytes(s.prim_glass, (unsigned)bp) != 0) {
                ShadeOut rr;
                const float4 hp = g_hitp[gib], og = g_org[gib], dr = g_dir[gib], md = g_md[gib];
                rr.nrm = v3(nrm4.x, nrm4.y, nrm4.z);
                rr.hitp = v3(hp.x, hp.y, hp.z);
                rr.org = v3(og.x, og.y, og.z);
                rr.dirraw = v3(dr.x, dr.y, dr.z);
                rr.m_d_r = md.x;
                rr.m_d_g = md.y;
                rr.m_d_b = md.z;
                const float4 c = phong_term(mats[__float_as_int(md.w)], s.lights[sh], rr);
                acc_b += c.x;
                acc_g += c.y;
                acc_r += c.z;
            }
            sh = next_light(sh + 1, nrm4);
            if (sh >= 0) continue;
            val = make_float4(acc_b, acc_g, acc_r, 1.0f);
        } else {
            ShadeOut r;
            shade_eval(s, mats, lut255, L, fp.max_level, true, o4, d4, rtime, make_float4(bt, bu, bv, __int_as_float(bp)),
                       r);
            if (COUNT && lead) {
                atomicAdd(&bst.trav_vis, (unsigned long long)rvis);
                atomicAdd(&bst.trav_test, (unsigned long long)rtest);
                if (bp >= 0) {
                    atomicAdd(&bst.hits, 1ull);
                    if (r.kind == 2 && mats[r.mid].tex >= 0) atomicAdd(&bst.textured, 1ull);
                }
            }
            if (r.kind == 1) {  // dielectric: the node's frame, the refraction child as a task, on with the reflection
                if (lead) {
                    atomicAdd(&bst.alloc[L], (unsigned long long)r.nchild);
                    if (r.nchild == 2 && L + 1 < kMaxLevels) atomicAdd(&bst.refract[L + 1], 1);
                }
                const int fi = t * NF + h;
                f_att[fi] = r.att;
                f_org[fi] = child_org(r);
                f_rdir[fi] = make_float4(r.refr_dir.x, r.refr_dir.y, r.refr_dir.z, r.n2);
                f_nch[fi] = r.nchild;
                f_cnt[fi] = 0;
                if (r.nchild == 2) {  // publish the refraction child once its frame is written
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    if (lead) {
                        atomicAdd(&s_tasks, 1);
                        atomicOr(&s_task[fi >> 6], 1ull << (fi & 63));
                    }
                }
                o4 = child_org(r);
                d4 = child_dir(r.refl_dir);
                rtime = r.n1;
                h = 2 * h + 1;
                ++L;
                continue;
            }
            if (r.kind == 2 && r.nshadow > 0) {  // opaque: its shadow rays next, one per iteration
                if (lead) atomicAdd(&bst.alloc[L], (unsigned long long)r.nshadow << 32);
                const float4 nrm4 = make_float4(r.nrm.x, r.nrm.y, r.nrm.z, 0.0f);
                g_nrm[gib] = nrm4;
                g_hitp[gib] = make_float4(r.hitp.x, r.hitp.y, r.hitp.z, 0.0f);
                g_org[gib] = make_float4(r.org.x, r.org.y, r.org.z, 0.0f);
                g_dir[gib] = make_float4(r.dirraw.x, r.dirraw.y, r.dirraw.z, 0.0f);
                g_md[gib] = make_float4(r.m_d_r, r.m_d_g, r.m_d_b, __int_as_float(r.mid));
                acc_b = acc_g = acc_r = 0.0f;
                sh = next_light(0, nrm4);  // nshadow > 0: a light passes
                continue;
            }
            val = r.color;  // a miss (environment), a hit at max_level, an opaque hit with no lit candidate
        }
#else
        // ---- one ray: trace and shade (raytracer.cpp:241-393) ----
        float bt = d4.w, bu = 0.0f, bv = 0.0f;
        int bp = -1;
        unsigned rvis = 0, rtest = 0;
        trace8_group<G, COUNT>(s, o4, d4, k, gshift, &gstk[0][gib], kGroups, bt, bu, bv, bp, rvis, rtest);
        ShadeOut r;
        shade_eval(s, mats, lut255, L, fp.max_level, true, o4, d4, rtime, make_float4(bt, bu, bv, __int_as_float(bp)), r);
        if (COUNT && lead) {
            atomicAdd(&bst.trav_vis, (unsigned long long)rvis);
            atomicAdd(&bst.trav_test, (unsigned long long)rtest);
            if (bp >= 0) {
                atomicAdd(&bst.hits, 1ull);
                if (r.kind == 2 && mats[r.mid].tex >= 0) atomicAdd(&bst.textured, 1ull);
            }
        }
        if (r.kind == 1) {  // dielectric: the node's frame, the refraction child as a task, on with the reflection
            if (lead) {
                atomicAdd(&bst.alloc[L], (unsigned long long)r.nchild);
                if (r.nchild == 2 && L + 1 < kMaxLevels) atomicAdd(&bst.refract[L + 1], 1);
            }
            const int fi = t * NF + h;
            f_att[fi] = r.att;
            f_org[fi] = child_org(r);
            f_rdir[fi] = make_float4(r.refr_dir.x, r.refr_dir.y, r.refr_dir.z, r.n2);
            f_nch[fi] = r.nchild;
            f_cnt[fi] = 0;
            if (r.nchild == 2) {  // publish the refraction child once its frame is written
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lead) {
                    atomicAdd(&s_tasks, 1);
                    atomicOr(&s_task[fi >> 6], 1ull << (fi & 63));
                }
            }
            o4 = child_org(r);
            d4 = child_dir(r.refl_dir);
            rtime = r.n1;
            h = 2 * h + 1;
            ++L;
            continue;
        }
        float4 val;
        if (r.kind == 2 && r.nshadow > 0) {  // opaque: is_illuminated per light, the lit Phong terms
            if (lead) atomicAdd(&bst.alloc[L], (unsigned long long)r.nshadow << 32);
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
                if (COUNT && lead) {
                    atomicAdd(&bst.shadow_vis, (unsigned long long)svis);
                    atomicAdd(&bst.shadow_test, (unsigned long long)stest);
                }
                if (sprim < 0 || *at_bytes(s.prim_glass, (unsigned)sprim) != 0) {  // raytracer.cpp:163-173
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
#endif
        // ---- deliver the colour up the tree: the last child of a frame settles it ----
        for (;;) {
            if (h == 0) {  // the root is final: k_combine(level - 1) reads its colour
                if (lead) {
                    const int i = root_i[t];
                    st_stream(nodes.color + i, val);
                    st_stream(nodes.link + i, make_int4(-1, -1, -1, 0));
                    atomicOr(&s_free, 1ull << t);
                    atomicSub(&s_busy, 1);
                }
                have = false;
                break;
            }
            const int p = (h - 1) >> 1;
            const int fi = t * NF + p;
            if (h & 1) f_c0[fi] = val;
            else f_c1[fi] = val;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            int old = 0;
            if (lead) old = atomicAdd(&f_cnt[fi], 1);
            old = __shfl(old, gshift, 64);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            if (old + 1 < f_nch[fi]) {  // the sibling is still being evaluated: it settles the frame
                if (lead) atomicSub(&s_busy, 1);
                have = false;
                break;
            }
            const float4 att = f_att[fi];
            const float4 c = f_nch[fi] == 2 ? mix_srgb(f_c0[fi], f_c1[fi], att.w) : f_c0[fi];  // raytracer.cpp:318-321
            val = make_float4(c.x * att.x, c.y * att.y, c.z * att.z, 1);
            h = p;
        }
    }
    __syncthreads();
    for (int l = tid; l < kMaxLevels; l += kSubtreeBlock) {
        if (bst.alloc[l]) atomicAdd(&fc->alloc[l], bst.alloc[l]);
        if (bst.refract[l]) atomicAdd(&fc->refract[l], bst.refract[l]);
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

#if PGRT_STEP_PROFILE
// diagnostics build only: copy out (and optionally reset) the per-tree step records
extern "C" int pgrt_diag_step_profile(unsigned long long* out, int max_records, int* n, int reset) {
    unsigned cnt = 0;
    if (hipMemcpyFromSymbol(&cnt, HIP_SYMBOL(g_step_count), sizeof(cnt)) != hipSuccess) return PGRT_ERR_HIP;
    const int m = (int)std::min<unsigned>(std::min<unsigned>(cnt, (unsigned)kStepRecs), (unsigned)std::max(0, max_records));
    if (out && m > 0 &&
        hipMemcpyFromSymbol(out, HIP_SYMBOL(g_step_rec), sizeof(unsigned long long) * kStepWords * m) != hipSuccess)
        return PGRT_ERR_HIP;
    if (n) *n = (int)cnt;
    if (reset) {
        cnt = 0;
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_step_count), &cnt, sizeof(cnt)) != hipSuccess) return PGRT_ERR_HIP;
    }
    return PGRT_OK;
}
#endif

bool subtree_available(const SceneView& s) { return s.depth8 + 1 <= kGroupStack; }

// PGRT_COOP_WATCHDOG (diagnostics): a coop wave past 2^20 loop iterations prints its block's state and stops
// PGRT_SUBTREE_COOP (A/B switch, compile time): 1 = the cooperative kernel where it applies
#ifndef PGRT_SUBTREE_COOP
#define PGRT_SUBTREE_COOP 0
#endif
constexpr size_t kCoopLdsBytes = 48 * 1024;
static bool subtree_coop_enabled() { return PGRT_SUBTREE_COOP != 0; }

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
    // cooperative trees: depth <= kCoopMaxDepth and their frames within kCoopLdsBytes
    const size_t coop_lds = (size_t)groups * ((1u << frames) - 1u) * kCoopFrameBytes;
    if (subtree_coop_enabled() && frames <= kCoopMaxDepth && coop_lds <= kCoopLdsBytes &&
        groups * ((1 << frames) - 1) <= 64 * kCoopTaskWords) {
#define PGRT_LAUNCH_COOP(G, T, C)                                                                                  \
    hipLaunchKernelGGL((k_subtree_coop<G, T, C>), dim3(grid), dim3(kSubtreeBlock), coop_lds, stream, s, fp, level, q, \
                       nodes, fc, frames)
        if (count) {
            if (g4) { if (tables) PGRT_LAUNCH_COOP(4, true, true); else PGRT_LAUNCH_COOP(4, false, true); }
            else { if (tables) PGRT_LAUNCH_COOP(8, true, true); else PGRT_LAUNCH_COOP(8, false, true); }
        } else {
            if (g4) { if (tables) PGRT_LAUNCH_COOP(4, true, false); else PGRT_LAUNCH_COOP(4, false, false); }
            else { if (tables) PGRT_LAUNCH_COOP(8, true, false); else PGRT_LAUNCH_COOP(8, false, false); }
        }
#undef PGRT_LAUNCH_COOP
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
