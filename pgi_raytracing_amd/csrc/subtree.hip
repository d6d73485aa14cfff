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

template <int G, bool LDS_TABLES, bool COUNT>
#ifndef PGRT_SUBTREE_WAVES
#define PGRT_SUBTREE_WAVES 1
#endif
__global__ __launch_bounds__(kSubtreeBlock, PGRT_SUBTREE_WAVES) void k_subtree(SceneView s, FrameParams fp, int level, Queue q,
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
