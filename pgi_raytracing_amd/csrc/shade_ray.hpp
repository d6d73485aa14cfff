// shade_ray.hpp -- the per-ray Whitted shading step (APP/raytracer.cpp:237-394, one level of
// Raytracer::trace), in phases (k_shade, render.hip):
//   shade_eval_a  what the ray's hit produces and how many queue slots it needs (kind, dielectric
//                 children, shadow rays)
//   shade_alloc   queue slots for the children / shadow rays: ballot + mbcnt inside the wave, ONE
//                 packed 64-bit atomic (children | shadow rays << 32) per block and iteration --
//                 split in _begin / _end, and between them
//   shade_eval_b  the long-latency colours (environment / texture fetch, attenuation, R) while the
//                 atomic is in flight
//   shade_emit    writes the children, the shadow rays with their Phong terms and the node record
// (shade_eval = _a then _b, for the kernels that allocate no slots: subtree, path tracer)
// Float operation order is the reference's (see shade_ops.hpp), so results are bit-identical
// wherever the phases run.
#pragma once

#include "cache_ops.hpp"
#include "shade_ops.hpp"
#include "trace.hpp"

namespace pgrt {

// child order in the next level's queue: per block (256 parents), its reflections then its
// refractions (r2k A/B: per wave, or interleaved, was slower)

// shading tables in LDS when they fit (the hit -> attributes -> material -> texture chain has one
// global round trip fewer per hop)
constexpr int kLdsMats = 64, kLdsTex = 32;

// Wave-level slot allocation for small per-lane counts (children <= 2, shadow rays <= lights):
// the exclusive prefix is sum_b 2^b * (lanes below with bit b set), one ballot + mbcnt per bit.
// Every lane of the wave must be active.
__device__ __forceinline__ void wave_prefix_small(int x, int bits, int& prefix, int& total) {
    prefix = 0;
    total = 0;
    for (int b = 0; b < bits; ++b) {
        const unsigned long long m = __ballot((x >> b) & 1);
        const int below = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
        prefix += below << b;
        total += __popcll(m) << b;
    }
}

__device__ __forceinline__ int lanes_below(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

struct ShadeOut {
    int kind;  // 0 final colour, 1 dielectric (children), 2 opaque (shadow rays pending)
    int nchild, nshadow, mid;
    float4 color, att;
    V3 org, dirraw, nrm, hitp, refl_dir, refr_dir;
    float n1, n2;
    float m_d_r, m_d_g, m_d_b;
};

// the hit triangle's 16 shading floats (n0 n1 n2 uv0 uv1 uv2 material), fetched as 4 x 16 B and
// kept as plain floats (reading a float4 array through a float pointer is type punning: with
// TBAA the optimiser may order those float reads before the float4 stores that fill the array)
struct HitAttr {
    float f[16];
};
__device__ __forceinline__ HitAttr load_attr(const SceneView& s, float4 h) {
    HitAttr a;
    const int prim = __float_as_int(h.w);
    float4 q0 = make_float4(0, 0, 0, 0), q1 = q0, q2 = q0, q3 = q0;
    if (prim >= 0) {
        const float4* p = at_bytes(reinterpret_cast<const float4*>(s.attr), (unsigned)prim << 6);
        q0 = p[0];
        q1 = p[1];
        q2 = p[2];
        q3 = p[3];
    }
    const float4 q[4] = {q0, q1, q2, q3};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        a.f[4 * k] = q[k].x;
        a.f[4 * k + 1] = q[k].y;
        a.f[4 * k + 2] = q[k].z;
        a.f[4 * k + 3] = q[k].w;
    }
    return a;
}

__device__ __forceinline__ void shade_init(ShadeOut& r) {
    r.kind = 0;
    r.color = make_float4(0, 0, 0, 1);
    r.nshadow = 0;
    r.nchild = 0;
    r.org = r.dirraw = r.nrm = r.hitp = r.refl_dir = r.refr_dir = v3(0, 0, 0);
    r.n1 = r.n2 = 0;
    r.att = make_float4(0, 0, 0, 0);
    r.m_d_r = r.m_d_g = r.m_d_b = 0;
    r.mid = 0;
}

// Phase 1 in two parts around the block's slot allocation (k_shade): part A
// settles what the allocation needs -- the kind and the children / shadow-ray counts (hit,
// attributes, normal, material, reflection / refraction directions) -- and part B, run while the
// allocation atomic is in flight, the long-latency colours: a miss's environment texel, a textured
// hit's texel, a dielectric's attenuation and R.  Same functions, same float operations in the same
// order per value: bit-identical to shade_eval.
struct ShadeDefer {
    float t, tu, tv;  // hit distance (attenuation), texture coordinates (textured opaque hits)
};
__device__ __forceinline__ void shade_eval_a(const SceneView& s, const DevMaterial* mats, int level, int max_level,
                                             bool active, float4 o4, float4 d4, float rtime, float4 h, ShadeOut& r,
                                             ShadeDefer& df) {
    shade_init(r);
    df.t = df.tu = df.tv = 0.0f;
    if (!active) return;
    r.org = v3(o4.x, o4.y, o4.z);
    r.dirraw = v3(d4.x, d4.y, d4.z);
    if (d4.w < 0.0f) {
        r.color = make_float4(0, 0, 0, 0);  // padding slot
        return;
    }
    const int prim = __float_as_int(h.w);
    if (prim < 0) {
        r.kind = 3;  // a miss: its environment texel in part B (raytracer.cpp:390-393)
        return;
    }
    const V3 d = normalize(r.dirraw);
    const HitAttr ha = load_attr(s, h);
    const float* a = ha.f;
    const float t = h.x, u = h.y, v = h.z;
    V3 nn = v3(interp1(a[0], a[3], a[6], u, v), interp1(a[1], a[4], a[7], u, v), interp1(a[2], a[5], a[8], u, v));
    const int mid = __float_as_int(a[15]);
    const DevMaterial& m = mats[mid];
    nn = normalize(nn);
    const V3 hitp = r.org + scale(t, r.dirraw);
    float n1, n2;
    if (rtime == PGRT_IOR_AIR) {
        n1 = PGRT_IOR_AIR;
        n2 = m.ior;
    } else {
        n1 = m.ior;
        n2 = PGRT_IOR_AIR;
    }
    if (dot(nn, d) > 0) nn = -nn;
    r.mid = mid;
    r.hitp = hitp;
    r.n1 = n1;
    r.n2 = n2;
    r.nrm = nn;
    if (level >= max_level) return;  // r.color (0, 0, 0, 1): raytracer.cpp:282-283
    if (m.type == PGRT_MATERIAL_DIELECTRIC) {
        V3 refl, refr;
        {  // get_reflection_ray (raytracer.cpp:209-235)
            const V3 dd = normalize(d), rn = normalize(nn);
            refl = dd - scale(2, scale(dot(dd, rn), rn));
        }
        {  // get_refraction_ray (raytracer.cpp:178-207)
            const V3 dd = normalize(d), rn = normalize(nn);
            const float n1_n2 = n1 / n2;
            const float d_n = dot(dd, rn);
            const V3 sd = v3(dd.x * n1_n2, dd.y * n1_n2, dd.z * n1_n2);
            const float kk = n1_n2 * d_n + sqrtf(1 - ((n1_n2 * n1_n2) * (1 - (d_n * d_n))));
            refr = sd - scale(kk, rn);
        }
        r.kind = 1;
        r.nchild = refr.x == refr.x ? 2 : 1;  // 1: total internal reflection
        r.refl_dir = refl;
        r.refr_dir = refr;
        df.t = t;
    } else {
        if (m.tex >= 0) {
            df.tu = interp1(a[9], a[11], a[13], u, v);
            df.tv = interp1(a[10], a[12], a[14], u, v);
        }
        int nshadow = 0;
        for (int li = 0; li < s.nlight; ++li) {
            const DevLight& L = s.lights[li];
            if (!(dot(nn, v3(L.pos[0], L.pos[1], L.pos[2])) < 0)) ++nshadow;
        }
        r.kind = 2;
        r.nshadow = nshadow;
    }
}
__device__ __forceinline__ void shade_eval_b(const SceneView& s, const DevMaterial* mats, const float* lut,
                                             ShadeOut& r, const ShadeDefer& df) {
    if (r.kind == 3) {
        r.color = env_texel(s, lut, normalize(r.dirraw));
        r.kind = 0;
    } else if (r.kind == 1) {
        const DevMaterial& m = mats[r.mid];
        const float ax = pg_expf(-(1 - m.kd[0]) * df.t);  // raytracer.cpp:303-305
        const float ay = pg_expf(-(1 - m.kd[1]) * df.t);
        const float az = pg_expf(-(1 - m.kd[2]) * df.t);
        float R = 0.0f;
        if (r.nchild == 2) {
            const V3 d = normalize(r.dirraw);
            const float cos1 = fabsf(dot(r.nrm, -d));
            const float alpha = (r.n1 - r.n2) / (r.n1 + r.n2);
            R = (float)((double)(alpha * alpha + (1 - (alpha * alpha))) * pg_pow_d((double)(1 - cos1), 5.0));
        }
        r.att = make_float4(ax, ay, az, R);
    } else if (r.kind == 2) {
        const DevMaterial& m = mats[r.mid];
        if (m.tex < 0) {
            r.m_d_r = m.kd[2];
            r.m_d_g = m.kd[1];
            r.m_d_b = m.kd[0];
        } else {
            const V3 tx = tex_texel(s.tex[m.tex], s.texels, lut, df.tu, 1.0f - df.tv);
            r.m_d_r = tx.x;
            r.m_d_g = tx.y;
            r.m_d_b = tx.z;
        }
    }
}

// Phase 1 for one ray (o4 = org|tnear, d4 = dir|tfar, rtime = medium IOR, h = t|u|v|prim): both
// parts back to back (the subtree and path kernels, which allocate no queue slots)
__device__ __forceinline__ void shade_eval(const SceneView& s, const DevMaterial* mats, const float* lut,
                                           int level, int max_level, bool active, float4 o4, float4 d4,
                                           float rtime, float4 h, ShadeOut& r) {
    ShadeDefer df;
    shade_eval_a(s, mats, level, max_level, active, o4, d4, rtime, h, r, df);
    shade_eval_b(s, mats, lut, r, df);
}

// LDS of the block-level allocation (BLOCK threads)
template <int BLOCK>
struct ShadeAllocLds {
    unsigned long long wtot[2][BLOCK / 64];
    int wrefl[2][BLOCK / 64];  // reflection children per wave
    int wrefr[2][BLOCK / 64];  // refraction children per wave (statistics)
    unsigned long long bbase;
};

struct ShadeSlots {
    int refl, refr, shadow;
};

// Phase 2: every thread of the block calls it in the same iteration (uniform control flow; it
// has two barriers).  it_par alternates per iteration.  shade_alloc_begin claims the block's
// slots (thread 0's atomic is in flight when it returns), shade_alloc_end hands them out: work
// placed between the two overlaps the atomic's round trip.
struct ShadeAllocPending {
    int spre;
    unsigned long long mrefl, mrefr;
    unsigned long long base;  // thread 0: the atomic's result
};
// The block's children (low word) and shadow rays (high word) are counted on fc->alloc[level]
// (one packed atomic).
// refr_acc: thread 0's running count of refraction children (statistics, fc->refract), flushed by
// the caller once per launch (shade_refract_flush); nullptr: one atomic per block and iteration.
// (A same-address atomic per WAVE, as before r3, serialised ~27k atomics on one word for an
// 8-frame C2 level 1.)
template <int BLOCK>
__device__ __forceinline__ ShadeAllocPending shade_alloc_begin(ShadeAllocLds<BLOCK>& lds, int it_par, FrameCounters* fc,
                                                               int level, int sbits, const ShadeOut& r,
                                                               int* refr_acc = nullptr) {
    ShadeAllocPending pa;
    int cpre, ctot, stot;
    wave_prefix_small(r.nchild, 2, cpre, ctot);
    wave_prefix_small(r.nshadow, sbits, pa.spre, stot);
    (void)cpre;
    const int rtot = (int)__popcll(__ballot(r.nchild == 2));
    const unsigned long long wtot = ((unsigned long long)(unsigned)stot << 32) | (unsigned)ctot;
    const int w = threadIdx.x >> 6;
    pa.mrefl = __ballot(r.nchild >= 1);
    pa.mrefr = __ballot(r.nchild == 2);
    if (__lane_id() == 0) {
        lds.wtot[it_par][w] = wtot;
        lds.wrefl[it_par][w] = (int)__popcll(pa.mrefl);
        lds.wrefr[it_par][w] = rtot;
    }
    __syncthreads();
    pa.base = 0;
    if (threadIdx.x == 0) {
        unsigned long long btot = 0;
        int brefr = 0;
        for (int k = 0; k < BLOCK / 64; ++k) {
            btot += lds.wtot[it_par][k];
            brefr += lds.wrefr[it_par][k];
        }
        if (refr_acc) *refr_acc += brefr;
        else if (brefr && level + 1 < kMaxLevels) atomicAdd(&fc->refract[level + 1], brefr);  // statistics
        pa.base = btot ? atomicAdd(&fc->alloc[level], btot) : 0ull;
    }
    return pa;
}
template <int BLOCK>
__device__ __forceinline__ ShadeSlots shade_alloc_end(ShadeAllocLds<BLOCK>& lds, int& it_par, int sq_base,
                                                      const ShadeAllocPending& pa) {
    if (threadIdx.x == 0) lds.bbase = pa.base;
    __syncthreads();
    const int w = threadIdx.x >> 6;
    unsigned long long old = lds.bbase;
    for (int k = 0; k < w; ++k) old += lds.wtot[it_par][k];
    int refl_below = 0, refl_block = 0;  // reflections of the block's waves below this one / all
    for (int k = 0; k < BLOCK / 64; ++k) {
        const int c = lds.wrefl[it_par][k];
        refl_block += c;
        if (k < w) refl_below += c;
    }
    it_par ^= 1;
    const int cb = __builtin_amdgcn_readfirstlane((int)(unsigned)(old & 0xffffffffull));
    const int sb = __builtin_amdgcn_readfirstlane((int)(unsigned)(old >> 32));
    ShadeSlots o;
    // the BLOCK's reflection rays first, then its refraction rays, each group in pixel order: a
    // reflection leaves the surface and a refraction enters it, so a next-level wave that mixes
    // the two spans > 90 degrees and its packet traversal visits the union of both paths
    const int bb = __builtin_amdgcn_readfirstlane((int)(unsigned)(lds.bbase & 0xffffffffull));
    const int rb = __builtin_amdgcn_readfirstlane(refl_below), rk = __builtin_amdgcn_readfirstlane(refl_block);
    o.refl = bb + rb + lanes_below(pa.mrefl);
    o.refr = bb + rk + (cb - bb - rb) + lanes_below(pa.mrefr);
    o.shadow = sq_base + sb + pa.spre;
    return o;
}
template <int BLOCK>
__device__ __forceinline__ ShadeSlots shade_alloc(ShadeAllocLds<BLOCK>& lds, int& it_par, FrameCounters* fc, int level,
                                                  int sq_base, int sbits, const ShadeOut& r, int* refr_acc = nullptr) {
    return shade_alloc_end(lds, it_par, sq_base,
                           shade_alloc_begin(lds, it_par, fc, level, sbits, r, refr_acc));
}
// thread 0 at the end of a launch: its block's refraction children into fc->refract[level + 1]
__device__ __forceinline__ void shade_refract_flush(FrameCounters* fc, int level, int refr_acc) {
    if (threadIdx.x == 0 && refr_acc && level + 1 < kMaxLevels) atomicAdd(&fc->refract[level + 1], refr_acc);
}

// Phong term of a lit hit for one light (raytracer.cpp:355-382): (blue, green, red, 0)
__device__ __forceinline__ float4 phong_term(const DevMaterial& m, const DevLight& L, const ShadeOut& r) {
    const V3 nrm = r.nrm, hitp = r.hitp, org = r.org, dirraw = r.dirraw;
    const V3 lp = v3(L.pos[0], L.pos[1], L.pos[2]);
    const V3 lv = normalize(v3(lp.x - hitp.x, lp.y - hitp.y, lp.z - hitp.z));
    const V3 cv = normalize(v3(org.x - dirraw.x, org.y - dirraw.y, org.z - dirraw.z));
    const float gam = m.ns;
    const float i_d_r = L.kd[2], i_d_g = L.kd[1], i_d_b = L.kd[0];
    const float i_s_r = L.ks[2], i_s_g = L.ks[1], i_s_b = L.ks[0];
    const float m_s_r = m.ks[2], m_s_g = m.ks[1], m_s_b = m.ks[0];
    const float nl = dot(nrm, lv);
    V3 l_r = scale(2 * nl, nrm) - lv;
    l_r = normalize(l_r);
    const float spec = pg_powf(dot(cv, l_r), gam);
    const float tb = i_d_b * r.m_d_b * dot(nrm, lv) + i_s_b * m_s_b * spec;
    const float tg = i_d_g * r.m_d_g * dot(nrm, lv) + i_s_g * m_s_g * spec;
    const float tr = i_d_r * r.m_d_r * dot(nrm, lv) + i_s_r * m_s_r * spec;
    return make_float4(tb, tg, tr, 0.0f);
}

// the children of a dielectric hit (raytracer.cpp:306-316): reflection (medium n1), refraction
// (medium n2); origin the hit point, tnear 0.01, tfar FLT_MAX
__device__ __forceinline__ float4 child_org(const ShadeOut& r) { return make_float4(r.hitp.x, r.hitp.y, r.hitp.z, 0.01f); }
__device__ __forceinline__ float4 child_dir(V3 d) { return make_float4(d.x, d.y, d.z, 3.402823466e+38f); }

// Phase 3a: a dielectric hit's children into the next level's queue; returns the node link
// (refl, refr or -1); -1, -1 when a queue was full (overflow: the frame is re-rendered)
__device__ __forceinline__ int4 emit_children(int level, const ShadeOut& r, const ShadeSlots& sl, Queue next,
                                              FrameCounters* fc) {
    int4 link = make_int4(-1, -1, -1, 0);
    if ((r.nchild == 2 ? max(sl.refl, sl.refr) : sl.refl) >= next.cap || level + 1 >= kMaxLevels) {
        atomicOr(&fc->overflow, 1);
        return link;
    }
    st_stream(next.ro + sl.refl, child_org(r));
    st_stream(next.rd + sl.refl, child_dir(r.refl_dir));
    st_stream_nt(next.time + sl.refl, r.n1);
    link.x = sl.refl;
    if (r.nchild == 2) {
        st_stream(next.ro + sl.refr, child_org(r));
        st_stream(next.rd + sl.refr, child_dir(r.refr_dir));
        st_stream_nt(next.time + sl.refr, r.n2);
        link.y = sl.refr;
    }
    return link;
}

// Phase 3b for an active ray i: the node record (attenuation of a dielectric; an opaque hit's
// shadow rays with their Phong terms; a final colour).  link: emit_children's result for a
// dielectric.  use_pre0: light 0's Phong term is pre0 (computed earlier by the caller).
// owner >= 0: the node's pixel, carried in the shadow rays' Phong terms (contrib.w; ShadowFinal)
__device__ __forceinline__ void emit_node(const SceneView& s, const DevMaterial* mats, int i, const ShadeOut& r,
                                          const ShadeSlots& sl, int4 link, LevelNodes nodes, ShadowQueue sq,
                                          FrameCounters* fc, bool use_pre0 = false,
                                          float4 pre0 = make_float4(0, 0, 0, 0), int owner = -1) {
    if (r.kind == 1) {
        st_stream(nodes.att + i, r.att);
    } else if (r.kind == 2 && r.nshadow > 0) {
        if (sl.shadow + r.nshadow > sq.cap) {
            atomicOr(&fc->overflow, 1);
        } else {
            const DevMaterial& m = mats[r.mid];
            const V3 nrm = r.nrm, hitp = r.hitp;
            int k = sl.shadow;
            for (int li = 0; li < s.nlight; ++li) {
                const DevLight& L = s.lights[li];
                const V3 lp = v3(L.pos[0], L.pos[1], L.pos[2]);
                if (dot(nrm, lp) < 0) continue;  // is_illuminated's N.L test (raytracer.cpp:155)
                // LightSource::GenerateRay(hit): org = light, dir = hit position vector
                if (sq.ro) st_stream(sq.ro + k, make_float4(lp.x, lp.y, lp.z, 0.01f));
                st_stream(sq.rd + k,
                          make_float4(hitp.x, hitp.y, hitp.z, length(v3(lp.x - hitp.x, lp.y - hitp.y, lp.z - hitp.z))));
                // Phong term for this light (raytracer.cpp:355-382)
                float4 c = (use_pre0 && li == 0) ? pre0 : phong_term(m, L, r);
                if (owner >= 0) c.w = __int_as_float(owner);
                st_stream(sq.contrib + k, c);
                ++k;
            }
            if (owner < 0) {  // (owner >= 0: the shadow trace writes the colour, k_combine skips the node)
                link.z = sl.shadow;
                link.w = r.nshadow;
            }
        }
    }
    st_stream(nodes.link + i, link);
    if (link.x < 0 && link.z < 0 && owner < 0) st_stream(nodes.color + i, r.color);  // else derived later
}

// Phase 3 for an active ray i.
__device__ __forceinline__ void shade_emit(const SceneView& s, const DevMaterial* mats, int level, int i,
                                           const ShadeOut& r, const ShadeSlots& sl, Queue next, LevelNodes nodes,
                                           ShadowQueue sq, FrameCounters* fc, bool use_pre0 = false,
                                           float4 pre0 = make_float4(0, 0, 0, 0), int owner = -1) {
    const int4 link = r.kind == 1 ? emit_children(level, r, sl, next, fc) : make_int4(-1, -1, -1, 0);
    emit_node(s, mats, i, r, sl, link, nodes, sq, fc, use_pre0, pre0, owner);
}

}  // namespace pgrt
