// shade_ray.hpp -- the per-ray Whitted shading step (APP/raytracer.cpp:237-394, one level of
// Raytracer::trace), in three phases (k_shade, render.hip):
//   shade_eval   what the ray's hit produces (final colour, dielectric children, shadow rays)
//   shade_alloc  queue slots for the children / shadow rays: ballot + mbcnt inside the wave, ONE
//                packed 64-bit atomic (children | shadow rays << 32) per block and iteration
//   shade_emit   writes the children, the shadow rays with their Phong terms and the node record
// Float operation order is the reference's (see shade_ops.hpp), so results are bit-identical
// wherever the phases run.
#pragma once

#include "shade_ops.hpp"
#include "trace.hpp"

namespace pgrt {

// child order in the next level's queue: 2 = per block (256 parents), its reflections then its
// refractions; 1 = the same per wave; 0 = interleaved
#ifndef PGRT_CHILD_SPLIT
#define PGRT_CHILD_SPLIT 2
#endif

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

// the hit triangle's 16 shading floats (n0 n1 n2 uv0 uv1 uv2 material), 4 x 16 B
struct HitAttr {
    float4 q[4];
};
__device__ __forceinline__ HitAttr load_attr(const SceneView& s, float4 h) {
    HitAttr a;
    const int prim = __float_as_int(h.w);
    if (prim >= 0) {
        const float4* p = reinterpret_cast<const float4*>(s.attr + 16 * (size_t)prim);
        a.q[0] = p[0];
        a.q[1] = p[1];
        a.q[2] = p[2];
        a.q[3] = p[3];
    } else {
        a.q[0] = a.q[1] = a.q[2] = a.q[3] = make_float4(0, 0, 0, 0);
    }
    return a;
}

// Phase 1 for one ray (o4 = org|tnear, d4 = dir|tfar, rtime = medium IOR, h = t|u|v|prim).
__device__ __forceinline__ void shade_eval(const SceneView& s, const DevMaterial* mats, const float* lut,
                                           int level, int max_level, bool active, float4 o4, float4 d4,
                                           float rtime, float4 h, ShadeOut& r) {
    r.kind = 0;
    r.color = make_float4(0, 0, 0, 1);
    r.nshadow = 0;
    r.nchild = 0;
    r.org = r.dirraw = r.nrm = r.hitp = r.refl_dir = r.refr_dir = v3(0, 0, 0);
    r.n1 = r.n2 = 0;
    r.att = make_float4(0, 0, 0, 0);
    r.m_d_r = r.m_d_g = r.m_d_b = 0;
    r.mid = 0;
    if (!active) return;
    r.org = v3(o4.x, o4.y, o4.z);
    r.dirraw = v3(d4.x, d4.y, d4.z);
    if (d4.w < 0.0f) {
        r.color = make_float4(0, 0, 0, 0);  // padding slot
        return;
    }
    const V3 d = normalize(r.dirraw);
    const int prim = __float_as_int(h.w);
    if (prim < 0) {
        r.color = env_texel(s, lut, d);  // miss (raytracer.cpp:390-393)
        return;
    }
    const float t = h.x;
    const HitAttr ha = load_attr(s, h);
    const float* a = reinterpret_cast<const float*>(ha.q);
    const float u = h.y, v = h.z;
    V3 nn = v3(interp1(a[0], a[3], a[6], u, v), interp1(a[1], a[4], a[7], u, v), interp1(a[2], a[5], a[8], u, v));
    r.mid = __float_as_int(a[15]);
    const DevMaterial& m = mats[r.mid];
    nn = normalize(nn);
    r.hitp = r.org + scale(t, r.dirraw);
    if (rtime == PGRT_IOR_AIR) {
        r.n1 = PGRT_IOR_AIR;
        r.n2 = m.ior;
    } else {
        r.n1 = m.ior;
        r.n2 = PGRT_IOR_AIR;
    }
    if (dot(nn, d) > 0) nn = -nn;
    r.nrm = nn;
    if (level >= max_level) {
        r.color = make_float4(0, 0, 0, 1);  // raytracer.cpp:282-283
    } else if (m.type == PGRT_MATERIAL_DIELECTRIC) {
        r.kind = 1;
        {  // get_reflection_ray (raytracer.cpp:209-235)
            const V3 dd = normalize(d), rn = normalize(nn);
            r.refl_dir = dd - scale(2, scale(dot(dd, rn), rn));
        }
        r.att.x = pg_expf(-(1 - m.kd[0]) * t);  // raytracer.cpp:303-305
        r.att.y = pg_expf(-(1 - m.kd[1]) * t);
        r.att.z = pg_expf(-(1 - m.kd[2]) * t);
        {  // get_refraction_ray (raytracer.cpp:178-207)
            const V3 dd = normalize(d), rn = normalize(nn);
            const float n1_n2 = r.n1 / r.n2;
            const float d_n = dot(dd, rn);
            const V3 sd = v3(dd.x * n1_n2, dd.y * n1_n2, dd.z * n1_n2);
            const float kk = n1_n2 * d_n + sqrtf(1 - ((n1_n2 * n1_n2) * (1 - (d_n * d_n))));
            r.refr_dir = sd - scale(kk, rn);
        }
        r.nchild = 1;
        if (r.refr_dir.x == r.refr_dir.x) {  // no total internal reflection
            r.nchild = 2;
            const float cos1 = fabsf(dot(nn, -d));
            const float alpha = (r.n1 - r.n2) / (r.n1 + r.n2);
            r.att.w = (float)((double)(alpha * alpha + (1 - (alpha * alpha))) * pg_pow_d((double)(1 - cos1), 5.0));
        }
    } else {
        r.kind = 2;
        if (m.tex < 0) {
            r.m_d_r = m.kd[2];
            r.m_d_g = m.kd[1];
            r.m_d_b = m.kd[0];
        } else {
            const float tu = interp1(a[9], a[11], a[13], u, v);
            const float tv = interp1(a[10], a[12], a[14], u, v);
            const V3 tx = tex_texel(s.tex[m.tex], s.texels, lut, tu, 1.0f - tv);
            r.m_d_r = tx.x;
            r.m_d_g = tx.y;
            r.m_d_b = tx.z;
        }
        for (int li = 0; li < s.nlight; ++li) {
            const DevLight& L = s.lights[li];
            if (!(dot(nn, v3(L.pos[0], L.pos[1], L.pos[2])) < 0)) ++r.nshadow;
        }
        r.color = make_float4(0, 0, 0, 1);
    }
}

// LDS of the block-level allocation (BLOCK threads)
template <int BLOCK>
struct ShadeAllocLds {
    unsigned long long wtot[2][BLOCK / 64];
    int wrefl[2][BLOCK / 64];  // reflection children per wave (PGRT_CHILD_SPLIT 2)
    unsigned long long bbase;
};

struct ShadeSlots {
    int refl, refr, shadow;
};

// Phase 2: every thread of the block calls it in the same iteration (uniform control flow; it
// has two barriers).  it_par alternates per iteration.
template <int BLOCK>
__device__ __forceinline__ ShadeSlots shade_alloc(ShadeAllocLds<BLOCK>& lds, int& it_par, FrameCounters* fc, int level,
                                                  int sq_base, int sbits, const ShadeOut& r) {
    int cpre, ctot, spre, stot;
    wave_prefix_small(r.nchild, 2, cpre, ctot);
    wave_prefix_small(r.nshadow, sbits, spre, stot);
    const int rtot = (int)__popcll(__ballot(r.nchild == 2));
    const unsigned long long wtot = ((unsigned long long)(unsigned)stot << 32) | (unsigned)ctot;
    const int w = threadIdx.x >> 6;
    const unsigned long long mrefl = __ballot(r.nchild >= 1), mrefr = __ballot(r.nchild == 2);
    if (__lane_id() == 0) {
        lds.wtot[it_par][w] = wtot;
#if PGRT_CHILD_SPLIT == 2
        lds.wrefl[it_par][w] = (int)__popcll(mrefl);
#endif
        if (rtot && level + 1 < kMaxLevels) atomicAdd(&fc->refract[level + 1], rtot);  // statistics
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long btot = 0;
        for (int k = 0; k < BLOCK / 64; ++k) btot += lds.wtot[it_par][k];
        lds.bbase = btot ? atomicAdd(&fc->alloc[level], btot) : 0ull;
    }
    __syncthreads();
    unsigned long long old = lds.bbase;
    for (int k = 0; k < w; ++k) old += lds.wtot[it_par][k];
#if PGRT_CHILD_SPLIT == 2
    int refl_below = 0, refl_block = 0;  // reflections of the block's waves below this one / all
    for (int k = 0; k < BLOCK / 64; ++k) {
        const int c = lds.wrefl[it_par][k];
        refl_block += c;
        if (k < w) refl_below += c;
    }
#endif
    it_par ^= 1;
    const int cb = __builtin_amdgcn_readfirstlane((int)(unsigned)(old & 0xffffffffull));
    const int sb = __builtin_amdgcn_readfirstlane((int)(unsigned)(old >> 32));
    ShadeSlots o;
#if PGRT_CHILD_SPLIT == 2
    // the BLOCK's reflection rays first, then its refraction rays, each group in pixel order: a
    // reflection leaves the surface and a refraction enters it, so a next-level wave that mixes
    // the two spans > 90 degrees and its packet traversal visits the union of both paths
    const int bb = __builtin_amdgcn_readfirstlane((int)(unsigned)(lds.bbase & 0xffffffffull));
    const int rb = __builtin_amdgcn_readfirstlane(refl_below), rk = __builtin_amdgcn_readfirstlane(refl_block);
    o.refl = bb + rb + lanes_below(mrefl);
    o.refr = bb + rk + (cb - bb - rb) + lanes_below(mrefr);
    (void)cpre;
#elif PGRT_CHILD_SPLIT
    // the wave's reflection rays first, then its refraction rays, each group in pixel order:
    // the next level's waves are coherent bundles instead of alternating reflect / refract
    o.refl = cb + lanes_below(mrefl);
    o.refr = cb + (int)__popcll(mrefl) + lanes_below(mrefr);
    (void)cpre;
#else
    o.refl = cb + cpre;
    o.refr = o.refl + 1;
#endif
    o.shadow = sq_base + sb + spre;
    return o;
}

// Phase 3 for an active ray i.
__device__ __forceinline__ void shade_emit(const SceneView& s, const DevMaterial* mats, int level, int i,
                                           const ShadeOut& r, const ShadeSlots& sl, Queue next, LevelNodes nodes,
                                           ShadowQueue sq, FrameCounters* fc) {
    int4 link = make_int4(-1, -1, -1, 0);
    if (r.kind == 1) {
        if ((r.nchild == 2 ? max(sl.refl, sl.refr) : sl.refl) >= next.cap || level + 1 >= kMaxLevels) {
            atomicOr(&fc->overflow, 1);
        } else {
            next.ro[sl.refl] = make_float4(r.hitp.x, r.hitp.y, r.hitp.z, 0.01f);
            next.rd[sl.refl] = make_float4(r.refl_dir.x, r.refl_dir.y, r.refl_dir.z, 3.402823466e+38f);
            next.time[sl.refl] = r.n1;
            if (next.key) next.key[sl.refl] = (unsigned char)dir_octant(r.refl_dir.x, r.refl_dir.y, r.refl_dir.z);
            link.x = sl.refl;
            if (r.nchild == 2) {
                next.ro[sl.refr] = make_float4(r.hitp.x, r.hitp.y, r.hitp.z, 0.01f);
                next.rd[sl.refr] = make_float4(r.refr_dir.x, r.refr_dir.y, r.refr_dir.z, 3.402823466e+38f);
                next.time[sl.refr] = r.n2;
                if (next.key) next.key[sl.refr] = (unsigned char)dir_octant(r.refr_dir.x, r.refr_dir.y, r.refr_dir.z);
                link.y = sl.refr;
            }
        }
        nodes.att[i] = r.att;
    } else if (r.kind == 2 && r.nshadow > 0) {
        if (sl.shadow + r.nshadow > sq.cap) {
            atomicOr(&fc->overflow, 1);
        } else {
            const DevMaterial& m = mats[r.mid];
            const V3 nrm = r.nrm, hitp = r.hitp, org = r.org, dirraw = r.dirraw;
            int k = sl.shadow;
            for (int li = 0; li < s.nlight; ++li) {
                const DevLight& L = s.lights[li];
                const V3 lp = v3(L.pos[0], L.pos[1], L.pos[2]);
                if (dot(nrm, lp) < 0) continue;  // is_illuminated's N.L test (raytracer.cpp:155)
                // LightSource::GenerateRay(hit): org = light, dir = hit position vector
                if (sq.ro) sq.ro[k] = make_float4(lp.x, lp.y, lp.z, 0.01f);
                sq.rd[k] = make_float4(hitp.x, hitp.y, hitp.z, length(v3(lp.x - hitp.x, lp.y - hitp.y, lp.z - hitp.z)));
                // Phong term for this light (raytracer.cpp:355-382)
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
                sq.contrib[k] = make_float4(tb, tg, tr, 0.0f);
                ++k;
            }
            link.z = sl.shadow;
            link.w = r.nshadow;
        }
    }
    nodes.link[i] = link;
    if (link.x < 0 && link.z < 0) nodes.color[i] = r.color;  // else derived by k_finish
}

}  // namespace pgrt
