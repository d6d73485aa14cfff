// render.hip -- wavefront Whitted pipeline kernels (ray generation, shading, shadow resolve,
// bottom-up combine of the non-linear mix_srgb tree, sample accumulation, resolve + gamma).
//
// Reference: Raytracer::get_pixel / trace (APP/raytracer.cpp:237-437), PinHoleCamera
// (APP/PinHoleCamera.cpp:31-105), LightSource::GenerateRay (APP/LightSource.cpp:11-32).
// The recursion of trace() becomes one ray queue per level: level L+1 holds the reflection /
// refraction children of the dielectric hits of level L, appended with one atomic per wave
// (__ballot-free prefix by __shfl_up, the wave's total claimed by its last lane).  Shadow rays
// of every level go to one batch-wide queue, traced once after the last level by the same
// closest-hit kernel.  Because mix_srgb is non-linear (it clamps and sRGB-encodes before the
// attenuation multiply, :318-321), colours are combined bottom-up, one level per launch,
// once every level is traced.
#include "shade_ops.hpp"
#include "trace.hpp"
#include "camera_ops.hpp"

namespace pgrt {

constexpr int kBlock = 256;

// grid of a grid-stride kernel: cover the expected count, at most 4096 workgroups
static int grid_for(int max_count, int expect) {
    const int n = (expect > 0 && expect < max_count) ? expect : max_count;
    const int g = ceil_div(n, kBlock);
    return g < 1 ? 1 : (g > 4096 ? 4096 : g);
}

// Wave-level slot allocation for small per-lane counts (children <= 2, shadow rays <= lights):
// the exclusive prefix is sum_b 2^b * (lanes below with bit b set), one ballot + mbcnt per bit,
// and lane 0 issues the queue atomics together (one round trip).  Every lane of the wave must
// be active (k_shade keeps whole waves in its loop).
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

// ------------------------------------------------------------------ ray generation

__global__ __launch_bounds__(kBlock) void k_raygen(CameraView cam, FrameParams fp, const int4* __restrict__ tiles,
                                                   Queue q, int n0, FrameCounters* fc) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i == 0) fc->count0 = n0;
    if (i >= n0) return;
    float4 o, d;
    const bool valid = primary_ray(cam, fp, tiles, i, o, d);
    q.ro[i] = o;
    q.rd[i] = d;
    q.time[i] = valid ? PGRT_IOR_AIR : 0.0f;  // raytracer.cpp:416
}

void launch_raygen(const CameraView& cam, const FrameParams& fp, const int4* tiles, Queue q, int n0,
                   FrameCounters* fc, hipStream_t stream) {
    if (n0 <= 0) return;
    hipLaunchKernelGGL(k_raygen, dim3(ceil_div(n0, kBlock)), dim3(kBlock), 0, stream, cam, fp, tiles, q, n0, fc);
}

// ------------------------------------------------------------------ shading (trace body)

// LDS_TABLES: the material and texture-descriptor tables are copied to LDS per block, so the
// hit -> attributes -> material -> texture chain has one global round trip fewer per hop
constexpr int kLdsMats = 64, kLdsTex = 32;

// queue allocation in k_shade: 0 two 32-bit atomics per wave, 1 one packed 64-bit atomic per
// wave, 2 one packed 64-bit atomic per block and grid-stride iteration
// child order in the next level's queue: 1 = per wave, its reflections then its refractions
#ifndef PGRT_CHILD_SPLIT
#define PGRT_CHILD_SPLIT 1
#endif
// k_shade block size: mode 2 issues one allocation atomic per block and iteration
#ifndef PGRT_SHADE_BLOCK
#define PGRT_SHADE_BLOCK 256
#endif
constexpr int kShadeBlock = PGRT_SHADE_BLOCK;
static_assert(kShadeBlock % kBlock == 0, "k_shade blocks are whole multiples of kBlock");
#ifndef PGRT_ALLOC_MODE
#define PGRT_ALLOC_MODE 2
#endif

template <bool LDS_TABLES, bool GEN>
__global__ __launch_bounds__(kShadeBlock) void k_shade(SceneView s, FrameParams fp, int level, Queue q, Queue next,
                                                  LevelNodes nodes, ShadowQueue sq, FrameCounters* fc, PrimaryGen gen,
                                                  int n_gen) {
    __shared__ float lut255[256];
    __shared__ DevMaterial smat[LDS_TABLES ? kLdsMats : 1];
    __shared__ DevTexture stex[LDS_TABLES ? kLdsTex : 1];
    if constexpr (LDS_TABLES) {
        for (int k = threadIdx.x; k < s.nmat; k += kShadeBlock) smat[k] = s.mats[k];
        for (int k = threadIdx.x; k < s.ntex; k += kShadeBlock) stex[k] = s.tex[k];
        s.tex = stex;  // env_texel / tex_texel read descriptors through s.tex
    }
#if PGRT_ALLOC_MODE == 2
    __shared__ unsigned long long s_wtot[2][kShadeBlock / 64];
    __shared__ unsigned long long s_bbase;
    int it_par = 0;
#endif
    const DevMaterial* mats = LDS_TABLES ? smat : s.mats;
    fill_byte_lut(lut255);  // ends with __syncthreads: the tables above are visible too
    // GEN (level 0, fused primary rays): n_gen rays regenerated from the camera, no ray queue
    // was written; this launch publishes the level-0 count in raygen's place
    const int n = GEN ? n_gen : min(fc_count(*fc, level), q.cap);
    const int tid = threadIdx.x;
    if (GEN && blockIdx.x == 0 && tid == 0) fc->count0 = n_gen;
    // one shadow queue for the whole batch: level L's rays follow those of levels < L (final by now)
    int sq_base = 0;
    for (int l = 0; l < level; ++l) sq_base += fc_shadow(*fc, l);
    const int sbits = s.nlight > 0 ? 32 - __clz(s.nlight) : 0;  // bits of a lane's shadow-ray count
    // software pipeline over the grid-stride loop: the next ray's record and hit are loaded
    // while this one is shaded (big queues give every thread several rays)
    const int stride = gridDim.x * kShadeBlock;
    float4 nx_o = make_float4(0, 0, 0, 0), nx_d = make_float4(0, 0, 0, 0), nx_h = make_float4(0, 0, 0, 0);
    float nx_t = 0.0f;
    {
        const int i0 = blockIdx.x * kShadeBlock + tid;
        if (i0 < n) {
            if constexpr (!GEN) {
                nx_o = q.ro[i0];
                nx_d = q.rd[i0];
                nx_t = q.time[i0];
            }
            nx_h = q.hit[i0];
        }
    }
    for (int base_i = blockIdx.x * kShadeBlock; base_i < n; base_i += stride) {
        const int i = base_i + tid;
        const bool active = i < n;
        float4 cur_o = nx_o, cur_d = nx_d;
        const float4 cur_h = nx_h;
        float cur_t = nx_t;
        if (i + stride < n) {
            if constexpr (!GEN) {
                nx_o = q.ro[i + stride];
                nx_d = q.rd[i + stride];
                nx_t = q.time[i + stride];
            }
            nx_h = q.hit[i + stride];
        }
        if constexpr (GEN) {
            if (active) cur_t = primary_ray(gen.cam, gen.fp, gen.tiles, i, cur_o, cur_d) ? PGRT_IOR_AIR : 0.0f;
        }
        int kind = 0;  // 0 final colour, 1 dielectric, 2 opaque (shadow rays pending)
        float4 color = make_float4(0, 0, 0, 1);
        int nshadow = 0, nchild = 0;
        V3 org = v3(0, 0, 0), dirraw = v3(0, 0, 0), d = v3(0, 0, 0), nrm = v3(0, 0, 0), hitp = v3(0, 0, 0);
        V3 refl_dir = v3(0, 0, 0), refr_dir = v3(0, 0, 0);
        float n1 = 0, n2 = 0, t = 0;
        float4 att = make_float4(0, 0, 0, 0);
        float m_d_r = 0, m_d_g = 0, m_d_b = 0;
        int mid = 0;
        if (active) {
            const float4 o4 = cur_o;
            const float4 d4 = cur_d;
            const float rtime = cur_t;
            const float4 h = cur_h;
            org = v3(o4.x, o4.y, o4.z);
            dirraw = v3(d4.x, d4.y, d4.z);
            if (d4.w < 0.0f) {
                color = make_float4(0, 0, 0, 0);  // padding slot
            } else {
                d = normalize(dirraw);
                const int prim = __float_as_int(h.w);
                if (prim < 0) {
                    color = env_texel(s, lut255, d);  // miss (raytracer.cpp:390-393)
                } else {
                    t = h.x;
                    const float* a = s.attr + 16 * (size_t)prim;
                    const float u = h.y, v = h.z;
                    V3 nn = v3(interp1(a[0], a[3], a[6], u, v), interp1(a[1], a[4], a[7], u, v),
                               interp1(a[2], a[5], a[8], u, v));
                    mid = __float_as_int(a[15]);
                    const DevMaterial& m = mats[mid];
                    nn = normalize(nn);
                    hitp = org + scale(t, dirraw);
                    if (rtime == PGRT_IOR_AIR) {
                        n1 = PGRT_IOR_AIR;
                        n2 = m.ior;
                    } else {
                        n1 = m.ior;
                        n2 = PGRT_IOR_AIR;
                    }
                    if (dot(nn, d) > 0) nn = -nn;
                    nrm = nn;
                    if (level >= fp.max_level) {
                        color = make_float4(0, 0, 0, 1);  // raytracer.cpp:282-283
                    } else if (m.type == PGRT_MATERIAL_DIELECTRIC) {
                        kind = 1;
                        {  // get_reflection_ray (raytracer.cpp:209-235)
                            const V3 dd = normalize(d), rn = normalize(nn);
                            refl_dir = dd - scale(2, scale(dot(dd, rn), rn));
                        }
                        att.x = pg_expf(-(1 - m.kd[0]) * t);  // raytracer.cpp:303-305
                        att.y = pg_expf(-(1 - m.kd[1]) * t);
                        att.z = pg_expf(-(1 - m.kd[2]) * t);
                        {  // get_refraction_ray (raytracer.cpp:178-207)
                            const V3 dd = normalize(d), rn = normalize(nn);
                            const float n1_n2 = n1 / n2;
                            const float d_n = dot(dd, rn);
                            const V3 sd = v3(dd.x * n1_n2, dd.y * n1_n2, dd.z * n1_n2);
                            const float kk = n1_n2 * d_n + sqrtf(1 - ((n1_n2 * n1_n2) * (1 - (d_n * d_n))));
                            refr_dir = sd - scale(kk, rn);
                        }
                        nchild = 1;
                        if (refr_dir.x == refr_dir.x) {  // no total internal reflection
                            nchild = 2;
                            const float cos1 = fabsf(dot(nn, -d));
                            const float alpha = (n1 - n2) / (n1 + n2);
                            att.w = (float)((double)(alpha * alpha + (1 - (alpha * alpha))) *
                                            pg_pow_d((double)(1 - cos1), 5.0));
                        }
                    } else {
                        kind = 2;
                        if (m.tex < 0) {
                            m_d_r = m.kd[2];
                            m_d_g = m.kd[1];
                            m_d_b = m.kd[0];
                        } else {
                            const float tu = interp1(a[9], a[11], a[13], u, v);
                            const float tv = interp1(a[10], a[12], a[14], u, v);
                            const V3 tx = tex_texel(s.tex[m.tex], s.texels, lut255, tu, 1.0f - tv);
                            m_d_r = tx.x;
                            m_d_g = tx.y;
                            m_d_b = tx.z;
                        }
                        for (int li = 0; li < s.nlight; ++li) {
                            const DevLight& L = s.lights[li];
                            if (!(dot(nn, v3(L.pos[0], L.pos[1], L.pos[2])) < 0)) ++nshadow;
                        }
                        color = make_float4(0, 0, 0, 1);
                    }
                }
            }
        }
        // ---- queue allocation (wave-uniform control flow) ----
        int cpre, ctot, spre, stot;
        wave_prefix_small(nchild, 2, cpre, ctot);
        wave_prefix_small(nshadow, sbits, spre, stot);
        const int rtot = (int)__popcll(__ballot(nchild == 2));
        const unsigned long long wtot = ((unsigned long long)(unsigned)stot << 32) | (unsigned)ctot;
        unsigned long long old = 0;
#if PGRT_ALLOC_MODE == 2
        // one returning atomic per BLOCK and iteration reserves both ranges (children | shadow
        // rays << 32) for its 4 waves: a quarter of the same-address atomics of a per-wave
        // allocation; wave totals double-buffered by iteration parity (a slow wave may still read
        // the previous iteration's entries when a fast one writes the next)
        {
            const int w = tid >> 6;
            if (__lane_id() == 0) {
                s_wtot[it_par][w] = wtot;
                if (rtot && level + 1 < kMaxLevels) atomicAdd(&fc->refract[level + 1], rtot);  // statistics
            }
            __syncthreads();
            if (tid == 0) {
                unsigned long long btot = 0;
                for (int k = 0; k < kShadeBlock / 64; ++k) btot += s_wtot[it_par][k];
                s_bbase = btot ? atomicAdd(&fc->alloc[level], btot) : 0ull;
            }
            __syncthreads();
            old = s_bbase;
            for (int k = 0; k < w; ++k) old += s_wtot[it_par][k];
            it_par ^= 1;
        }
#else
        if (__lane_id() == 0) {
#if PGRT_ALLOC_MODE == 1
            // one returning atomic per wave reserves both ranges (children | shadow rays << 32)
            if (wtot) old = atomicAdd(&fc->alloc[level], wtot);
#else
            // two 32-bit atomics per wave on the halves of the same word
            unsigned lo = 0, hi = 0;
            if (ctot) lo = atomicAdd(reinterpret_cast<unsigned*>(&fc->alloc[level]), (unsigned)ctot);
            if (stot) hi = atomicAdd(reinterpret_cast<unsigned*>(&fc->alloc[level]) + 1, (unsigned)stot);
            old = ((unsigned long long)hi << 32) | lo;
#endif
            if (rtot && level + 1 < kMaxLevels) atomicAdd(&fc->refract[level + 1], rtot);  // statistics: no return
        }
#endif
        const int cb = __builtin_amdgcn_readfirstlane((int)(unsigned)(old & 0xffffffffull));
        const int sb = __builtin_amdgcn_readfirstlane((int)(unsigned)(old >> 32));
#if PGRT_CHILD_SPLIT
        // the wave's reflection rays first, then its refraction rays, each group in pixel order:
        // the next level's waves are coherent bundles instead of alternating reflect / refract
        const unsigned long long mrefl = __ballot(nchild >= 1), mrefr = __ballot(nchild == 2);
        const int refl_slot = cb + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mrefl >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((unsigned)mrefl, 0u));
        const int refr_slot = cb + (int)__popcll(mrefl) +
                              (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mrefr >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((unsigned)mrefr, 0u));
        (void)cpre;
#else
        const int refl_slot = cb + cpre, refr_slot = refl_slot + 1;
#endif
        const int sbase = sq_base + sb + spre;
        if (!active) continue;
        int4 link = make_int4(-1, -1, -1, 0);
        if (kind == 1) {
            if ((nchild == 2 ? max(refl_slot, refr_slot) : refl_slot) >= next.cap || level + 1 >= kMaxLevels) {
                atomicOr(&fc->overflow, 1);
            } else {
                next.ro[refl_slot] = make_float4(hitp.x, hitp.y, hitp.z, 0.01f);
                next.rd[refl_slot] = make_float4(refl_dir.x, refl_dir.y, refl_dir.z, 3.402823466e+38f);
                next.time[refl_slot] = n1;
                link.x = refl_slot;
                if (nchild == 2) {
                    next.ro[refr_slot] = make_float4(hitp.x, hitp.y, hitp.z, 0.01f);
                    next.rd[refr_slot] = make_float4(refr_dir.x, refr_dir.y, refr_dir.z, 3.402823466e+38f);
                    next.time[refr_slot] = n2;
                    link.y = refr_slot;
                }
            }
            nodes.att[i] = att;
        } else if (kind == 2 && nshadow > 0) {
            if (sbase + nshadow > sq.cap) {
                atomicOr(&fc->overflow, 1);
            } else {
                const DevMaterial& m = mats[mid];
                int k = sbase;
                for (int li = 0; li < s.nlight; ++li) {
                    const DevLight& L = s.lights[li];
                    const V3 lp = v3(L.pos[0], L.pos[1], L.pos[2]);
                    if (dot(nrm, lp) < 0) continue;  // is_illuminated's N.L test (raytracer.cpp:155)
                    // LightSource::GenerateRay(hit): org = light, dir = hit position vector
                    sq.ro[k] = make_float4(lp.x, lp.y, lp.z, 0.01f);
                    sq.rd[k] = make_float4(hitp.x, hitp.y, hitp.z,
                                           length(v3(lp.x - hitp.x, lp.y - hitp.y, lp.z - hitp.z)));
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
                    const float tb = i_d_b * m_d_b * dot(nrm, lv) + i_s_b * m_s_b * spec;
                    const float tg = i_d_g * m_d_g * dot(nrm, lv) + i_s_g * m_s_g * spec;
                    const float tr = i_d_r * m_d_r * dot(nrm, lv) + i_s_r * m_s_r * spec;
                    sq.contrib[k] = make_float4(tb, tg, tr, 0.0f);
                    ++k;
                }
                link.z = sbase;
                link.w = nshadow;
            }
        }
        nodes.link[i] = link;
        if (link.x < 0 && link.z < 0) nodes.color[i] = color;  // else derived by k_finish
    }
}

void launch_shade(const SceneView& s, const FrameParams& fp, int level, Queue q, Queue next, LevelNodes nodes,
                  ShadowQueue sq, FrameCounters* fc, int max_count, hipStream_t stream, int expect,
                  const PrimaryGen* gen) {
    if (max_count <= 0) return;
    const int per_block = kShadeBlock / kBlock;  // grid_for counts kBlock-thread blocks
    const int grid = std::max(1, grid_for(max_count, expect) / per_block);
    const PrimaryGen g = gen ? *gen : PrimaryGen{};
    const bool lds = s.nmat <= kLdsMats && s.ntex <= kLdsTex;
#define PGRT_LAUNCH_S(L, G)                                                                                    \
    hipLaunchKernelGGL((k_shade<L, G>), dim3(grid), dim3(kShadeBlock), 0, stream, s, fp, level, q, next, nodes, sq, \
                       fc, g, max_count)
    if (lds) {
        if (gen) PGRT_LAUNCH_S(true, true); else PGRT_LAUNCH_S(true, false);
    } else {
        if (gen) PGRT_LAUNCH_S(false, true); else PGRT_LAUNCH_S(false, false);
    }
#undef PGRT_LAUNCH_S
}

// ------------------------------------------------------------------ combine + finish
//
// Colours are settled bottom-up.  k_combine(L), for L = max_level-1 .. 1, gives every level-L
// node its final colour: an opaque node is the sum of its lit Phong terms (the shadow resolve,
// raytracer.cpp:344-386 with is_illuminated :150-175), a dielectric node mixes its children of
// level L+1 (raytracer.cpp:316-321), any other node already carries its colour.  k_finish does
// the same for level 0 and then sums each pixel's samples in order (raytracer.cpp:422-429); the
// last batch applies the gamma (:431-435) and writes the framebuffer, earlier batches keep the
// running sum in `accum`.

__device__ __forceinline__ float4 opaque_color(const SceneView& s, const ShadowQueue& sq, int base, int cnt) {
    float blue = 0, green = 0, red = 0;
    for (int j = 0; j < cnt; ++j) {
        const int k = base + j;
        const int prim = __float_as_int(sq.hit[k].w);
        bool lit = true;  // is_illuminated (raytracer.cpp:163-173): closest hit decides
        if (prim >= 0) lit = s.prim_glass[prim] != 0;  // the occluder's material is dielectric
        if (lit) {
            const float4 c = sq.contrib[k];
            blue += c.x;
            green += c.y;
            red += c.z;
        }
    }
    return make_float4(blue, green, red, 1.0f);
}

// final colour of node i of a level whose children (next level) are final
__device__ __forceinline__ float4 node_color(const SceneView& s, const ShadowQueue& sq, LevelNodes nodes,
                                             const float4* __restrict__ child, int i) {
    const int4 lk = nodes.link[i];
    if (lk.x >= 0) {
        const float4 att = nodes.att[i];
        const float4 refl = child[lk.x];
        // raytracer.cpp:318-319 (refraction present) or :321 (total internal reflection)
        const float4 c = lk.y >= 0 ? mix_srgb(refl, child[lk.y], att.w) : refl;
        return make_float4(c.x * att.x, c.y * att.y, c.z * att.z, 1);
    }
    if (lk.z >= 0) return opaque_color(s, sq, lk.z, lk.w);
    return nodes.color[i];
}

__global__ __launch_bounds__(kBlock) void k_combine(SceneView s, int level, LevelNodes nodes,
                                                    const float4* __restrict__ child, ShadowQueue sq,
                                                    const FrameCounters* fc, int cap) {
    const int n = min(fc_count(*fc, level), cap);
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        const int4 lk = nodes.link[i];
        if (lk.x < 0 && lk.z < 0) continue;  // colour written by k_shade
        nodes.color[i] = node_color(s, sq, nodes, child, i);
    }
}

void launch_combine(const SceneView& s, int level, LevelNodes nodes, const float4* child, ShadowQueue sq,
                    const FrameCounters* fc, int max_count, hipStream_t stream, int expect) {
    if (max_count <= 0) return;
    const int grid = grid_for(max_count, expect);
    hipLaunchKernelGGL(k_combine, dim3(grid), dim3(kBlock), 0, stream, s, level, nodes, child, sq, fc, max_count);
}

__global__ __launch_bounds__(kBlock) void k_finish(SceneView s, FrameParams fp, const int4* __restrict__ tiles,
                                                   LevelNodes l0, const float4* __restrict__ child, ShadowQueue sq,
                                                   float4* __restrict__ accum, float* __restrict__ out, int out_mode,
                                                   int ox, int oy, int pitch, int npix, int first, int last, int K,
                                                   int j, int resolved) {
    const int p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= npix) return;
    float4 acc = first ? make_float4(0.0f, 0.0f, 0.0f, 1.0f) : accum[p];
    for (int k = 0; k < fp.nsb; ++k) {  // final_color += result_colors[x][y] (raytracer.cpp:422-429)
        // resolved: a k_combine pass over level 0 already wrote every sample's final colour (many
        // samples per pixel: their trees are evaluated in parallel, only the ordered sum is here)
        const float4 v = resolved ? l0.color[p * fp.nsb + k] : node_color(s, sq, l0, child, p * fp.nsb + k);
        acc.x += v.x;
        acc.y += v.y;
        acc.z += v.z;
    }
    if (!last) {
        accum[p] = acc;
        return;
    }
    int px, py;
    bool valid;
    tile_pixel(p, tiles, px, py, valid);
    if (!valid) return;
    const int area = fp.spp_side * fp.spp_side;
    // gamma(Color4f{final.b/area, final.g/area, final.r/area}) (raytracer.cpp:431-435)
    // x / 1 == x exactly: the (correctly rounded, ~10-instruction) divisions only for S > 1
    const float4 o = area == 1 ? gamma_rgba(acc.z, acc.y, acc.x, fp.gamma)
                               : gamma_rgba(acc.z / (float)area, acc.y / (float)area, acc.x / (float)area, fp.gamma);
    if (out_mode == 0) {
        float* dst = out + (size_t)frame_of_tile(fp, p / (kTile * kTile)) * fp.frame_stride +
                     ((size_t)(py - oy) * (size_t)pitch + (size_t)(px - ox)) * 4;
        *reinterpret_cast<float4*>(dst) = o;
        return;
    }
    const int tile = p / (kTile * kTile);
    const int4 tr = tiles[tile];
    size_t gtile = (size_t)tile * K + j;  // position in the caller's tile list
    if (fp.frame_tiles > 0) {  // multi-frame call: frame f's tiles start at f * frame_out_tiles
        const size_t f = gtile / fp.frame_tiles;
        gtile += f * (size_t)(fp.frame_out_tiles - fp.frame_tiles);
    }
    const size_t q = gtile * kTile * kTile + (size_t)(py - tr.y) * kTile + (size_t)(px - tr.x);
    if (out_mode == 1) {
        *reinterpret_cast<float4*>(out + q * 4) = o;
    } else {  // 2: RGB only (alpha is always 1): the multi-GPU gather moves 12 B per pixel
        out[q * 3 + 0] = o.x;
        out[q * 3 + 1] = o.y;
        out[q * 3 + 2] = o.z;
    }
}

void launch_finish(const SceneView& s, const FrameParams& fp, const int4* tiles, LevelNodes l0, const float4* child,
                   ShadowQueue sq, float4* accum, float* out, int out_mode, int ox, int oy, int pitch, int npix,
                   bool first, bool last, int K, int j, bool resolved, hipStream_t stream) {
    if (npix <= 0) return;
    hipLaunchKernelGGL(k_finish, dim3(ceil_div(npix, kBlock)), dim3(kBlock), 0, stream, s, fp, tiles, l0, child, sq,
                       accum, out, out_mode, ox, oy, pitch, npix, first ? 1 : 0, last ? 1 : 0, K, j, resolved ? 1 : 0);
}

// ------------------------------------------------------------------ multi-GPU unpack

// g holds, per rank, `frames` frames of tiles_per_rank tiles each (frame-major); frame `frame` of
// every rank is unpacked into rgba
__global__ __launch_bounds__(kBlock) void k_unpack(const float* __restrict__ g, float4* __restrict__ rgba, int width,
                                                   int height, int world, int tiles_per_rank, int channels,
                                                   int frames, int frame) {
    const long long idx = (long long)blockIdx.x * kBlock + threadIdx.x;
    const long long per_rank = (long long)tiles_per_rank * kTile * kTile;
    if (idx >= per_rank * world) return;
    const int rank = (int)(idx / per_rank);
    const long long r = idx - rank * per_rank;
    const int j = (int)(r / (kTile * kTile));
    const int p = (int)(r - (long long)j * kTile * kTile);
    const int tiles_x = (width + kTile - 1) / kTile;
    const int tiles_y = (height + kTile - 1) / kTile;
    const int t = j * world + rank;
    if (t >= tiles_x * tiles_y) return;
    const int x = (t % tiles_x) * kTile + (p % kTile);
    const int y = (t / tiles_x) * kTile + (p / kTile);
    if (x >= width || y >= height) return;
    const long long src = ((long long)rank * frames + frame) * per_rank + r;
    rgba[(size_t)y * width + x] = channels == 4 ? reinterpret_cast<const float4*>(g)[src]
                                                 : make_float4(g[src * 3], g[src * 3 + 1], g[src * 3 + 2], 1.0f);
}

void launch_unpack_tiles(const float* gathered, float* rgba, int width, int height, int world, int tiles_per_rank,
                         int channels, hipStream_t stream, int frames, int frame) {
    const long long total = (long long)world * tiles_per_rank * kTile * kTile;
    if (total <= 0) return;
    hipLaunchKernelGGL(k_unpack, dim3((unsigned)((total + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream, gathered,
                       reinterpret_cast<float4*>(rgba), width, height, world, tiles_per_rank, channels, frames, frame);
}

// ------------------------------------------------------------------ progressive accumulation
//
// The reference's Producer re-renders forever (simpleguidx11.cpp:86-128) and shows the latest
// frame; with jitter / DoF every frame is a new noisy estimate.  The frame sink keeps a running
// sum of the resolved frames (accumulated in frame order, one add per frame) and its mean.
__global__ __launch_bounds__(kBlock) void k_accumulate_frame(const float4* __restrict__ frame,
                                                            float4* __restrict__ sum, float4* __restrict__ mean,
                                                            long long n, int count) {
    const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float4 f = frame[i];
    float4 a = count == 1 ? f : sum[i];
    if (count > 1) {
        a.x += f.x;
        a.y += f.y;
        a.z += f.z;
        a.w += f.w;
    }
    sum[i] = a;
    const float c = (float)count;
    mean[i] = make_float4(a.x / c, a.y / c, a.z / c, a.w / c);
}

void launch_accumulate_frame(const float* frame, float* sum, float* mean, long long pixels, int count,
                             hipStream_t stream) {
    if (pixels <= 0) return;
    hipLaunchKernelGGL(k_accumulate_frame, dim3((unsigned)((pixels + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream,
                       reinterpret_cast<const float4*>(frame), reinterpret_cast<float4*>(sum),
                       reinterpret_cast<float4*>(mean), pixels, count);
}

// ------------------------------------------------------------------ counter export

// last launch of a slot's frame: the frame counters go to pinned host memory and the device
// copy is zeroed for the next frame (replaces a D2H copy + a memset: two fewer queue operations
// per frame)
__global__ void k_export_counters(uint4* dev, uint4* host, int n16) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += gridDim.x * blockDim.x) {
        host[i] = dev[i];
        dev[i] = make_uint4(0u, 0u, 0u, 0u);
    }
}

void launch_export_counters(FrameCounters* dev, FrameCounters* host, int n, hipStream_t stream) {
    static_assert(sizeof(FrameCounters) % 16 == 0, "FrameCounters must be a multiple of 16 bytes");
    const int n16 = (int)(sizeof(FrameCounters) / 16) * n;
    hipLaunchKernelGGL(k_export_counters, dim3((unsigned)std::min(64, (n16 + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       stream, reinterpret_cast<uint4*>(dev), reinterpret_cast<uint4*>(host), n16);
}

// ------------------------------------------------------------------ math self-test

__global__ void k_selftest(const float* in, int n, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float a = in[2 * i], b = in[2 * i + 1];
    float* o = out + 8 * (size_t)i;
    o[0] = sqrtf(a);
    o[1] = a / b;
    o[2] = gamma_pow(a, b);  // == pg_powf(a, b), with k_finish's exact y = 0.5 shortcut
    o[3] = pg_expf(a);
    o[4] = pg_atan2f(a, b);
    o[5] = pg_asinf(a);
    o[6] = 1 / sqrtf(a);
    o[7] = (float)pg_pow_d((double)a, (double)b);
}

void launch_selftest_math(const float* in, int n, float* out, hipStream_t stream) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_selftest, dim3(ceil_div(n, 256)), dim3(256), 0, stream, in, n, out);
}

}  // namespace pgrt
