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
#include "shade_ray.hpp"
#include "tiles.hpp"
#include "stamps.hpp"
#include "cache_ops.hpp"

namespace pgrt {

constexpr int kBlock = 256;

// grid of a grid-stride kernel: cover the expected count, at most 4096 workgroups
static int grid_for(int max_count, int expect) {
    const int n = (expect > 0 && expect < max_count) ? expect : max_count;
    const int g = ceil_div(n, kBlock);
    return g < 1 ? 1 : (g > 4096 ? 4096 : g);
}

// ------------------------------------------------------------------ ray generation

__global__ __launch_bounds__(kBlock) void k_raygen(CameraView cam, FrameParams fp, const int4* __restrict__ tiles,
                                                   Queue q, int n0, FrameCounters* fc,
                                                   unsigned long long* __restrict__ stamps) {
    PGRT_STAMP_BEGIN(stamps);
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i == 0) fc->count0 = n0;
    if (i < n0) {
        float4 o, d;
        const bool valid = primary_ray(cam, fp, tiles, i, o, d);
        st_stream(q.ro + i, o);
        st_stream(q.rd + i, d);
        st_stream_nt(q.time + i, valid ? PGRT_IOR_AIR : 0.0f);  // raytracer.cpp:416
    }
    PGRT_STAMP_END(stamps);
}

void launch_raygen(const CameraView& cam, const FrameParams& fp, const int4* tiles, Queue q, int n0,
                   FrameCounters* fc, hipStream_t stream) {
    if (n0 <= 0) return;
    const int grid = ceil_div(n0, kBlock);
    hipLaunchKernelGGL(k_raygen, dim3(grid), dim3(kBlock), 0, stream, cam, fp, tiles, q, n0, fc,
                       stamp_next(kStampRaygen, 0, grid, kBlock));
}

// ------------------------------------------------------------------ shading (trace body)

// k_shade block size (one allocation atomic per block and iteration, shade_ray.hpp; r1f A/B:
// 256 beat 512 and 1024).  The kernel is latency-bound (dependent hit -> attribute -> texel
// chain): it is compiled for 6 waves per SIMD (80 VGPRs, 2 spilled) instead of the 4 the
// unconstrained 98 VGPRs allow -- r2c C2 A/B: 0.1938 -> 0.1901 ms/frame (5 waves 0.1907)
constexpr int kShadeBlock = 256;
static_assert(kShadeBlock % kBlock == 0, "k_shade blocks are whole multiples of kBlock");
// level 0 of a 1-spp batch at 6 waves per SIMD (80 VGPRs; r4aa: driver line 0.177 -> 0.173 ms/frame)
#ifndef PGRT_SHADE_L0F_WAVES
#define PGRT_SHADE_L0F_WAVES 6
#endif
constexpr int kShadeL0fWaves = PGRT_SHADE_L0F_WAVES;
#ifndef PGRT_SHADE_WAVES
#define PGRT_SHADE_WAVES 6
#endif

#if PGRT_STEP_PROFILE
// diagnostics build only (tools/step_profile.py --shade): one record per wave and shading iteration
// -- the level, the shader-clock cycles of each phase (part A, allocation begin, part B, allocation
// end, emit) and the wave's rays by kind after part A (miss, dielectric, opaque, other)
constexpr int kShadeRecs = 1 << 20;
__device__ unsigned long long g_shade_rec[kShadeRecs][4];
__device__ unsigned g_shade_count;
extern "C" int pgrt_diag_shade_profile(unsigned long long* out, int max_records, int* n, int reset) {
    unsigned cnt = 0;
    if (hipMemcpyFromSymbol(&cnt, HIP_SYMBOL(g_shade_count), sizeof(cnt)) != hipSuccess) return PGRT_ERR_HIP;
    const unsigned m = std::min<unsigned>(std::min<unsigned>(cnt, (unsigned)kShadeRecs), (unsigned)std::max(0, max_records));
    if (out && m > 0 && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_shade_rec), sizeof(unsigned long long) * 4 * m) != hipSuccess)
        return PGRT_ERR_HIP;
    if (n) *n = (int)cnt;
    if (reset) {
        cnt = 0;
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_shade_count), &cnt, sizeof(cnt)) != hipSuccess) return PGRT_ERR_HIP;
    }
    return PGRT_OK;
}
#endif

// L0F: level 0 of a 1-spp batch (L0Final) -- final-colour pixels written here
template <bool LDS_TABLES, bool L0F>
__global__ __launch_bounds__(kShadeBlock, L0F ? kShadeL0fWaves : PGRT_SHADE_WAVES) void k_shade(SceneView s, FrameParams fp, int level, Queue q, Queue next,
                                                       LevelNodes nodes, ShadowQueue sq, FrameCounters* fc,
                                                       PinholeOrigin l0, L0Final l0f) {
    PGRT_STAMP_BEGIN(s.stamps);
    __shared__ float lut255[256];
    __shared__ DevMaterial smat[LDS_TABLES ? kLdsMats : 1];
    __shared__ DevTexture stex[LDS_TABLES ? kLdsTex : 1];
    __shared__ ShadeAllocLds<kShadeBlock> alds;
    if constexpr (LDS_TABLES) {
        for (int k = threadIdx.x; k < s.nmat; k += kShadeBlock) smat[k] = s.mats[k];
        for (int k = threadIdx.x; k < s.ntex; k += kShadeBlock) stex[k] = s.tex[k];
        s.tex = stex;  // env_texel / tex_texel read descriptors through s.tex
    }
    int it_par = 0, refr_acc = 0;
    const DevMaterial* mats = LDS_TABLES ? smat : s.mats;
    fill_byte_lut(lut255);  // ends with __syncthreads: the tables above are visible too
    const int n = min(fc_count(*fc, level), q.cap);
    const int tid = threadIdx.x;
    // one shadow queue for the whole batch: level L's rays follow those of levels < L (final by now)
    int sq_base = 0;
    for (int l = 0; l < level; ++l) sq_base += fc_shadow(*fc, l);
    const int sbits = s.nlight > 0 ? 32 - __clz(s.nlight) : 0;  // bits of a lane's shadow-ray count
    // software pipeline over the grid-stride loop: the next ray's record and hit are loaded
    // while this one is shaded (big queues give every thread several rays)
    const int stride = gridDim.x * kShadeBlock;
    float4 nx_o = make_float4(0, 0, 0, 0), nx_d = make_float4(0, 0, 0, 0), nx_h = make_float4(0, 0, 0, 0);
    float nx_t = 0.0f;
    // level 0 of a pinhole frame: only the directions were stored (camera_ops.hpp PrimaryGen)
    const bool from_cam = l0.on != 0;
    const float4 cam_o = make_float4(l0.x, l0.y, l0.z, 0.001f);
    // 1-spp level 0 (L0Final): a miss has no hit record (its mask bit is clear) and is finished here
    constexpr bool l0final = L0F;
    const float4 no_hit = make_float4(0.0f, 0.0f, 0.0f, __int_as_float(-1));
    auto load_hit = [&](int k) {
        if (!l0final) return ld_stream(q.hit + k);
        const unsigned long long hm = l0f.hit[__builtin_amdgcn_readfirstlane(k >> 6)];
        return ((hm >> (k & 63)) & 1ull) ? ld_stream(q.hit + k) : no_hit;
    };
    {
        const int i0 = blockIdx.x * kShadeBlock + tid;
        if (i0 < n) {
            nx_d = ld_stream(q.rd + i0);
            nx_h = load_hit(i0);
            if (!from_cam) {
                nx_o = ld_stream(q.ro + i0);
                nx_t = ld_stream_nt(q.time + i0);
            }
        }
    }
    for (int base_i = blockIdx.x * kShadeBlock; base_i < n; base_i += stride) {
        const int i = base_i + tid;
        const bool active = i < n;
        const float4 cur_d = nx_d, cur_h = nx_h;
        const float4 cur_o = from_cam ? cam_o : nx_o;
        const float cur_t = from_cam ? (cur_d.w >= 0.0f ? PGRT_IOR_AIR : 0.0f) : nx_t;
        if (i + stride < n) {
            nx_d = ld_stream(q.rd + i + stride);
            nx_h = load_hit(i + stride);
            if (!from_cam) {
                nx_o = ld_stream(q.ro + i + stride);
                nx_t = ld_stream_nt(q.time + i + stride);
            }
        }
        ShadeOut r;
        // the kind and slot counts first, the long-latency colours while the allocation atomic is
        // in flight (shade_eval_a / _b; r5s / r5t)
        ShadeDefer df;
#if PGRT_STEP_PROFILE
        const long long pc0 = clock64();
#endif
        shade_eval_a(s, mats, level, fp.max_level, active, cur_o, cur_d, cur_t, cur_h, r, df);
#if PGRT_STEP_PROFILE
        asm volatile("" ::"v"(r.kind), "v"(r.nchild), "v"(r.nshadow));
        const long long pc1 = clock64();
        const unsigned long long kmiss = __ballot(active && r.kind == 3), kdiel = __ballot(active && r.kind == 1),
                                 kopq = __ballot(active && r.kind == 2), kact = __ballot(active);
#endif
        if (level == 0 && fp.tile_deep) {  // a wave lies in one tile (4096 * nsb rays per tile)
            const unsigned long long dm = __ballot(active && r.nchild > 0);
            if (dm != 0ull && __lane_id() == 0) fp.tile_deep[(i / fp.nsb) / (kTile * kTile)] = 1;
        }
        if (fp.count) {  // profile == 2 only: one atomic pair per wave (the whole-frame roofline)
            const bool hit = active && cur_d.w >= 0.0f && __float_as_int(cur_h.w) >= 0;
            const unsigned long long hm = __ballot(hit), tm = __ballot(hit && r.kind == 2 && mats[r.mid].tex >= 0);
            if (__lane_id() == 0 && hm) {
                atomicAdd(&fc->shade[level][0], (unsigned long long)__popcll(hm));
                atomicAdd(&fc->shade[level][1], (unsigned long long)__popcll(tm));
            }
        }
        const ShadeAllocPending pa = shade_alloc_begin<kShadeBlock>(alds, it_par, fc, level, sbits, r, &refr_acc);
#if PGRT_STEP_PROFILE
        const long long pc2 = clock64();
#endif
        shade_eval_b(s, mats, lut255, r, df);
#if PGRT_STEP_PROFILE
        asm volatile("" ::"v"(r.color.x), "v"(r.att.x), "v"(r.m_d_r));
        const long long pc3 = clock64();
#endif
        const ShadeSlots sl = shade_alloc_end<kShadeBlock>(alds, it_par, sq_base, pa);
#if PGRT_STEP_PROFILE
        const long long pc4 = clock64();
#endif
        if constexpr (l0final) {
            // a final colour (environment texel; padding; a hit at max_level) -> the pixel, now;
            // the others are completed by the finish (n is a multiple of 64: whole waves)
            // shadow_final (one light): an opaque pixel without a shadow ray has its final colour
            // too (k_finish would read it back from its node: nodes.color = r.color), and one with
            // a shadow ray is completed by the shadow trace -- the finish keeps the dielectric ones
            const bool opaque = r.kind == 2 && l0f.shadow_final;
            const bool fin = active && (r.kind == 0 || (opaque && r.nshadow == 0));
            const bool by_shadow = active && opaque && r.nshadow > 0;
            const unsigned long long pend = __ballot(active && !fin && !by_shadow);
            if (active && __lane_id() == 0) st_stream_nt(l0f.pending + (i >> 6), pend);
            if (fin) store_final_1spp(fp, l0f.tiles, l0f.fo, i, r.color);
            if (active && !fin)
                shade_emit(s, mats, level, i, r, sl, next, nodes, sq, fc, false, make_float4(0, 0, 0, 0),
                           by_shadow ? i : -1);
        } else if (active) {
            // ShadowFinal at every level: an opaque node's one shadow ray carries the node
            shade_emit(s, mats, level, i, r, sl, next, nodes, sq, fc, false, make_float4(0, 0, 0, 0),
                       l0f.shadow_final && r.kind == 2 && r.nshadow > 0 ? i : -1);
        }
#if PGRT_STEP_PROFILE
        {
            const long long pc5 = clock64();
            if (__lane_id() == 0) {
                const unsigned slot = atomicAdd(&g_shade_count, 1u);
                if (slot < (unsigned)kShadeRecs) {
                    unsigned long long* rec = g_shade_rec[slot];
                    // [0] level | active | miss | dielectric | opaque lanes; [1] part A | alloc begin;
                    // [2] part B | alloc end; [3] emit | total (cycles, 32 bits each)
                    rec[0] = (unsigned long long)level | ((unsigned long long)__popcll(kact) << 8) |
                             ((unsigned long long)__popcll(kmiss) << 16) | ((unsigned long long)__popcll(kdiel) << 24) |
                             ((unsigned long long)__popcll(kopq) << 32);
                    rec[1] = (unsigned long long)(unsigned)(pc1 - pc0) | ((unsigned long long)(unsigned)(pc2 - pc1) << 32);
                    rec[2] = (unsigned long long)(unsigned)(pc3 - pc2) | ((unsigned long long)(unsigned)(pc4 - pc3) << 32);
                    rec[3] = (unsigned long long)(unsigned)(pc5 - pc4) | ((unsigned long long)(unsigned)(pc5 - pc0) << 32);
                }
            }
        }
#endif
    }
    shade_refract_flush(fc, level, refr_acc);
    PGRT_STAMP_END(s.stamps);
}

void launch_shade(const SceneView& s_in, const FrameParams& fp, int level, Queue q, Queue next, LevelNodes nodes,
                  ShadowQueue sq, FrameCounters* fc, int max_count, hipStream_t stream, int expect,
                  const PinholeOrigin& l0, const L0Final& l0f) {
    if (max_count <= 0) return;
    const int per_block = kShadeBlock / kBlock;  // grid_for counts kBlock-thread blocks
    const int grid = std::max(1, grid_for(max_count, expect) / per_block);
    SceneView s = s_in;
    s.stamps = stamp_next(kStampShade, level, grid, kShadeBlock);
    const bool lds = s.nmat <= kLdsMats && s.ntex <= kLdsTex;
#define PGRT_LAUNCH_SHADE(T, F)                                                                                   \
    hipLaunchKernelGGL((k_shade<T, F>), dim3(grid), dim3(kShadeBlock), 0, stream, s, fp, level, q, next, nodes, sq, \
                       fc, l0, l0f)
    if (l0f.hit) {
        if (lds) PGRT_LAUNCH_SHADE(true, true); else PGRT_LAUNCH_SHADE(false, true);
    } else {
        if (lds) PGRT_LAUNCH_SHADE(true, false); else PGRT_LAUNCH_SHADE(false, false);
    }
#undef PGRT_LAUNCH_SHADE
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
        // the Phong term is loaded beside the verdict, not behind it (one round trip fewer per
        // pending pixel; an unlit ray's 16 B are read for nothing)
        const float4 c = ld_stream(sq.contrib + k);
        bool lit;  // is_illuminated (raytracer.cpp:163-173): closest hit decides
        if (sq.lit) {
            lit = ld_stream_nt(sq.lit + k) != 0;  // decided by the shadow trace (compact queue)
        } else {
            const int prim = __float_as_int(ld_stream(sq.hit + k).w);
            lit = prim < 0 || *at_bytes(s.prim_glass, (unsigned)prim) != 0;  // no occluder, or a dielectric one
        }
        if (lit) {
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
    const int4 lk = ld_stream(nodes.link + i);
    if (lk.x >= 0) {
        const float4 att = ld_stream(nodes.att + i);
        const float4 refl = ld_stream(child + lk.x);
        // raytracer.cpp:318-319 (refraction present) or :321 (total internal reflection)
        const float4 c = lk.y >= 0 ? mix_srgb(refl, ld_stream(child + lk.y), att.w) : refl;
        return make_float4(c.x * att.x, c.y * att.y, c.z * att.z, 1);
    }
    if (lk.z >= 0) return opaque_color(s, sq, lk.z, lk.w);
    return ld_stream(nodes.color + i);
}

__global__ __launch_bounds__(kBlock) void k_combine(SceneView s, int level, LevelNodes nodes,
                                                    const float4* __restrict__ child, ShadowQueue sq,
                                                    const FrameCounters* fc, int cap) {
    PGRT_STAMP_BEGIN(s.stamps);
    const int n = min(fc_count(*fc, level), cap);
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        const int4 lk = ld_stream(nodes.link + i);
        if (lk.x < 0 && lk.z < 0) continue;  // colour written by k_shade
        st_stream(nodes.color + i, node_color(s, sq, nodes, child, i));
    }
    PGRT_STAMP_END(s.stamps);
}

void launch_combine(const SceneView& s_in, int level, LevelNodes nodes, const float4* child, ShadowQueue sq,
                    const FrameCounters* fc, int max_count, hipStream_t stream, int expect) {
    if (max_count <= 0) return;
    const int grid = grid_for(max_count, expect);
    SceneView s = s_in;
    s.stamps = stamp_next(kStampCombine, level, grid, kBlock);
    hipLaunchKernelGGL(k_combine, dim3(grid), dim3(kBlock), 0, stream, s, level, nodes, child, sq, fc, max_count);
}

__device__ __forceinline__ void finish_body(const SceneView& s, const FrameParams& fp, const int4* __restrict__ tiles,
                                            const LevelNodes& l0, const float4* __restrict__ child,
                                            const ShadowQueue& sq, float4* __restrict__ accum, const FrameOut& fo,
                                            int npix, int first, int last, int resolved) {
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
    store_pixel(fp, tiles, fo, p, px, py, o);
}

__global__ __launch_bounds__(kBlock) void k_finish(SceneView s, FrameParams fp, const int4* __restrict__ tiles,
                                                   LevelNodes l0, const float4* __restrict__ child, ShadowQueue sq,
                                                   float4* __restrict__ accum, FrameOut fo, int npix, int first,
                                                   int last, int resolved) {
    PGRT_STAMP_BEGIN(s.stamps);
    finish_body(s, fp, tiles, l0, child, sq, accum, fo, npix, first, last, resolved);
    PGRT_STAMP_END(s.stamps);
}

// 1-spp batch whose level-0 shade finished every final-colour pixel (L0Final): the pixels of the
// pending masks only (with ShadowFinal: the dielectric ones)
__global__ __launch_bounds__(kBlock) void k_finish_pending(SceneView s, FrameParams fp, const int4* __restrict__ tiles,
                                                           LevelNodes l0, const float4* __restrict__ child,
                                                           ShadowQueue sq, FrameOut fo,
                                                           const unsigned long long* __restrict__ pending, int npix) {
    PGRT_STAMP_BEGIN(s.stamps);
    const int p = blockIdx.x * kBlock + threadIdx.x;
    if (p < npix) {
        const unsigned long long pm = pending[__builtin_amdgcn_readfirstlane(p >> 6)];
        if (((pm >> (p & 63)) & 1ull) != 0ull) store_final_1spp(fp, tiles, fo, p, node_color(s, sq, l0, child, p));
    }
    PGRT_STAMP_END(s.stamps);
}

void launch_finish(const SceneView& s_in, const FrameParams& fp, const int4* tiles, LevelNodes l0, const float4* child,
                   ShadowQueue sq, float4* accum, const FrameOut& fo, int npix, bool first, bool last, bool resolved,
                   const unsigned long long* pending, hipStream_t stream) {
    if (npix <= 0) return;
    SceneView s = s_in;
    s.stamps = stamp_next(kStampFinish, 0, ceil_div(npix, kBlock), kBlock);
    if (pending) {
        hipLaunchKernelGGL(k_finish_pending, dim3(ceil_div(npix, kBlock)), dim3(kBlock), 0, stream, s, fp, tiles, l0,
                           child, sq, fo, pending, npix);
        return;
    }
    hipLaunchKernelGGL(k_finish, dim3(ceil_div(npix, kBlock)), dim3(kBlock), 0, stream, s, fp, tiles, l0, child, sq,
                       accum, fo, npix, first ? 1 : 0, last ? 1 : 0, resolved ? 1 : 0);
}

// ------------------------------------------------------------------ multi-GPU unpack

// u.src[r] holds rank r's tiles of `frames` frames (frame-major, u.count[r] tiles per frame in
// the rank's local order of the tiles.hpp deal, `channels` floats per pixel); blockIdx.y = frame
// - frame0; every rank's tiles of that frame are unpacked into rgba + frame * W*H*4
__device__ __forceinline__ void unpack_body(const UnpackSrc& u, float4* __restrict__ rgba, int width, int height,
                                            const TileDeal& deal, int channels, int frame0) {
    const int world = deal.world;
    const int frame = frame0 + (int)blockIdx.y;
    const long long idx = (long long)blockIdx.x * kBlock + threadIdx.x;
    const int tile_slot = (int)(idx / (kTile * kTile));
    if (tile_slot >= u.prefix[world]) return;
    int rank = 0;
    while (rank + 1 < world && u.prefix[rank + 1] <= tile_slot) ++rank;
    const int j = tile_slot - u.prefix[rank];
    const int p = (int)(idx - (long long)tile_slot * kTile * kTile);
    const int tiles_x = (width + kTile - 1) / kTile;
    const int t = deal_tile(deal, rank, j);
    const int x = (t % tiles_x) * kTile + (p % kTile);
    const int y = (t / tiles_x) * kTile + (p / kTile);
    if (x >= width || y >= height) return;  // padding of an edge tile
    const long long src = ((long long)frame * u.count[rank] + j) * kTile * kTile + p;
    const float* g = u.src[rank];
    if (!g) return;  // a rank left out of this unpack (a re-gather of the re-rendered ranks only)
    rgba[(size_t)frame * width * height + (size_t)y * width + x] =
        channels == 4 ? reinterpret_cast<const float4*>(g)[src]
                      : make_float4(g[src * 3], g[src * 3 + 1], g[src * 3 + 2], 1.0f);
}

__global__ __launch_bounds__(kBlock) void k_unpack(UnpackSrc u, float4* __restrict__ rgba, int width, int height,
                                                   TileDeal deal, int channels, int frame0,
                                                   unsigned long long* __restrict__ stamps) {
    PGRT_STAMP_BEGIN(stamps);
    unpack_body(u, rgba, width, height, deal, channels, frame0);
    PGRT_STAMP_END(stamps);
}

void launch_unpack_tiles(const UnpackSrc& u, float* rgba, int width, int height, const TileDeal& deal, int channels,
                         hipStream_t stream, int frame0, int nframes) {
    const long long total = (long long)u.prefix[deal.world] * kTile * kTile;
    if (total <= 0 || nframes <= 0) return;
    const unsigned gx = (unsigned)((total + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_unpack, dim3(gx, (unsigned)nframes), dim3(kBlock), 0, stream, u,
                       reinterpret_cast<float4*>(rgba), width, height, deal, channels, frame0,
                       stamp_next(kStampUnpack, -1, (long long)gx * nframes, kBlock));
}

// ------------------------------------------------------------------ distributed overflow flags

__global__ void k_overflow_flag(FlagSrc f, int* out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int v = 0;
    for (int j = 0; j < f.K; ++j)
        for (int b = 0; b < f.n[j]; ++b) v |= f.fc[j][b].overflow;
    out[0] = gather_tail_flag(v != 0, f.poison != 0);
    out[1] = (int)f.seq;
}

void launch_overflow_flag(const FlagSrc& f, int* out, hipStream_t stream) {
    hipLaunchKernelGGL(k_overflow_flag, dim3(1), dim3(64), 0, stream, f, out);
}

__global__ void k_peer_flags(UnpackSrc u, int world, size_t floats_per_tile_count, int* flags) {
    const int r = threadIdx.x;
    if (r >= 1 && r < world) {  // src NULL: a rank not received in this gather
        const int* tail = u.src[r] ? reinterpret_cast<const int*>(u.src[r] + floats_per_tile_count * (size_t)u.count[r])
                                   : nullptr;
        flags[r] = tail ? tail[0] : 0;
        flags[kMaxRanks + r] = tail ? tail[1] : 0;
    }
}

void launch_peer_flags(const UnpackSrc& u, int world, size_t floats_per_tile_count, int* flags, hipStream_t stream) {
    hipLaunchKernelGGL(k_peer_flags, dim3(1), dim3(64), 0, stream, u, world, floats_per_tile_count, flags);
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

// ------------------------------------------------------------------ host framebuffer export
//
// SURVEY.md §8(d) times a frame to the framebuffer on the host (the reference's Producer copies
// it under the mutex, simpleguidx11.cpp:120-124).  A blit kernel storing into page-locked host
// memory moves 53 GB/s over PCIe where an SDMA copy of the same 33 MB moved 28-44
// (profiles/r5/r5a/d2h_probe.txt), and one is launched per pipeline slot right after that slot's
// finish: the bulk slot's pixels cross PCIe while the deep-tile slot is still rendering.  One wave
// per tile row: 64 consecutive 16-B pixels, full lines on the link.
__global__ __launch_bounds__(kBlock) void k_export_tiles(const int4* __restrict__ tiles, int rows,
                                                         const float4* __restrict__ src, float4* __restrict__ dst,
                                                         int ox, int oy, int pitch, long long frame_stride4,
                                                         unsigned long long* __restrict__ stamps) {
    PGRT_STAMP_BEGIN(stamps);
    const int x = threadIdx.x & 63;
    // only the workgroups the dispatcher places on XCD 0 (workgroups go to the 8 XCDs round-robin:
    // blockIdx % 8 == 0) copy: the PCIe stores then queue in one XCD's L2 and fabric port, and the
    // concurrent slot's waves on the other seven XCDs never wait behind them
    if (blockIdx.x % kXcds != 0) {
        PGRT_STAMP_END(stamps);
        return;
    }
    const int wg = blockIdx.x / kXcds, nwg = gridDim.x / kXcds;
    for (int r = wg * (kBlock / 64) + (threadIdx.x >> 6); r < rows; r += nwg * (kBlock / 64)) {
        const int4 tr = tiles[r >> 6];  // 64 rows per tile
        const int ly = r & 63;
        if (ly >= tr.w || x >= tile_width(tr)) continue;
        const size_t o = (size_t)frame_of_tile(tr) * (size_t)frame_stride4 + (size_t)(tr.y + ly - oy) * (size_t)pitch +
                         (size_t)(tr.x + x - ox);
        dst[o] = ld_stream(src + o);
    }
    PGRT_STAMP_END(stamps);
}

void launch_export_tiles(const int4* tiles, int ntiles, const float* src, float* dst_host, int ox, int oy, int pitch,
                         long long frame_stride, hipStream_t stream) {
    if (ntiles <= 0) return;
    const int rows = ntiles * kTile;
    // 32 copying workgroups, all on XCD 0 (r5h, synchronous host frame: 0.96 ms; 32 spread over the
    // 8 XCDs 1.02, 8 on XCD 0 1.18; r5d spread: 64 1.12, 256 1.14, 16 1.09-1.12, 8 1.32)
#ifndef PGRT_EXPORT_WG
#define PGRT_EXPORT_WG 32
#endif
    const int grid = kXcds * std::max(1, std::min(PGRT_EXPORT_WG, ceil_div(rows, kBlock / 64)));
    hipLaunchKernelGGL(k_export_tiles, dim3(grid), dim3(kBlock), 0, stream, tiles, rows,
                       reinterpret_cast<const float4*>(src), reinterpret_cast<float4*>(dst_host), ox, oy, pitch,
                       frame_stride / 4, stamp_next(kStampExportTiles, -1, grid, kBlock));
}

// A linear share of a host-output call's framebuffer into page-locked memory (PGRT_HOST_EXPORT_SPLIT):
// the copying workgroups on XCD 0 only, as k_export_tiles
__global__ __launch_bounds__(kBlock) void k_blit_host(const float4* __restrict__ src, float4* __restrict__ dst,
                                                      long long n4, unsigned long long* __restrict__ stamps) {
    PGRT_STAMP_BEGIN(stamps);
    if (blockIdx.x % kXcds == 0) {
        const long long nthr = (long long)(gridDim.x / kXcds) * kBlock;
        for (long long i = (long long)(blockIdx.x / kXcds) * kBlock + threadIdx.x; i < n4; i += nthr)
            dst[i] = ld_stream(src + i);
    }
    PGRT_STAMP_END(stamps);
}

void launch_blit_host(const float* src, float* dst_host, size_t bytes, hipStream_t stream) {
    const long long n4 = (long long)(bytes / 16);
    if (n4 <= 0) return;
    const int grid = kXcds * PGRT_EXPORT_WG;
    hipLaunchKernelGGL(k_blit_host, dim3(grid), dim3(kBlock), 0, stream, reinterpret_cast<const float4*>(src),
                       reinterpret_cast<float4*>(dst_host), n4, stamp_next(kStampExportTiles, -1, grid, kBlock));
}

// ------------------------------------------------------------------ counter export

// last launch of a slot's frame: the frame counters go to pinned host memory and the device
// copy is zeroed for the next frame (replaces a D2H copy + a memset: two fewer queue operations
// per frame)
__global__ void k_export_counters(uint4* dev, uint4* host, int n16, int* __restrict__ deep_dev,
                                  int* __restrict__ deep_host, int ndeep, unsigned long long* __restrict__ stamps) {
    PGRT_STAMP_BEGIN(stamps);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += gridDim.x * blockDim.x) {
        host[i] = dev[i];
        dev[i] = make_uint4(0u, 0u, 0u, 0u);
    }
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < ndeep; i += gridDim.x * blockDim.x) {
        deep_host[i] = deep_dev[i];
        deep_dev[i] = 0;
    }
    PGRT_STAMP_END(stamps);
}

void launch_export_counters(FrameCounters* dev, FrameCounters* host, int n, int* deep_dev, int* deep_host, int ndeep,
                            hipStream_t stream) {
    static_assert(sizeof(FrameCounters) % 16 == 0, "FrameCounters must be a multiple of 16 bytes");
    const int n16 = (int)(sizeof(FrameCounters) / 16) * n;
    if (!deep_dev || !deep_host) ndeep = 0;
    const int grid = std::min(64, (std::max(n16, ndeep) + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_export_counters, dim3((unsigned)grid), dim3(kBlock), 0, stream, reinterpret_cast<uint4*>(dev),
                       reinterpret_cast<uint4*>(host), n16, deep_dev, deep_host, ndeep,
                       stamp_next(kStampExport, -1, grid, kBlock));
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
    o[4] = atan2f_env(a, b);  // == pg_atan2f(a, b): the env map's fast path with its rounding test
    o[5] = asinf_env(a);      // == pg_asinf(a)
    o[6] = 1 / sqrtf(a);
    o[7] = (float)pg_pow_d((double)a, (double)b);
}

// srgb_expand / srgb_compress (the kernels' form) vs their exact pg_pow_d form, bitwise, over a
// range of float bit patterns (grid-stride); mismatches counted per function
__global__ __launch_bounds__(256) void k_selftest_srgb(uint32_t first, uint32_t count, unsigned long long* mism) {
    unsigned long long me = 0, mc = 0;
    for (uint32_t k = blockIdx.x * 256u + threadIdx.x; k < count; k += gridDim.x * 256u) {
        const float u = __uint_as_float(first + k);
        me += __float_as_uint(srgb_expand(u)) != __float_as_uint(srgb_expand_exact(u)) ? 1ull : 0ull;
        mc += __float_as_uint(srgb_compress(u)) != __float_as_uint(srgb_compress_exact(u)) ? 1ull : 0ull;
    }
    if (me) atomicAdd(&mism[0], me);
    if (mc) atomicAdd(&mism[1], mc);
}

void launch_selftest_srgb(uint32_t first_bits, uint32_t count, unsigned long long* mismatches, hipStream_t stream) {
    if (count == 0) return;
    hipLaunchKernelGGL(k_selftest_srgb, dim3(16384), dim3(256), 0, stream, first_bits, count, mismatches);
}

void launch_selftest_math(const float* in, int n, float* out, hipStream_t stream) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_selftest, dim3(ceil_div(n, 256)), dim3(256), 0, stream, in, n, out);
}

}  // namespace pgrt
