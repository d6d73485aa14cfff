// path.hip -- PGRT_MODE_PATH: the path tracer of the reference's README to-do list
// ("Whole pathtracing", README.md:17-21) on the same wavefront queues as the Whitted frames.
//
// The reference has no path tracer; the semantics (DESIGN.md §2 "Path tracing", restated in
// oracle/oracle.c path_sample) reuse its pieces: trace()'s hit setup, dielectric rays,
// attenuation and Fresnel-like R (APP/raytracer.cpp:241-316), the Phong term (:355-382) and the
// environment lookup on a miss (:390-393).  A path has at most one continuation ray per bounce,
// so there is no colour tree: every path carries its throughput T (float4 per queue entry) and
// its index into the batch's path accumulators (the level-0 ray index), and contributions are
// added to the accumulator in bounce order -- one bounce = trace, k_path_shade (miss: T * env;
// dielectric: reflect or refract; opaque: hard shadow rays with their T * Phong terms, then a
// cosine-weighted bounce), the bounce's shadow rays traced, k_path_resolve (lit terms added in
// light order by the path's first shadow ray).  Same float operations as the oracle, so frames
// are bit-identical to it.
#include "shade_ops.hpp"
#include "trace.hpp"
#include "camera_ops.hpp"
#include "shade_ray.hpp"
#include "path.hpp"

#include "stamps.hpp"

namespace pgrt {

constexpr int kPathBlock = 256;

// Building an orthonormal basis, revisited (Duff et al. 2017); oracle.c onb
__device__ __forceinline__ void path_onb(V3 n, V3& b1, V3& b2) {
    const float sign = copysignf(1.0f, n.z);
    const float a = -1.0f / (sign + n.z);
    const float b = n.x * n.y * a;
    b1 = v3(1.0f + sign * n.x * n.x * a, sign * b, -sign * n.x);
    b2 = v3(b, sign + n.y * n.y * a, -n.y);
}

// cosine-weighted direction about n (oracle.c cosine_dir): Malley's method over a
// rejection-sampled unit disk, up to 8 candidates, else the pole
__device__ __forceinline__ V3 path_cosine_dir(uint32_t key, uint32_t bounce, V3 n) {
    float x = 0.0f, y = 0.0f;
    for (uint32_t j = 0; j < 8u; ++j) {
        const float a = 2.0f * pg_path_u01(key, bounce, 1u + 2u * j) - 1.0f;
        const float c = 2.0f * pg_path_u01(key, bounce, 2u + 2u * j) - 1.0f;
        if (a * a + c * c < 1.0f) {
            x = a;
            y = c;
            break;
        }
    }
    const float z = sqrtf(1.0f - (x * x + y * y));
    V3 b1, b2;
    path_onb(n, b1, b2);
    return v3(x * b1.x + y * b2.x + z * n.x, x * b1.y + y * b2.y + z * n.y, x * b1.z + y * b2.z + z * n.z);
}

// the counter-hash key of path pid (level-0 ray index of the batch): its image pixel, sample
// and frame, as primary_ray derives them
__device__ __forceinline__ uint32_t path_key(const FrameParams& fp, const int4* tiles, int width, int pid) {
    const int slot_pix = pid / fp.nsb;
    const int sample = fp.s0 + (pid - slot_pix * fp.nsb);
    int px, py;
    bool valid;
    tile_pixel(slot_pix, tiles, px, py, valid);
    const uint32_t frame = fp.frame + (uint32_t)frame_of_tile(tiles[slot_pix / (kTile * kTile)]);
    return pg_path_key(fp.seed, frame, (uint32_t)py * (uint32_t)width + (uint32_t)px, (uint32_t)sample);
}

template <bool LDS_TABLES>
__global__ __launch_bounds__(kPathBlock) void k_path_shade(SceneView s, FrameParams fp, int width,
                                                           const int4* __restrict__ tiles, int level, Queue q,
                                                           Queue next, PathState ps, ShadowQueue sq,
                                                           FrameCounters* fc) {
    PGRT_STAMP_BEGIN(s.stamps);
    __shared__ float lut255[256];
    __shared__ DevMaterial smat[LDS_TABLES ? kLdsMats : 1];
    __shared__ DevTexture stex[LDS_TABLES ? kLdsTex : 1];
    __shared__ ShadeAllocLds<kPathBlock> alds;
    if constexpr (LDS_TABLES) {
        for (int k = threadIdx.x; k < s.nmat; k += kPathBlock) smat[k] = s.mats[k];
        for (int k = threadIdx.x; k < s.ntex; k += kPathBlock) stex[k] = s.tex[k];
        s.tex = stex;
    }
    const DevMaterial* mats = LDS_TABLES ? smat : s.mats;
    fill_byte_lut(lut255);  // ends with __syncthreads
    int it_par = 0, refr_w = 0;
    const int n = min(fc_count(*fc, level), q.cap);
    const int sbits = s.nlight > 0 ? 32 - __clz(s.nlight) : 0;
    for (int base_i = blockIdx.x * kPathBlock; base_i < n; base_i += gridDim.x * kPathBlock) {
        const int i = base_i + threadIdx.x;
        const bool active = i < n;
        float4 o4 = make_float4(0, 0, 0, 0), d4 = make_float4(0, 0, 0, -1.0f), h = make_float4(0, 0, 0, 0);
        float rtime = 0.0f;
        int pid = i;
        float4 T = make_float4(1.0f, 1.0f, 1.0f, 0.0f);
        if (active) {
            o4 = q.ro[i];
            d4 = q.rd[i];
            rtime = q.time[i];
            h = q.hit[i];
            if (level > 0) {
                pid = ps.pid_in[i];
                T = ps.thr_in[i];
            }
        }
        ShadeOut r;
        shade_eval(s, mats, lut255, level, fp.max_level, active, o4, d4, rtime, h, r);
        const bool miss = active && d4.w >= 0.0f && __float_as_int(h.w) < 0;
        // the path's continuation (0 / 1 ray) and its lit candidates (shadow rays)
        int child = 0, refract = 0;
        float4 Tn = T;
        V3 cdir = v3(0, 0, 0);
        float ctime = rtime;
        uint32_t key = 0;
        int nsh = 0;
        if (r.kind == 1) {  // dielectric: T *= attenuation, reflect or refract (oracle path_sample)
            if (r.nchild == 2) {
                key = path_key(fp, tiles, width, pid);
                refract = !(pg_path_u01(key, (uint32_t)level, 0u) < r.att.w) ? 1 : 0;
            }
            Tn = make_float4(T.x * r.att.x, T.y * r.att.y, T.z * r.att.z, 0.0f);
            child = 1;
            cdir = refract ? r.refr_dir : r.refl_dir;
            ctime = refract ? r.n2 : r.n1;
        } else if (r.kind == 2) {  // opaque: hard shadow rays, then a cosine-weighted bounce
            for (int li = 0; li < s.nlight; ++li) {
                const DevLight& L = s.lights[li];
                const V3 tol = v3(L.pos[0] - r.hitp.x, L.pos[1] - r.hitp.y, L.pos[2] - r.hitp.z);
                if (dot(r.nrm, tol) > 0) ++nsh;
            }
            Tn = make_float4(T.x * r.m_d_b, T.y * r.m_d_g, T.z * r.m_d_r, 0.0f);
            if (Tn.x > 0.0f || Tn.y > 0.0f || Tn.z > 0.0f) {
                key = path_key(fp, tiles, width, pid);
                cdir = path_cosine_dir(key, (uint32_t)level, r.nrm);
                child = 1;
            }
        }
        // slots: the Whitted allocation (one packed atomic per block and iteration)
        ShadeOut a;
        a.nchild = child;
        a.nshadow = nsh;
        const ShadeSlots sl = shade_alloc<kPathBlock>(alds, it_par, fc, level, 0, sbits, a);
        const unsigned long long mref = __ballot(child && refract);
        refr_w += (int)__popcll(mref);  // statistics: one atomic per wave and launch (below)
        if (!active) continue;
        if (level == 0) {  // the path's accumulator starts at 0 (oracle: L = {0, 0, 0})
            const float4 e = miss ? r.color : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            ps.acc[pid] = make_float4(0.0f + T.x * e.x, 0.0f + T.y * e.y, 0.0f + T.z * e.z, 1.0f);
        } else if (miss) {
            const float4 acc = ps.acc[pid];
            ps.acc[pid] = make_float4(acc.x + T.x * r.color.x, acc.y + T.y * r.color.y, acc.z + T.z * r.color.z, 1.0f);
        }
        if (child) {
            if (sl.refl >= next.cap) {
                atomicOr(&fc->overflow, 1);
            } else {
                next.ro[sl.refl] = make_float4(r.hitp.x, r.hitp.y, r.hitp.z, 0.01f);
                next.rd[sl.refl] = make_float4(cdir.x, cdir.y, cdir.z, 3.402823466e+38f);
                next.time[sl.refl] = ctime;
                ps.pid_out[sl.refl] = pid;
                ps.thr_out[sl.refl] = Tn;
            }
        }
        if (nsh > 0) {
            if (sl.shadow + nsh > sq.cap) {
                atomicOr(&fc->overflow, 1);
            } else {
                const DevMaterial& m = mats[r.mid];
                int k = sl.shadow;
                for (int li = 0; li < s.nlight; ++li) {
                    const DevLight& L = s.lights[li];
                    const V3 lp = v3(L.pos[0], L.pos[1], L.pos[2]);
                    const V3 tol = v3(lp.x - r.hitp.x, lp.y - r.hitp.y, lp.z - r.hitp.z);
                    if (!(dot(r.nrm, tol) > 0)) continue;
                    const V3 lv = normalize(tol);
                    sq.ro[k] = make_float4(r.hitp.x, r.hitp.y, r.hitp.z, 0.01f);
                    sq.rd[k] = make_float4(lv.x, lv.y, lv.z, length(tol));
                    // the Phong term of shade_phong (raytracer.cpp:355-382), times T
                    const V3 cv = normalize(v3(r.org.x - r.dirraw.x, r.org.y - r.dirraw.y, r.org.z - r.dirraw.z));
                    const float nl = dot(r.nrm, lv);
                    V3 l_r = scale(2 * nl, r.nrm) - lv;
                    l_r = normalize(l_r);
                    const float spec = pg_powf(dot(cv, l_r), m.ns);
                    const float tb = L.kd[0] * r.m_d_b * dot(r.nrm, lv) + L.ks[0] * m.ks[0] * spec;
                    const float tg = L.kd[1] * r.m_d_g * dot(r.nrm, lv) + L.ks[1] * m.ks[1] * spec;
                    const float tr = L.kd[2] * r.m_d_r * dot(r.nrm, lv) + L.ks[2] * m.ks[2] * spec;
                    // w: the owning path on its first shadow ray, -1 on the others
                    sq.contrib[k] = make_float4(T.x * tb, T.y * tg, T.z * tr, __int_as_float(k == sl.shadow ? pid : -1));
                    ++k;
                }
            }
        }
    }
    if (__lane_id() == 0 && refr_w && level + 1 < kMaxLevels) atomicAdd(&fc->refract[level + 1], refr_w);
    PGRT_STAMP_END(s.stamps);
}

// lit shadow terms of one bounce, added to the path accumulators in light order
__global__ __launch_bounds__(kPathBlock) void k_path_resolve(SceneView s, int level, ShadowQueue sq, PathState ps,
                                                             const FrameCounters* fc) {
    PGRT_STAMP_BEGIN(s.stamps);
    const int n = min(fc_shadow(*fc, level), sq.cap);
    for (int k = blockIdx.x * kPathBlock + threadIdx.x; k < n; k += gridDim.x * kPathBlock) {
        const float4 c0 = sq.contrib[k];
        const int pid = __float_as_int(c0.w);
        if (pid < 0) continue;  // not the path's first shadow ray
        float4 acc = ps.acc[pid];
        for (int j = k; j < n; ++j) {
            const float4 c = j == k ? c0 : sq.contrib[j];
            if (j > k && __float_as_int(c.w) != -1) break;
            const int prim = __float_as_int(sq.hit[j].w);
            if (prim < 0 || *at_bytes(s.prim_glass, (unsigned)prim) != 0) {  // no occluder, or a dielectric one
                acc.x = acc.x + c.x;
                acc.y = acc.y + c.y;
                acc.z = acc.z + c.z;
            }
        }
        ps.acc[pid] = acc;
    }
    PGRT_STAMP_END(s.stamps);
}

void launch_path_shade(const SceneView& s_in, const FrameParams& fp, int width, const int4* tiles, int level, Queue q,
                       Queue next, const PathState& ps, ShadowQueue sq, FrameCounters* fc, int max_count, int expect,
                       hipStream_t stream) {
    if (max_count <= 0) return;
    const int ex = expect > 0 && expect < max_count ? expect : max_count;
    const int grid = std::max(1, std::min(4096, ceil_div(ex, kPathBlock)));
    SceneView s = s_in;
    s.stamps = stamp_next(kStampPathShade, level, grid, kPathBlock);
    if (s.nmat <= kLdsMats && s.ntex <= kLdsTex)
        hipLaunchKernelGGL((k_path_shade<true>), dim3(grid), dim3(kPathBlock), 0, stream, s, fp, width, tiles, level,
                           q, next, ps, sq, fc);
    else
        hipLaunchKernelGGL((k_path_shade<false>), dim3(grid), dim3(kPathBlock), 0, stream, s, fp, width, tiles, level,
                           q, next, ps, sq, fc);
}

void launch_path_resolve(const SceneView& s_in, int level, ShadowQueue sq, const PathState& ps, const FrameCounters* fc,
                         int max_count, int expect, hipStream_t stream) {
    if (max_count <= 0) return;
    const int ex = expect > 0 && expect < max_count ? expect : max_count;
    const int grid = std::max(1, std::min(4096, ceil_div(ex, kPathBlock)));
    SceneView s = s_in;
    s.stamps = stamp_next(kStampPathResolve, level, grid, kPathBlock);
    hipLaunchKernelGGL(k_path_resolve, dim3(grid), dim3(kPathBlock), 0, stream, s, level, sq, ps, fc);
}

}  // namespace pgrt
