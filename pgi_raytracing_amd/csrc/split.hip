// split.hip -- BVH primitive references with budgeted early split clipping, and the PLOC build
// driver over them.
//
// A long or diagonal triangle has an AABB far larger than the triangle (the avenger proxy's
// glass antenna rods: 95-unit slivers; stud cap fans; canopy facets).  Its box overlaps
// everything around it, so rays near it descend into subtrees they never hit; the deep
// Whitted levels (rays bouncing inside glass) are bound by exactly those rays.  Following Ernst
// & Greiner ("Early Split Clipping for Bounding Volume Hierarchies", 2007) with the global
// split budget of Karras & Aila ("Fast Parallel Construction of High-Quality Bounding Volume
// Hierarchies", HPG 2013, §4), every triangle becomes 1..kMaxRefs references, each with the
// tight box of the triangle clipped to one cell of a recursive longest-axis midpoint split.
//
//   1. waste_i = half_area(AABB_i) - A_i (|nx| + |ny| + |nz|)   (the AABB area that finer
//      splitting can remove: a planar piece's box tends to its three axis projections).
//      Greedy marginal gain waste/k^2 -> k_i proportional to sqrt(waste_i).
//   2. q_i = sqrt(waste_i) / scene extent in 32.32 fixed point, summed with integer atomics
//      (order independent -> the build is deterministic); extra_i = floor(beta n q_i / sum q).
//   3. exclusive scan of 1 + extra_i -> reference slots.
//   4. per triangle: split the current tight box at the midpoint of its longest axis, clip
//      the ORIGINAL triangle to each half (Sutherland-Hodgman, <= 9 vertices) and recurse
//      with the counts halved; every leaf cell emits one reference (padded box, triangle id).
//      The cells' union covers the triangle, so the closest hit is unchanged; a triangle may
//      be tested twice along one ray, which gives the same (t, prim) and the same tie-break.
//   5. Morton codes of the reference centroids, radix sort, PLOC (ploc.hip) over references.
#include <hipcub/hipcub.hpp>

#include "trace.hpp"

namespace pgrt {

namespace {

constexpr int kB = 256;
constexpr int kMaxRefs = 32;  // per triangle (power of two: the halving recursion is <= 5 deep)

__device__ __forceinline__ int f2ord(float f) {
    int i = __float_as_int(f);
    return i >= 0 ? i : i ^ 0x7fffffff;
}
__device__ __forceinline__ float ord2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }

__device__ __forceinline__ unsigned long long spread3(unsigned int a) {
    unsigned long long x = a & 0x1fffffu;
    x = (x | x << 32) & 0x1f00000000ffffull;
    x = (x | x << 16) & 0x1f0000ff0000ffull;
    x = (x | x << 8) & 0x100f00f00f00f00full;
    x = (x | x << 4) & 0x10c30c30c30c30c3ull;
    x = (x | x << 2) & 0x1249249249249249ull;
    return x;
}

struct Box3 {
    float lo[3], hi[3];
};

__device__ __forceinline__ float half_area3(const Box3& b) {
    const float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
    return dx * dy + dy * dz + dz * dx;
}

__device__ __forceinline__ Box3 tri_box(const float* p) {
    Box3 b;
    for (int k = 0; k < 3; ++k) {
        b.lo[k] = fminf(fminf(p[k], p[3 + k]), p[6 + k]);
        b.hi[k] = fmaxf(fmaxf(p[k], p[3 + k]), p[6 + k]);
    }
    return b;
}

// bounds of triangle p ∩ box c (Sutherland-Hodgman against the 6 planes); false if empty
__device__ bool clip_bounds(const float* p, const Box3& c, Box3& out) {
    float poly[10][3], tmp[10][3];
    int np = 3;
    for (int v = 0; v < 3; ++v)
        for (int k = 0; k < 3; ++k) poly[v][k] = p[3 * v + k];
    for (int pl = 0; pl < 6; ++pl) {
        const int a = pl >> 1;
        const float val = (pl & 1) ? c.hi[a] : c.lo[a];
        const float side = (pl & 1) ? -1.0f : 1.0f;  // keep side * (x - val) >= 0
        int no = 0;
        for (int k = 0; k < np; ++k) {
            const float* P = poly[k];
            const float* Q = poly[k + 1 == np ? 0 : k + 1];
            const float dp = side * (P[a] - val), dq = side * (Q[a] - val);
            if (dp >= 0.0f && no < 10) {
                tmp[no][0] = P[0];
                tmp[no][1] = P[1];
                tmp[no][2] = P[2];
                ++no;
            }
            if ((dp >= 0.0f) != (dq >= 0.0f) && no < 10) {
                const float t = dp / (dp - dq);
                for (int j = 0; j < 3; ++j) tmp[no][j] = P[j] + t * (Q[j] - P[j]);
                tmp[no][a] = val;  // exactly on the plane
                ++no;
            }
        }
        np = no;
        if (np == 0) return false;
        for (int k = 0; k < np; ++k)
            for (int j = 0; j < 3; ++j) poly[k][j] = tmp[k][j];
    }
    for (int j = 0; j < 3; ++j) {
        out.lo[j] = 3.4e38f;
        out.hi[j] = -3.4e38f;
    }
    for (int k = 0; k < np; ++k)
        for (int j = 0; j < 3; ++j) {
            out.lo[j] = fminf(out.lo[j], poly[k][j]);
            out.hi[j] = fmaxf(out.hi[j], poly[k][j]);
        }
    for (int j = 0; j < 3; ++j) {  // never outside the cell (rounding of the intersections)
        out.lo[j] = fmaxf(out.lo[j], c.lo[j]);
        out.hi[j] = fminf(out.hi[j], c.hi[j]);
    }
    return true;
}

__global__ __launch_bounds__(kB) void k_split_weight(const float* __restrict__ pos, int n, float inv_ext,
                                                     unsigned long long* __restrict__ q,
                                                     unsigned long long* __restrict__ total) {
    const int i = blockIdx.x * kB + threadIdx.x;
    unsigned long long v = 0;
    if (i < n) {
        const float* p = pos + 9 * (size_t)i;
        const Box3 b = tri_box(p);
        const float e1x = p[3] - p[0], e1y = p[4] - p[1], e1z = p[5] - p[2];
        const float e2x = p[6] - p[0], e2y = p[7] - p[1], e2z = p[8] - p[2];
        // |nx| + |ny| + |nz| of the unnormalised cross product = 2 A (|nx| + |ny| + |nz|)_unit
        const float nx = e1y * e2z - e1z * e2y, ny = e1z * e2x - e1x * e2z, nz = e1x * e2y - e1y * e2x;
        const float ideal = 0.5f * (fabsf(nx) + fabsf(ny) + fabsf(nz));
        const float waste = fmaxf(half_area3(b) - ideal, 0.0f);
        const float w = sqrtf(waste) * inv_ext;  // ~[0, 2]
        v = (unsigned long long)((double)w * 4294967296.0);
        if (!(w >= 0.0f) || w > 1e6f) v = 0;
        q[i] = v;
    }
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if (__lane_id() == 0 && v) atomicAdd(total, v);
}

__global__ __launch_bounds__(kB) void k_split_count(const unsigned long long* __restrict__ q, int n,
                                                    const unsigned long long* __restrict__ total, double budget,
                                                    int* __restrict__ refs) {
    const int i = blockIdx.x * kB + threadIdx.x;
    if (i >= n) return;
    const unsigned long long t = *total;
    int extra = 0;
    if (t > 0) extra = (int)floor(budget * ((double)q[i] / (double)t));
    refs[i] = 1 + min(max(extra, 0), kMaxRefs - 1);
}

__global__ __launch_bounds__(kB) void k_split_emit(const float* __restrict__ pos, int n, const int* __restrict__ refs,
                                                   const int* __restrict__ offset, float pad, float4* __restrict__ rlo,
                                                   float4* __restrict__ rhi) {
    const int i = blockIdx.x * kB + threadIdx.x;
    if (i >= n) return;
    const float* p = pos + 9 * (size_t)i;
    const float id = __int_as_float(i);
    int slot = offset[i];
    auto emit = [&](const Box3& b) {
        rlo[slot] = make_float4(b.lo[0] - pad, b.lo[1] - pad, b.lo[2] - pad, id);
        rhi[slot] = make_float4(b.hi[0] + pad, b.hi[1] + pad, b.hi[2] + pad, 0.0f);
        ++slot;
    };
    Box3 stk[8];
    int cnt[8];
    int sp = 0;
    stk[0] = tri_box(p);
    cnt[0] = refs[i];
    sp = 1;
    while (sp > 0) {
        --sp;
        const Box3 b = stk[sp];
        const int c = cnt[sp];
        int a = 0;
        float ext = b.hi[0] - b.lo[0];
        for (int k = 1; k < 3; ++k)
            if (b.hi[k] - b.lo[k] > ext) {
                ext = b.hi[k] - b.lo[k];
                a = k;
            }
        Box3 L, R;
        bool ok = c > 1 && ext > 0.0f && sp + 2 <= 8;
        if (ok) {
            const float mid = 0.5f * (b.lo[a] + b.hi[a]);
            Box3 cl = b, cr = b;
            cl.hi[a] = mid;
            cr.lo[a] = mid;
            ok = clip_bounds(p, cl, L) && clip_bounds(p, cr, R);
        }
        if (!ok) {  // degenerate cell: keep the slot count with copies of this box
            for (int k = 0; k < c; ++k) emit(b);
            continue;
        }
        const int c0 = c >> 1;
        stk[sp] = R;
        cnt[sp] = c - c0;
        stk[sp + 1] = L;
        cnt[sp + 1] = c0;
        sp += 2;
    }
}

// no splitting: one reference per triangle
__global__ __launch_bounds__(kB) void k_refs_plain(const float* __restrict__ pos, int n, float pad,
                                                   float4* __restrict__ rlo, float4* __restrict__ rhi) {
    const int i = blockIdx.x * kB + threadIdx.x;
    if (i >= n) return;
    const Box3 b = tri_box(pos + 9 * (size_t)i);
    rlo[i] = make_float4(b.lo[0] - pad, b.lo[1] - pad, b.lo[2] - pad, __int_as_float(i));
    rhi[i] = make_float4(b.hi[0] + pad, b.hi[1] + pad, b.hi[2] + pad, 0.0f);
}

__global__ __launch_bounds__(kB) void k_ref_centroid_bounds(const float4* __restrict__ rlo,
                                                            const float4* __restrict__ rhi, int m, int* bounds) {
    float lo[3] = {3.4e38f, 3.4e38f, 3.4e38f}, hi[3] = {-3.4e38f, -3.4e38f, -3.4e38f};
    for (int i = blockIdx.x * kB + threadIdx.x; i < m; i += gridDim.x * kB) {
        const float4 a = rlo[i], b = rhi[i];
        const float c[3] = {0.5f * (a.x + b.x), 0.5f * (a.y + b.y), 0.5f * (a.z + b.z)};
        for (int k = 0; k < 3; ++k) {
            lo[k] = fminf(lo[k], c[k]);
            hi[k] = fmaxf(hi[k], c[k]);
        }
    }
    for (int k = 0; k < 3; ++k)
        for (int off = 32; off > 0; off >>= 1) {
            lo[k] = fminf(lo[k], __shfl_xor(lo[k], off, 64));
            hi[k] = fmaxf(hi[k], __shfl_xor(hi[k], off, 64));
        }
    if (__lane_id() == 0)
        for (int k = 0; k < 3; ++k) {
            atomicMin(&bounds[k], f2ord(lo[k]));
            atomicMax(&bounds[3 + k], f2ord(hi[k]));
        }
}

__global__ __launch_bounds__(kB) void k_ref_morton(const float4* __restrict__ rlo, const float4* __restrict__ rhi,
                                                   int m, const int* __restrict__ bounds,
                                                   unsigned long long* __restrict__ keys, int* __restrict__ vals) {
    const int i = blockIdx.x * kB + threadIdx.x;
    if (i >= m) return;
    const float4 a = rlo[i], b = rhi[i];
    const float c[3] = {0.5f * (a.x + b.x), 0.5f * (a.y + b.y), 0.5f * (a.z + b.z)};
    unsigned int q[3];
    for (int k = 0; k < 3; ++k) {
        const float lo = ord2f(bounds[k]), hi = ord2f(bounds[3 + k]);
        const float ext = hi - lo;
        float f = ext > 0 ? (c[k] - lo) / ext : 0.5f;
        f = fminf(fmaxf(f, 0.0f), 1.0f);
        const unsigned int v = (unsigned int)(f * 2097152.0f);
        q[k] = v > 2097151u ? 2097151u : v;
    }
    keys[i] = (spread3(q[0]) << 2) | (spread3(q[1]) << 1) | spread3(q[2]);
    vals[i] = i;
}

}  // namespace

int build_ploc_refs(const float* pos, int n, float beta, float pad, float extent, DevBuf<float4>& tri,
                    DevBuf<BvhNode>& nodes, BuildOut* out, hipStream_t stream) {
    PGRT_REQUIRE(n > 0, PGRT_ERR_INVALID_ARGUMENT, "empty scene");
    const int grid = ceil_div(n, kB);
    int m = n;
    DevBuf<float4> rlo, rhi;
    if (beta > 0.0f && n >= 2) {
        DevBuf<unsigned long long> q, total;
        DevBuf<int> refs, offset;
        q.alloc(n);
        total.alloc(1);
        refs.alloc(n);
        offset.alloc(n);
        PGRT_HIP(hipMemsetAsync(total.p, 0, sizeof(unsigned long long), stream));
        hipLaunchKernelGGL(k_split_weight, dim3(grid), dim3(kB), 0, stream, pos, n, 1.0f / extent, q.p, total.p);
        hipLaunchKernelGGL(k_split_count, dim3(grid), dim3(kB), 0, stream, q.p, n, total.p, (double)beta * n, refs.p);
        size_t sb = 0;
        PGRT_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, sb, refs.p, offset.p, n, stream));
        DevBuf<unsigned char> tmp;
        tmp.alloc(sb);
        PGRT_HIP(hipcub::DeviceScan::ExclusiveSum(tmp.p, sb, refs.p, offset.p, n, stream));
        int last[2];
        PGRT_HIP(hipMemcpyAsync(&last[0], offset.p + n - 1, sizeof(int), hipMemcpyDeviceToHost, stream));
        PGRT_HIP(hipMemcpyAsync(&last[1], refs.p + n - 1, sizeof(int), hipMemcpyDeviceToHost, stream));
        PGRT_HIP(hipStreamSynchronize(stream));
        m = last[0] + last[1];
        PGRT_REQUIRE(m >= n && m < (1 << 27), PGRT_ERR_INVALID_ARGUMENT, "too many BVH references");
        rlo.alloc(m);
        rhi.alloc(m);
        hipLaunchKernelGGL(k_split_emit, dim3(grid), dim3(kB), 0, stream, pos, n, refs.p, offset.p, pad, rlo.p, rhi.p);
    } else {
        rlo.alloc(n);
        rhi.alloc(n);
        hipLaunchKernelGGL(k_refs_plain, dim3(grid), dim3(kB), 0, stream, pos, n, pad, rlo.p, rhi.p);
    }
    // Morton order of the reference centroids
    DevBuf<int> bounds, vals[2];
    DevBuf<unsigned long long> keys[2];
    bounds.alloc(8);
    for (int b = 0; b < 2; ++b) {
        vals[b].alloc(m);
        keys[b].alloc(m);
    }
    const int hb[8] = {0x7fffffff, 0x7fffffff, 0x7fffffff, (int)0x80000000, (int)0x80000000, (int)0x80000000, 0, 0};
    PGRT_HIP(hipMemcpyAsync(bounds.p, hb, sizeof(hb), hipMemcpyHostToDevice, stream));
    const int gm = ceil_div(m, kB);
    hipLaunchKernelGGL(k_ref_centroid_bounds, dim3(gm > 2048 ? 2048 : gm), dim3(kB), 0, stream, rlo.p, rhi.p, m,
                       bounds.p);
    hipLaunchKernelGGL(k_ref_morton, dim3(gm), dim3(kB), 0, stream, rlo.p, rhi.p, m, bounds.p, keys[0].p, vals[0].p);
    size_t sort_bytes = 0;
    PGRT_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, keys[0].p, keys[1].p, vals[0].p, vals[1].p, m,
                                                0, 63, stream));
    DevBuf<unsigned char> sort_tmp;
    sort_tmp.alloc(sort_bytes);
    PGRT_HIP(hipcub::DeviceRadixSort::SortPairs(sort_tmp.p, sort_bytes, keys[0].p, keys[1].p, vals[0].p, vals[1].p,
                                                m, 0, 63, stream));
    tri.alloc((size_t)m * 3);
    nodes.alloc((size_t)std::max(1, m - 1));
    build_ploc(pos, rlo.p, rhi.p, vals[1].p, m, tri.p, nodes.p, out, &out->iterations, stream);
    out->refs = m;
    return m;
}

}  // namespace pgrt
