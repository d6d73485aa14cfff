// bvh.hip -- on-device LBVH build (replaces Embree's rtcCommitScene BVH build,
// APP/raytracer.cpp:127).
//
//   1. triangle centroids -> scene/centroid bounds (block reduction + order-preserving int atomics)
//   2. 63-bit Morton codes (21 bits per axis)
//   3. radix sort of (code, triangle) pairs (hipcub / rocPRIM onesweep)
//   4. Karras 2012 hierarchy: one thread per internal node finds its range and split; equal
//      codes are split by index (delta = 64 + clz(i ^ j)); subtrees of <= kLeafMaxTris
//      triangles become leaves (a contiguous range of the sorted triangle array)
//   5. bottom-up refit with one arrival counter per node: the second child to arrive unions
//      both child boxes (agent-scope release before the counter, acquire after it, so the
//      sibling's box is read past this CU's L1 on any XCD)
//   6. triangles gathered into sorted order as {v0 | original id, e1 = v0 - v1, e2 = v2 - v0}
// Boxes are padded by `pad` world units so the traversal's slab test stays conservative.
#include <hipcub/hipcub.hpp>

#include "trace.hpp"
#include "shade_ops.hpp"

namespace pgrt {

namespace {

constexpr int kB = 256;

__device__ __forceinline__ int f2ord(float f) {
    int i = __float_as_int(f);
    return i >= 0 ? i : i ^ 0x7fffffff;
}
__device__ __forceinline__ float ord2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }

// bounds[0..2] = centroid min (ord), [3..5] = centroid max (ord)
__global__ __launch_bounds__(kB) void k_centroid_bounds(const float* __restrict__ pos, int n, int* bounds) {
    float lo[3] = {3.4e38f, 3.4e38f, 3.4e38f}, hi[3] = {-3.4e38f, -3.4e38f, -3.4e38f};
    for (int i = blockIdx.x * kB + threadIdx.x; i < n; i += gridDim.x * kB) {
        const float* p = pos + 9 * (size_t)i;
        for (int k = 0; k < 3; ++k) {
            const float mn = fminf(fminf(p[k], p[3 + k]), p[6 + k]);
            const float mx = fmaxf(fmaxf(p[k], p[3 + k]), p[6 + k]);
            const float c = 0.5f * (mn + mx);
            lo[k] = fminf(lo[k], c);
            hi[k] = fmaxf(hi[k], c);
        }
    }
    for (int k = 0; k < 3; ++k) {
        for (int off = 32; off > 0; off >>= 1) {
            lo[k] = fminf(lo[k], __shfl_xor(lo[k], off, 64));
            hi[k] = fmaxf(hi[k], __shfl_xor(hi[k], off, 64));
        }
    }
    if (__lane_id() == 0) {
        for (int k = 0; k < 3; ++k) {
            atomicMin(&bounds[k], f2ord(lo[k]));
            atomicMax(&bounds[3 + k], f2ord(hi[k]));
        }
    }
}

__device__ __forceinline__ unsigned long long spread3(unsigned int a) {
    unsigned long long x = a & 0x1fffffu;
    x = (x | x << 32) & 0x1f00000000ffffull;
    x = (x | x << 16) & 0x1f0000ff0000ffull;
    x = (x | x << 8) & 0x100f00f00f00f00full;
    x = (x | x << 4) & 0x10c30c30c30c30c3ull;
    x = (x | x << 2) & 0x1249249249249249ull;
    return x;
}

__global__ __launch_bounds__(kB) void k_morton(const float* __restrict__ pos, int n, const int* __restrict__ bounds,
                                               unsigned long long* __restrict__ keys, int* __restrict__ vals) {
    const int i = blockIdx.x * kB + threadIdx.x;
    if (i >= n) return;
    const float* p = pos + 9 * (size_t)i;
    unsigned int q[3];
    for (int k = 0; k < 3; ++k) {
        const float mn = fminf(fminf(p[k], p[3 + k]), p[6 + k]);
        const float mx = fmaxf(fmaxf(p[k], p[3 + k]), p[6 + k]);
        const float c = 0.5f * (mn + mx);
        const float lo = ord2f(bounds[k]), hi = ord2f(bounds[3 + k]);
        const float ext = hi - lo;
        float f = ext > 0 ? (c - lo) / ext : 0.5f;
        f = fminf(fmaxf(f, 0.0f), 1.0f);
        unsigned int v = (unsigned int)(f * 2097152.0f);
        q[k] = v > 2097151u ? 2097151u : v;
    }
    keys[i] = (spread3(q[0]) << 2) | (spread3(q[1]) << 1) | spread3(q[2]);
    vals[i] = i;
}

__device__ __forceinline__ int delta(const unsigned long long* __restrict__ k, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    const unsigned long long a = k[i], b = k[j];
    if (a == b) return 64 + __clz((unsigned)(i ^ j));
    return __clzll(a ^ b);
}

// kids[2*i], kids[2*i+1]: children in combined index space (internal 0..n-2, leaf n-1+k)
__global__ __launch_bounds__(kB) void k_karras(const unsigned long long* __restrict__ k, int n, BvhNode* nodes,
                                               int* __restrict__ parent, int* __restrict__ kids, int leaf_max) {
    const int i = blockIdx.x * kB + threadIdx.x;
    if (i >= n - 1) return;
    const int d = (delta(k, n, i, i + 1) - delta(k, n, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = delta(k, n, i, i - d);
    int lmax = 2;
    while (delta(k, n, i, i + lmax * d) > dmin) lmax <<= 1;
    int l = 0;
    for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (delta(k, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = delta(k, n, i, j);
    int s = 0;
    for (int div = 2;; div <<= 1) {
        const int t = (l + div - 1) / div;
        if (delta(k, n, i, i + (s + t) * d) > dnode) s += t;
        if (t <= 1) break;
    }
    const int g = i + s * d + (d < 0 ? -1 : 0);
    const int first = i < j ? i : j, last = i < j ? j : i;
    const int left = (first == g) ? (n - 1 + g) : g;
    const int right = (last == g + 1) ? (n - 1 + g + 1) : g + 1;
    kids[2 * i] = left;
    kids[2 * i + 1] = right;
    parent[left] = i;
    parent[right] = i;
    const int cl = g - first + 1, cr = last - g;
    int4 dd;
    dd.x = cl <= leaf_max ? leaf_encode(first, cl) : g;
    dd.y = cr <= leaf_max ? leaf_encode(g + 1, cr) : g + 1;
    dd.z = first;
    dd.w = last;
    nodes[i].d = dd;
}

__global__ __launch_bounds__(kB) void k_gather_tris(const float* __restrict__ pos, const int* __restrict__ order,
                                                    int n, float4* __restrict__ tri) {
    const int k = blockIdx.x * kB + threadIdx.x;
    if (k >= n) return;
    const int o = order[k];
    const float* p = pos + 9 * (size_t)o;
    const float v0x = p[0], v0y = p[1], v0z = p[2];
    tri[3 * k] = make_float4(v0x, v0y, v0z, __int_as_float(o));
    tri[3 * k + 1] = make_float4(v0x - p[3], v0y - p[4], v0z - p[5], 0.0f);  // e1 = v0 - v1
    tri[3 * k + 2] = make_float4(p[6] - v0x, p[7] - v0y, p[8] - v0z, 0.0f);  // e2 = v2 - v0
}

__device__ __forceinline__ void write_slot(BvhNode* nd, int slot, const float* lo, const float* hi) {
    if (slot == 0) {
        nd->a = make_float4(lo[0], hi[0], lo[1], hi[1]);
        nd->c.x = lo[2];
        nd->c.y = hi[2];
    } else {
        nd->b = make_float4(lo[0], hi[0], lo[1], hi[1]);
        nd->c.z = lo[2];
        nd->c.w = hi[2];
    }
}

__global__ __launch_bounds__(kB) void k_refit(const float* __restrict__ pos, const int* __restrict__ order, int n,
                                              float pad, BvhNode* nodes, const int* __restrict__ parent,
                                              const int* __restrict__ kids, int* flags) {
    const int k = blockIdx.x * kB + threadIdx.x;
    if (k >= n) return;
    const float* p = pos + 9 * (size_t)order[k];
    float lo[3], hi[3];
    for (int c = 0; c < 3; ++c) {
        lo[c] = fminf(fminf(p[c], p[3 + c]), p[6 + c]) - pad;
        hi[c] = fmaxf(fmaxf(p[c], p[3 + c]), p[6 + c]) + pad;
    }
    int cur = n - 1 + k;
    for (;;) {
        const int par = parent[cur];
        if (par < 0) break;
        const int slot = (kids[2 * par] == cur) ? 0 : 1;
        write_slot(&nodes[par], slot, lo, hi);
        __threadfence();  // release this box to whichever CU/XCD finishes the parent
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int old = atomicAdd(&flags[par], 1);
        if (old == 0) break;  // sibling not done yet: it will continue upward
        __threadfence();  // acquire: drop stale L1 lines before reading the sibling's box
        const float4 a = nodes[par].a;
        const float4 b = nodes[par].b;
        const float4 c = nodes[par].c;
        lo[0] = fminf(a.x, b.x);
        hi[0] = fmaxf(a.y, b.y);
        lo[1] = fminf(a.z, b.z);
        hi[1] = fmaxf(a.w, b.w);
        lo[2] = fminf(c.x, c.z);
        hi[2] = fmaxf(c.y, c.w);
        cur = par;
    }
}

__global__ __launch_bounds__(kB) void k_depth(int n, const int* __restrict__ parent, int* max_depth) {
    const int k = blockIdx.x * kB + threadIdx.x;
    if (k >= n) return;
    int cur = n - 1 + k, depth = 0;
    while (parent[cur] >= 0) {
        cur = parent[cur];
        ++depth;
    }
    atomicMax(max_depth, depth);
}

__global__ void k_tri_normals(const float4* __restrict__ tri, int m, float4* __restrict__ ng) {
    const int k = blockIdx.x * kB + threadIdx.x;
    if (k < m) ng[k] = tri_normal(tri[3 * k + 1], tri[3 * k + 2]);
}

}  // namespace

void compute_tri_normals(const float4* tri, int m, float4* ng, hipStream_t stream) {
    if (m <= 0) return;
    hipLaunchKernelGGL(k_tri_normals, dim3(ceil_div(m, kB)), dim3(kB), 0, stream, tri, m, ng);
    PGRT_HIP(hipGetLastError());
}

size_t lbvh_sort_temp_bytes(int ntri) {
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                       (int*)nullptr, (int*)nullptr, ntri, 0, 63);
    return bytes;
}

// scratch ints: keys (2 x 2n ints as u64), vals 2n, parent 2n, kids 2n, flags n, bounds 8, depth 1
size_t lbvh_scratch_ints(int ntri) { return (size_t)ntri * 4 + (size_t)ntri * 2 + (size_t)ntri * 2 * 3 + ntri + 64; }

void build_lbvh(const float* pos, int n, float4* tri, BvhNode* nodes, int* scratch, void* sort_tmp,
                size_t sort_tmp_bytes, float pad, BuildOut* out, hipStream_t stream) {
    PGRT_REQUIRE(n > 0, PGRT_ERR_INVALID_ARGUMENT, "empty scene");
    unsigned long long* keys_a = reinterpret_cast<unsigned long long*>(scratch);
    unsigned long long* keys_b = keys_a + n;
    int* vals_a = scratch + 4 * (size_t)n;
    int* vals_b = vals_a + n;
    int* parent = vals_b + n;           // 2n
    int* kids = parent + 2 * (size_t)n;  // 2n
    int* flags = kids + 2 * (size_t)n;   // n
    int* bounds = flags + n;             // 8
    int* depth = bounds + 8;             // 1
    const int hb[8] = {0x7fffffff, 0x7fffffff, 0x7fffffff, (int)0x80000000, (int)0x80000000, (int)0x80000000, 0, 0};
    PGRT_HIP(hipMemcpyAsync(bounds, hb, sizeof(hb), hipMemcpyHostToDevice, stream));
    PGRT_HIP(hipMemsetAsync(parent, 0xff, sizeof(int) * 2 * (size_t)n, stream));
    PGRT_HIP(hipMemsetAsync(flags, 0, sizeof(int) * (size_t)n, stream));
    PGRT_HIP(hipMemsetAsync(depth, 0, sizeof(int), stream));
    int grid = ceil_div(n, kB);
    hipLaunchKernelGGL(k_centroid_bounds, dim3(grid > 2048 ? 2048 : grid), dim3(kB), 0, stream, pos, n, bounds);
    hipLaunchKernelGGL(k_morton, dim3(grid), dim3(kB), 0, stream, pos, n, bounds, keys_a, vals_a);
    size_t tb = sort_tmp_bytes;
    PGRT_HIP(hipcub::DeviceRadixSort::SortPairs(sort_tmp, tb, keys_a, keys_b, vals_a, vals_b, n, 0, 63, stream));
    hipLaunchKernelGGL(k_gather_tris, dim3(grid), dim3(kB), 0, stream, pos, vals_b, n, tri);
    if (n >= 2) {
        hipLaunchKernelGGL(k_karras, dim3(ceil_div(n - 1, kB)), dim3(kB), 0, stream, keys_b, n, nodes, parent, kids,
                           out->leaf_max);
        hipLaunchKernelGGL(k_refit, dim3(grid), dim3(kB), 0, stream, pos, vals_b, n, pad, nodes, parent, kids, flags);
        hipLaunchKernelGGL(k_depth, dim3(grid), dim3(kB), 0, stream, n, parent, depth);
    }
    PGRT_HIP(hipGetLastError());
    int md = 0;
    PGRT_HIP(hipMemcpyAsync(&md, depth, sizeof(int), hipMemcpyDeviceToHost, stream));
    PGRT_HIP(hipStreamSynchronize(stream));
    out->root = (n >= 2) ? 0 : leaf_encode(0, 1);
    out->num_nodes = n >= 2 ? n - 1 : 0;
    out->max_depth = md;
    out->refs = n;
}

}  // namespace pgrt
