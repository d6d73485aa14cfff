// ploc.hip -- on-device BVH2 built by Parallel Locally-Ordered Clustering (Meister & Bittner,
// "Parallel Locally-Ordered Clustering for Bounding Volume Hierarchy Construction", TVCG 2018)
// over the LBVH's Morton order, then an SAH leaf collapse.
//
// Why: the plain Karras LBVH splits on Morton bits, so large triangles (the glass canopy) end
// up in boxes that overlap everything near them; secondary rays bouncing inside the canopy
// then visit ~200 nodes and every Whitted level waits for its slowest ray.  PLOC merges the
// mutually nearest clusters (smallest union surface area within a +-kRadius window of the
// Morton-sorted list) bottom up, which gives SAH-grade trees while staying fully parallel.
//
// Per iteration (host loop, one 16-byte readback): nearest neighbour (LDS window), merge
// flags, one 64-bit exclusive scan (merges << 32 | survivors), compaction that also writes the
// new internal nodes.  Then: bottom-up counts + SAH cost with per-node arrival counters
// (agent-scope release/acquire as in the LBVH refit), leaf ranges by walking to the root,
// and the 64-byte BvhNode layout with leaves of <= leaf_max (<= kLeafMaxTris) contiguous
// triangles.
#include <hipcub/hipcub.hpp>

#include "trace.hpp"

namespace pgrt {

namespace {

constexpr int kB = 256;
constexpr int kMaxRadius = 64;     // LDS window bound; the search radius is a runtime knob
constexpr int kDefaultRadius = 16;
constexpr float kDefaultCostTri = 1.0f;  // SAH: one triangle test relative to one node step

__device__ __forceinline__ float half_area(float4 lo, float4 hi) {
    const float dx = hi.x - lo.x, dy = hi.y - lo.y, dz = hi.z - lo.z;
    return dx * dy + dy * dz + dz * dx;
}

// leaves = references (padded boxes; rlo.w = triangle id bits) in Morton order
__global__ __launch_bounds__(kB) void k_ploc_init(const float4* __restrict__ rlo, const float4* __restrict__ rhi,
                                                  const int* __restrict__ order, int n, float4* nlo, float4* nhi,
                                                  int* cl_node, float4* cl_lo, float4* cl_hi, int* parent) {
    const int i = blockIdx.x * kB + threadIdx.x;
    if (i >= n) return;
    const int r = order[i];
    float4 lo = rlo[r], hi = rhi[r];
    lo.w = hi.w = 0.0f;
    nlo[i] = lo;
    nhi[i] = hi;
    cl_node[i] = i;
    cl_lo[i] = lo;
    cl_hi[i] = hi;
    parent[i] = -1;
}

__global__ __launch_bounds__(kB) void k_ploc_nn(int m, const float4* __restrict__ cl_lo,
                                                const float4* __restrict__ cl_hi, int* __restrict__ nn, int kRadius) {
    __shared__ float4 slo[kB + 2 * kMaxRadius], shi[kB + 2 * kMaxRadius];
    const int b0 = blockIdx.x * kB;
    for (int k = threadIdx.x; k < kB + 2 * kRadius; k += kB) {
        const int j = b0 - kRadius + k;
        if (j >= 0 && j < m) {
            slo[k] = cl_lo[j];
            shi[k] = cl_hi[j];
        }
    }
    __syncthreads();
    const int i = b0 + threadIdx.x;
    if (i >= m) return;
    const int li = threadIdx.x + kRadius;
    const float4 lo = slo[li], hi = shi[li];
    float best = 3.4e38f;
    int bj = -1;
    const int j0 = max(0, i - kRadius), j1 = min(m - 1, i + kRadius);
    for (int j = j0; j <= j1; ++j) {  // ascending j: strict < keeps the smallest j on ties
        if (j == i) continue;
        const float4 ol = slo[j - b0 + kRadius], oh = shi[j - b0 + kRadius];
        const float4 ul = make_float4(fminf(lo.x, ol.x), fminf(lo.y, ol.y), fminf(lo.z, ol.z), 0.0f);
        const float4 uh = make_float4(fmaxf(hi.x, oh.x), fmaxf(hi.y, oh.y), fmaxf(hi.z, oh.z), 0.0f);
        const float c = half_area(ul, uh);
        if (c < best) {
            best = c;
            bj = j;
        }
    }
    nn[i] = bj;
}

__global__ __launch_bounds__(kB) void k_ploc_flags(int m, const int* __restrict__ nn,
                                                   unsigned long long* __restrict__ packed) {
    const int i = blockIdx.x * kB + threadIdx.x;
    if (i >= m) return;
    const int j = nn[i];
    const bool mutual = j >= 0 && nn[j] == i;
    const unsigned long long create = (mutual && i < j) ? 1ull : 0ull;
    const unsigned long long valid = (mutual && i > j) ? 0ull : 1ull;
    packed[i] = (create << 32) | valid;
}

__global__ __launch_bounds__(kB) void k_ploc_compact(int m, const int* __restrict__ nn,
                                                     const unsigned long long* __restrict__ packed,
                                                     const unsigned long long* __restrict__ scanned,
                                                     const int* __restrict__ cl_node, const float4* __restrict__ cl_lo,
                                                     const float4* __restrict__ cl_hi, int* __restrict__ out_node,
                                                     float4* __restrict__ out_lo, float4* __restrict__ out_hi,
                                                     int node_base, float4* nlo, float4* nhi, int2* kids,
                                                     int* parent) {
    const int i = blockIdx.x * kB + threadIdx.x;
    if (i >= m) return;
    const unsigned long long p = packed[i];
    if (!(p & 1ull)) return;
    const unsigned long long s = scanned[i];
    const int pos = (int)(s & 0xffffffffull);
    if (p >> 32) {
        const int id = node_base + (int)(s >> 32);
        const int j = nn[i];
        const int a = cl_node[i], b = cl_node[j];
        const float4 la = cl_lo[i], ha = cl_hi[i], lb = cl_lo[j], hb = cl_hi[j];
        const float4 lo = make_float4(fminf(la.x, lb.x), fminf(la.y, lb.y), fminf(la.z, lb.z), 0.0f);
        const float4 hi = make_float4(fmaxf(ha.x, hb.x), fmaxf(ha.y, hb.y), fmaxf(ha.z, hb.z), 0.0f);
        nlo[id] = lo;
        nhi[id] = hi;
        kids[id] = make_int2(a, b);
        parent[a] = id;
        parent[b] = id;
        parent[id] = -1;
        out_node[pos] = id;
        out_lo[pos] = lo;
        out_hi[pos] = hi;
    } else {
        out_node[pos] = cl_node[i];
        out_lo[pos] = cl_lo[i];
        out_hi[pos] = cl_hi[i];
    }
}

// bottom-up triangle counts and SAH cost; collapse[p] = subtree becomes one leaf
__global__ __launch_bounds__(kB) void k_ploc_cost(int n, const float4* __restrict__ nlo,
                                                  const float4* __restrict__ nhi, const int2* __restrict__ kids,
                                                  const int* __restrict__ parent, int* count, float* cost,
                                                  int* collapse, int* flags, int leaf_max, float kCostTri) {
    constexpr float kCostNode = 1.0f;
    const int i = blockIdx.x * kB + threadIdx.x;
    if (i >= n) return;
    count[i] = 1;
    cost[i] = kCostTri * half_area(nlo[i], nhi[i]);
    int cur = i;
    for (;;) {
        const int par = parent[cur];
        if (par < 0) break;
        __threadfence();  // release this subtree's count/cost
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (atomicAdd(&flags[par], 1) == 0) break;  // sibling still running
        __threadfence();  // acquire the sibling's values
        const int2 k = kids[par];
        const int c = count[k.x] + count[k.y];
        const float a = half_area(nlo[par], nhi[par]);
        const float node_cost = kCostNode * a + cost[k.x] + cost[k.y];
        const float leaf_cost = kCostTri * a * (float)c;
        const bool leaf = c <= leaf_max && leaf_cost <= node_cost;
        count[par] = c;
        cost[par] = leaf ? leaf_cost : node_cost;
        collapse[par] = leaf ? 1 : 0;
        cur = par;
    }
}

// first sorted-triangle slot of every node's subtree (leaves in left-to-right order) and depth
__global__ __launch_bounds__(kB) void k_ploc_offsets(int total, const int2* __restrict__ kids,
                                                     const int* __restrict__ parent, const int* __restrict__ count,
                                                     int* offset, int* max_depth) {
    const int v = blockIdx.x * kB + threadIdx.x;
    if (v >= total) return;
    int off = 0, depth = 0, cur = v;
    for (int par = parent[cur]; par >= 0; cur = par, par = parent[cur]) {
        const int2 k = kids[par];
        if (k.y == cur) off += count[k.x];
        ++depth;
    }
    offset[v] = off;
    atomicMax(max_depth, depth);
}

__device__ __forceinline__ int encode_child(int c, int n, const int* count, const int* offset, const int* collapse) {
    if (c < n) return leaf_encode(offset[c], 1);
    if (collapse[c]) return leaf_encode(offset[c], count[c]);
    return c - n;
}

__global__ __launch_bounds__(kB) void k_ploc_write(int n, const float4* __restrict__ nlo,
                                                   const float4* __restrict__ nhi, const int2* __restrict__ kids,
                                                   const int* __restrict__ count, const int* __restrict__ offset,
                                                   const int* __restrict__ collapse, BvhNode* __restrict__ out) {
    const int q = blockIdx.x * kB + threadIdx.x;  // output node q = internal node n + q
    if (q >= n - 1) return;
    const int id = n + q;
    const int2 k = kids[id];
    const float4 l0 = nlo[k.x], h0 = nhi[k.x], l1 = nlo[k.y], h1 = nhi[k.y];
    BvhNode nd;
    nd.a = make_float4(l0.x, h0.x, l0.y, h0.y);
    nd.b = make_float4(l1.x, h1.x, l1.y, h1.y);
    nd.c = make_float4(l0.z, h0.z, l1.z, h1.z);
    nd.d = make_int4(encode_child(k.x, n, count, offset, collapse), encode_child(k.y, n, count, offset, collapse),
                     offset[id], count[id]);
    out[q] = nd;
}

__global__ __launch_bounds__(kB) void k_ploc_tris(const float* __restrict__ pos, const float4* __restrict__ rlo,
                                                  const int* __restrict__ order, const int* __restrict__ offset, int n,
                                                  float4* __restrict__ tri) {
    const int i = blockIdx.x * kB + threadIdx.x;
    if (i >= n) return;
    const int o = __float_as_int(rlo[order[i]].w);  // triangle of this reference
    const int k = offset[i];
    const float* p = pos + 9 * (size_t)o;
    const float v0x = p[0], v0y = p[1], v0z = p[2];
    tri[3 * k] = make_float4(v0x, v0y, v0z, __int_as_float(o));
    tri[3 * k + 1] = make_float4(v0x - p[3], v0y - p[4], v0z - p[5], 0.0f);  // e1 = v0 - v1
    tri[3 * k + 2] = make_float4(p[6] - v0x, p[7] - v0y, p[8] - v0z, 0.0f);  // e2 = v2 - v0
}

}  // namespace

// order: reference indices in Morton order (device); n references; builds nodes/tri like
// build_lbvh (one 48-B triangle record per reference, in leaf order).
void build_ploc(const float* pos, const float4* rlo, const float4* rhi, const int* order, int n, float4* tri,
                BvhNode* nodes, BuildOut* out, int* iterations, hipStream_t stream) {
    const int total = 2 * n - 1;
    // r1g A/B (profiles/r1g/c5_bvh_knobs_ab.txt): radius 8..32 and triangle cost 0.5..2 within 2 %
    const int radius = kDefaultRadius;
    const float cost_tri = kDefaultCostTri;
    DevBuf<float4> nlo, nhi, cl_lo[2], cl_hi[2];
    DevBuf<int2> kids;
    DevBuf<int> parent, cl_node[2], nn, count, collapse, flags, offset, misc;
    DevBuf<float> cost;
    DevBuf<unsigned long long> packed, scanned;
    nlo.alloc(total);
    nhi.alloc(total);
    kids.alloc(total);
    parent.alloc(total);
    for (int b = 0; b < 2; ++b) {
        cl_lo[b].alloc(n);
        cl_hi[b].alloc(n);
        cl_node[b].alloc(n);
    }
    nn.alloc(n);
    packed.alloc(n);
    scanned.alloc(n);
    size_t scan_bytes = 0;
    PGRT_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, packed.p, scanned.p, n, stream));
    DevBuf<unsigned char> scan_tmp;
    scan_tmp.alloc(scan_bytes);
    misc.alloc(4);
    const int grid = ceil_div(n, kB);
    hipLaunchKernelGGL(k_ploc_init, dim3(grid), dim3(kB), 0, stream, rlo, rhi, order, n, nlo.p, nhi.p, cl_node[0].p,
                       cl_lo[0].p, cl_hi[0].p, parent.p);
    int m = n, node_base = n, cur = 0, iters = 0;
    unsigned long long tail[2];
    while (m > 1) {
        const int g = ceil_div(m, kB);
        hipLaunchKernelGGL(k_ploc_nn, dim3(g), dim3(kB), 0, stream, m, cl_lo[cur].p, cl_hi[cur].p, nn.p, radius);
        hipLaunchKernelGGL(k_ploc_flags, dim3(g), dim3(kB), 0, stream, m, nn.p, packed.p);
        size_t sb = scan_bytes;
        PGRT_HIP(hipcub::DeviceScan::ExclusiveSum(scan_tmp.p, sb, packed.p, scanned.p, m, stream));
        hipLaunchKernelGGL(k_ploc_compact, dim3(g), dim3(kB), 0, stream, m, nn.p, packed.p, scanned.p,
                           cl_node[cur].p, cl_lo[cur].p, cl_hi[cur].p, cl_node[cur ^ 1].p, cl_lo[cur ^ 1].p,
                           cl_hi[cur ^ 1].p, node_base, nlo.p, nhi.p, kids.p, parent.p);
        PGRT_HIP(hipMemcpyAsync(&tail[0], packed.p + (m - 1), 8, hipMemcpyDeviceToHost, stream));
        PGRT_HIP(hipMemcpyAsync(&tail[1], scanned.p + (m - 1), 8, hipMemcpyDeviceToHost, stream));
        PGRT_HIP(hipStreamSynchronize(stream));
        const int new_m = (int)(tail[1] & 0xffffffffull) + (int)(tail[0] & 1ull);
        const int created = (int)(tail[1] >> 32) + (int)(tail[0] >> 32);
        PGRT_REQUIRE(created > 0, PGRT_ERR_HIP, "PLOC made no progress");
        node_base += created;
        m = new_m;
        cur ^= 1;
        ++iters;
    }
    PGRT_REQUIRE(node_base == total, PGRT_ERR_HIP, "PLOC node count mismatch");
    count.alloc(total);
    cost.alloc(total);
    collapse.alloc(total);
    flags.alloc(total);
    offset.alloc(total);
    PGRT_HIP(hipMemsetAsync(collapse.p, 0, sizeof(int) * total, stream));
    PGRT_HIP(hipMemsetAsync(flags.p, 0, sizeof(int) * total, stream));
    PGRT_HIP(hipMemsetAsync(misc.p, 0, sizeof(int) * 4, stream));
    hipLaunchKernelGGL(k_ploc_cost, dim3(grid), dim3(kB), 0, stream, n, nlo.p, nhi.p, kids.p, parent.p, count.p,
                       cost.p, collapse.p, flags.p, out->leaf_max, cost_tri);
    hipLaunchKernelGGL(k_ploc_offsets, dim3(ceil_div(total, kB)), dim3(kB), 0, stream, total, kids.p, parent.p,
                       count.p, offset.p, misc.p);
    if (n >= 2)
        hipLaunchKernelGGL(k_ploc_write, dim3(ceil_div(n - 1, kB)), dim3(kB), 0, stream, n, nlo.p, nhi.p, kids.p,
                           count.p, offset.p, collapse.p, nodes);
    hipLaunchKernelGGL(k_ploc_tris, dim3(grid), dim3(kB), 0, stream, pos, rlo, order, offset.p, n, tri);
    PGRT_HIP(hipGetLastError());
    int root_collapse = 0, root_count = 1, md = 0;
    const int root = total - 1;
    if (n >= 2) {
        PGRT_HIP(hipMemcpyAsync(&root_collapse, collapse.p + root, sizeof(int), hipMemcpyDeviceToHost, stream));
        PGRT_HIP(hipMemcpyAsync(&root_count, count.p + root, sizeof(int), hipMemcpyDeviceToHost, stream));
    }
    PGRT_HIP(hipMemcpyAsync(&md, misc.p, sizeof(int), hipMemcpyDeviceToHost, stream));
    PGRT_HIP(hipStreamSynchronize(stream));
    if (n == 1) out->root = leaf_encode(0, 1);
    else if (root_collapse) out->root = leaf_encode(0, root_count);
    else out->root = root - n;
    out->num_nodes = n >= 2 ? n - 1 : 0;
    out->max_depth = md;
    if (iterations) *iterations = iters;
}

}  // namespace pgrt
