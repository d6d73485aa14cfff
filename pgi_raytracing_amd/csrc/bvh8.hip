// bvh8.hip -- collapse of the binary BVH into an 8-wide BVH with 8-bit quantized child boxes
// (the compressed wide layout of Ylitie, Karras & Laine, "Efficient Incoherent Ray Traversal on
// GPUs Through Compressed Wide BVHs", HPG 2017), built on the device.
//
// Why: the closest-hit kernel is latency-bound on the deep Whitted levels -- a few hundred
// thousand rays spread over 1024 SIMDs, so every dependent node fetch is exposed.  An 8-wide
// node replaces about three binary levels by one 80-byte fetch, cutting both the dependent
// chain and the bytes per ray.
//
// Top-down, one launch per output level: a task is a binary subtree that becomes one wide node.
// Its candidate children start as the binary node's two children; the internal candidate with
// the largest surface area is replaced by its own two children until there are 8 (or only
// leaves).  Candidates go to slots by the octant of their centroid (slot bit k set = child lies
// on the + side of axis k), so the traversal can visit slots in an approximate front-to-back
// order from the ray's octant alone.  Internal children are stored contiguously from
// child_base in slot order; leaf triangles contiguously from tri_base.
//
// Boxes are quantized conservatively: origin = node box min, per-axis scale 2^e with
// e = ceil(log2(extent / 255)), q_lo = floor, q_hi = ceil (in double), so every decoded child
// box contains the padded binary box it came from.
#include "trace.hpp"

namespace pgrt {

namespace {

constexpr int kB = 128;

struct Cand {
    int code;  // binary child: >= 0 internal node index, < 0 leaf code
    float lo[3], hi[3];
};

__device__ __forceinline__ float half_area3(const float* lo, const float* hi) {
    const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return dx * dy + dy * dz + dz * dx;
}

__device__ __forceinline__ void node_children(const BvhNode& nd, Cand& c0, Cand& c1) {
    c0.code = nd.d.x;
    c0.lo[0] = nd.a.x; c0.hi[0] = nd.a.y; c0.lo[1] = nd.a.z; c0.hi[1] = nd.a.w;
    c0.lo[2] = nd.c.x; c0.hi[2] = nd.c.y;
    c1.code = nd.d.y;
    c1.lo[0] = nd.b.x; c1.hi[0] = nd.b.y; c1.lo[1] = nd.b.z; c1.hi[1] = nd.b.w;
    c1.lo[2] = nd.c.z; c1.hi[2] = nd.c.w;
}

// exponent e (unbiased) with extent / 2^e <= 255, clamped to the normal float range
__device__ __forceinline__ int quant_exp(double ext) {
    if (!(ext > 0.0)) return -126;
    int e;
    const double m = frexp(ext / 255.0, &e);  // ext/255 = m * 2^e, m in [0.5, 1)
    if (m == 0.5) --e;                         // exact power of two
    return e < -126 ? -126 : (e > 127 ? 127 : e);
}

// tasks: (binary ref, wide node index); counters: [0] wide nodes, [1] triangles, [2] next tasks,
// [3] max depth
__global__ __launch_bounds__(kB) void k_collapse(const BvhNode* __restrict__ bin, const float4* __restrict__ tri_in,
                                                 const int2* __restrict__ tasks, const int* __restrict__ ntask_p,
                                                 int2* __restrict__ next_tasks, int* __restrict__ counters, int depth,
                                                 float4 root_lo, float4 root_hi, Bvh8Node* __restrict__ out,
                                                 float4* __restrict__ tri_out) {
    const int t = blockIdx.x * kB + threadIdx.x;
    if (t >= *ntask_p) return;
    const int2 task = tasks[t];
    Cand c[8];
    int nc;
    if (task.x >= 0) {
        node_children(bin[task.x], c[0], c[1]);
        nc = 2;
    } else {  // the whole scene is one binary leaf
        c[0].code = task.x;
        c[0].lo[0] = root_lo.x; c[0].lo[1] = root_lo.y; c[0].lo[2] = root_lo.z;
        c[0].hi[0] = root_hi.x; c[0].hi[1] = root_hi.y; c[0].hi[2] = root_hi.z;
        nc = 1;
    }
    while (nc < 8) {  // open the largest internal candidate
        int best = -1;
        float ba = -1.0f;
        for (int k = 0; k < nc; ++k)
            if (c[k].code >= 0) {
                const float a = half_area3(c[k].lo, c[k].hi);
                if (a > ba) {
                    ba = a;
                    best = k;
                }
            }
        if (best < 0) break;
        Cand x, y;
        node_children(bin[c[best].code], x, y);
        c[best] = x;
        c[nc++] = y;
    }
    // node box and its centroid
    float lo[3] = {3.4e38f, 3.4e38f, 3.4e38f}, hi[3] = {-3.4e38f, -3.4e38f, -3.4e38f};
    for (int k = 0; k < nc; ++k)
        for (int a = 0; a < 3; ++a) {
            lo[a] = fminf(lo[a], c[k].lo[a]);
            hi[a] = fmaxf(hi[a], c[k].hi[a]);
        }
    // octant slot assignment: greedily take the (candidate, slot) pair of largest
    // dot(centroid offset, slot direction)
    int slot_of[8];
    unsigned used = 0, placed = 0;
    for (int r = 0; r < nc; ++r) {
        float bv = -3.4e38f;
        int bk = 0, bs = 0;
        for (int k = 0; k < nc; ++k) {
            if (placed & (1u << k)) continue;
            float off[3];
            for (int a = 0; a < 3; ++a) off[a] = (c[k].lo[a] + c[k].hi[a]) - (lo[a] + hi[a]);
            for (int s = 0; s < 8; ++s) {
                if (used & (1u << s)) continue;
                const float v = ((s & 1) ? off[0] : -off[0]) + ((s & 2) ? off[1] : -off[1]) +
                                ((s & 4) ? off[2] : -off[2]);
                if (v > bv) {
                    bv = v;
                    bk = k;
                    bs = s;
                }
            }
        }
        slot_of[bk] = bs;
        placed |= 1u << bk;
        used |= 1u << bs;
    }
    int at_slot[8];
    for (int s = 0; s < 8; ++s) at_slot[s] = -1;
    for (int k = 0; k < nc; ++k) at_slot[slot_of[k]] = k;
    int n_int = 0, n_tri = 0;
    for (int k = 0; k < nc; ++k) {
        if (c[k].code >= 0) ++n_int;
        else n_tri += leaf_count(c[k].code);
    }
    const int child_base = n_int ? atomicAdd(&counters[0], n_int) : 0;
    const int tri_base = n_tri ? atomicAdd(&counters[1], n_tri) : 0;
    const int task_base = n_int ? atomicAdd(&counters[2], n_int) : 0;
    if (n_int) atomicMax(&counters[3], depth + 1);
    // quantization frame
    int e[3];
    float scale[3];
    for (int a = 0; a < 3; ++a) {
        e[a] = quant_exp((double)hi[a] - (double)lo[a]);
        scale[a] = __uint_as_float((unsigned)(e[a] + 127) << 23);
    }
    unsigned char qlo[3][8], qhi[3][8], meta[8];
    unsigned imask = 0;
    int ci = 0, to = 0;
    for (int s = 0; s < 8; ++s) {
        const int k = at_slot[s];
        if (k < 0) {
            meta[s] = 0;
            for (int a = 0; a < 3; ++a) {
                qlo[a][s] = 0;
                qhi[a][s] = 0;
            }
            continue;
        }
        for (int a = 0; a < 3; ++a) {
            const double inv = 1.0 / (double)scale[a];  // exact: power of two
            double ql = floor(((double)c[k].lo[a] - (double)lo[a]) * inv);
            double qh = ceil(((double)c[k].hi[a] - (double)lo[a]) * inv);
            ql = ql < 0 ? 0 : (ql > 255 ? 255 : ql);
            qh = qh < 0 ? 0 : (qh > 255 ? 255 : qh);
            qlo[a][s] = (unsigned char)ql;
            qhi[a][s] = (unsigned char)qh;
        }
        if (c[k].code >= 0) {
            imask |= 1u << s;
            meta[s] = 0x80u;  // any non-zero value: slot in use
            next_tasks[task_base + ci] = make_int2(c[k].code, child_base + ci);
            ++ci;
        } else {
            const int first = leaf_first(c[k].code), cnt = leaf_count(c[k].code);
            meta[s] = (unsigned char)(0x80u | ((unsigned)(cnt - 1) << 5) | (unsigned)to);
            for (int j = 0; j < cnt; ++j) {
                const int src = 3 * (first + j), dst = 3 * (tri_base + to + j);
                tri_out[dst] = tri_in[src];
                tri_out[dst + 1] = tri_in[src + 1];
                tri_out[dst + 2] = tri_in[src + 2];
            }
            to += cnt;
        }
    }
    auto pack4 = [](const unsigned char* b) {
        return (unsigned)b[0] | ((unsigned)b[1] << 8) | ((unsigned)b[2] << 16) | ((unsigned)b[3] << 24);
    };
    Bvh8Node nd;
    nd.p = make_float4(lo[0], lo[1], lo[2],
                       __uint_as_float((unsigned)(e[0] + 127) | ((unsigned)(e[1] + 127) << 8) |
                                       ((unsigned)(e[2] + 127) << 16) | (imask << 24)));
    nd.m = make_uint4((unsigned)child_base, (unsigned)tri_base, pack4(meta), pack4(meta + 4));
    nd.qx = make_uint4(pack4(qlo[0]), pack4(qlo[0] + 4), pack4(qhi[0]), pack4(qhi[0] + 4));
    nd.qy = make_uint4(pack4(qlo[1]), pack4(qlo[1] + 4), pack4(qhi[1]), pack4(qhi[1] + 4));
    nd.qz = make_uint4(pack4(qlo[2]), pack4(qlo[2] + 4), pack4(qhi[2]), pack4(qhi[2] + 4));
    out[task.y] = nd;
}

}  // namespace

void build_bvh8(const BvhNode* bin, const float4* tri_in, int root, int n, float4 root_lo, float4 root_hi,
                Bvh8Node* out, float4* tri_out, int* num_nodes, int* depth, hipStream_t stream) {
    DevBuf<int2> tasks[2];
    tasks[0].alloc(n);
    tasks[1].alloc(n);
    DevBuf<int> cnt;  // per level: [0] nodes [1] tris [2] next tasks [3] depth; [4] current task count
    cnt.alloc(8);
    const int2 root_task = make_int2(root, 0);
    int init[8] = {1, 0, 0, 0, 1, 0, 0, 0};
    PGRT_HIP(hipMemcpyAsync(cnt.p, init, sizeof(init), hipMemcpyHostToDevice, stream));
    PGRT_HIP(hipMemcpyAsync(tasks[0].p, &root_task, sizeof(int2), hipMemcpyHostToDevice, stream));
    int ntask = 1, cur = 0, level = 0;
    while (ntask > 0) {
        PGRT_REQUIRE(level < 64, PGRT_ERR_HIP, "wide BVH collapse did not terminate");
        hipLaunchKernelGGL(k_collapse, dim3(ceil_div(ntask, kB)), dim3(kB), 0, stream, bin, tri_in, tasks[cur].p,
                           cnt.p + 4, tasks[cur ^ 1].p, cnt.p, level, root_lo, root_hi, out, tri_out);
        // next level: task count = counters[2]; reset counters[2]
        PGRT_HIP(hipMemcpyAsync(cnt.p + 4, cnt.p + 2, sizeof(int), hipMemcpyDeviceToDevice, stream));
        PGRT_HIP(hipMemcpyAsync(&ntask, cnt.p + 2, sizeof(int), hipMemcpyDeviceToHost, stream));
        PGRT_HIP(hipMemsetAsync(cnt.p + 2, 0, sizeof(int), stream));
        PGRT_HIP(hipStreamSynchronize(stream));
        cur ^= 1;
        ++level;
    }
    int h[4];
    PGRT_HIP(hipMemcpyAsync(h, cnt.p, sizeof(h), hipMemcpyDeviceToHost, stream));
    PGRT_HIP(hipStreamSynchronize(stream));
    PGRT_REQUIRE(h[1] == n, PGRT_ERR_HIP, "wide BVH collapse lost triangles");
    *num_nodes = h[0];
    *depth = h[3];
}

}  // namespace pgrt
