// bvh_layout.hip -- cache-line layout of the binary BVH, applied after either builder.
//
// The builders emit internal nodes in creation order (PLOC: merge iterations bottom-up; LBVH:
// Karras split order), so a node's children sit anywhere in the node array and every node visit
// of a traversal is a cache line of its own.  Here the two children of every internal node are
// stored side by side in one 128-B line (two 64-B nodes, "sibling pairs"), and the pairs are laid
// out in depth-first order of their parents:
//   - descending into the nearer child brings its sibling into the cache with it, so the later
//     pop of that sibling (the far child on the stack) is usually a cache hit instead of another
//     round trip to the L2 / MALL;
//   - a subtree occupies one contiguous range of lines (page and MALL locality for big scenes).
// The root is slot 0 (slot 1 is padding); pair j holds slots 2j + 2 and 2j + 3; a node with only
// one internal child fills half its pair.  Child codes of leaves are unchanged, so are the
// triangle records, and traversal results do not depend on node order (tests: every layout
// bit-exact against the oracle).
#include "common.hpp"
#include "trace.hpp"

namespace pgrt {
namespace {

constexpr int kB = 256;

// parent[c] = node index of c's parent (internal children only); depth by walking up
__global__ __launch_bounds__(kB) void k_lay_parents(const BvhNode* __restrict__ nodes, int n, int* __restrict__ parent) {
    const int q = blockIdx.x * kB + threadIdx.x;
    if (q >= n) return;
    const int4 d = nodes[q].d;
    if (d.x >= 0) parent[d.x] = q;
    if (d.y >= 0) parent[d.y] = q;
}

__global__ __launch_bounds__(kB) void k_lay_depth(const int* __restrict__ parent, int n, int root, int* __restrict__ depth,
                                                  int* __restrict__ max_depth) {
    const int q = blockIdx.x * kB + threadIdx.x;
    if (q >= n) return;
    int v = q, dd = 0;
    while (v != root && v >= 0 && dd < n) {
        v = parent[v];
        ++dd;
    }
    // nodes below a collapsed leaf (PLOC's SAH leaf collapse keeps them in the array, referenced
    // by a leaf code) have no parent chain to the root: depth -1, never placed
    depth[q] = v == root ? dd : -1;
    if (v == root) atomicMax(max_depth, dd);
}

// bottom-up, one tree level per launch: pairs[v] = line pairs in v's subtree (its own pair when it
// has an internal child + its internal children's)
__global__ __launch_bounds__(kB) void k_lay_up(const BvhNode* __restrict__ nodes, int n, const int* __restrict__ depth,
                                               int level, int* __restrict__ pairs) {
    const int q = blockIdx.x * kB + threadIdx.x;
    if (q >= n || depth[q] != level) return;
    const int4 d = nodes[q].d;
    int s = 0;
    if (d.x >= 0) s += pairs[d.x];
    if (d.y >= 0) s += pairs[d.y];
    pairs[q] = s + ((d.x >= 0 || d.y >= 0) ? 1 : 0);
}

// top-down, one tree level per launch: first[v] = v's own pair (its children's slots); the
// children's subtrees follow it in depth-first order (child 0's, then child 1's)
__global__ __launch_bounds__(kB) void k_lay_down(const BvhNode* __restrict__ nodes, int n, const int* __restrict__ depth,
                                                 int level, const int* __restrict__ pairs, int* __restrict__ first,
                                                 int* __restrict__ slot) {
    const int q = blockIdx.x * kB + threadIdx.x;
    if (q >= n || depth[q] != level) return;
    const int4 d = nodes[q].d;
    if (d.x < 0 && d.y < 0) return;
    const int base = first[q];
    int next = base + 1, k = 0;
    if (d.x >= 0) {
        slot[d.x] = 2 * base + 2 + k++;
        first[d.x] = next;
        next += pairs[d.x];
    }
    if (d.y >= 0) {
        slot[d.y] = 2 * base + 2 + k;
        first[d.y] = next;
    }
}

__global__ __launch_bounds__(kB) void k_lay_write(const BvhNode* __restrict__ nodes, int n, const int* __restrict__ depth,
                                                  const int* __restrict__ slot, BvhNode* __restrict__ out) {
    const int q = blockIdx.x * kB + threadIdx.x;
    if (q >= n || depth[q] < 0) return;
    BvhNode nd = nodes[q];
    if (nd.d.x >= 0) nd.d.x = slot[nd.d.x];
    if (nd.d.y >= 0) nd.d.y = slot[nd.d.y];
    out[slot[q]] = nd;
}

__global__ void k_lay_root(int root, int* __restrict__ slot, int* __restrict__ first) {
    slot[root] = 0;
    first[root] = 0;
}

}  // namespace

// nodes: num_nodes internal nodes rooted at *root (a node index; a leaf-code root is left alone).
// Rewrites nodes in the sibling-pair layout (the buffer may grow) and sets *root = 0; returns the
// new node count (slots, padding included).
int relayout_bvh(DevBuf<BvhNode>& nodes, int num_nodes, int* root, hipStream_t stream) {
    const int n = num_nodes;
    if (n < 2 || *root < 0) return n;
    DevBuf<int> parent, depth, pairs, first, slot, maxd;
    parent.alloc(n);
    depth.alloc(n);
    pairs.alloc(n);
    first.alloc(n);
    slot.alloc(n);
    maxd.alloc(1);
    PGRT_HIP(hipMemsetAsync(maxd.p, 0, sizeof(int), stream));
    PGRT_HIP(hipMemsetAsync(parent.p, 0xff, sizeof(int) * (size_t)n, stream));  // -1: no internal parent
    const int g = ceil_div(n, kB);
    hipLaunchKernelGGL(k_lay_parents, dim3(g), dim3(kB), 0, stream, nodes.p, n, parent.p);
    hipLaunchKernelGGL(k_lay_depth, dim3(g), dim3(kB), 0, stream, parent.p, n, *root, depth.p, maxd.p);
    int max_depth = 0;
    PGRT_HIP(hipMemcpyAsync(&max_depth, maxd.p, sizeof(int), hipMemcpyDeviceToHost, stream));
    PGRT_HIP(hipStreamSynchronize(stream));
    const int levels = max_depth + 1;  // internal-node levels
    for (int l = levels - 1; l >= 0; --l)
        hipLaunchKernelGGL(k_lay_up, dim3(g), dim3(kB), 0, stream, nodes.p, n, depth.p, l, pairs.p);
    hipLaunchKernelGGL(k_lay_root, dim3(1), dim3(1), 0, stream, *root, slot.p, first.p);
    for (int l = 0; l < levels; ++l)
        hipLaunchKernelGGL(k_lay_down, dim3(g), dim3(kB), 0, stream, nodes.p, n, depth.p, l, pairs.p, first.p, slot.p);
    int root_pairs = 0;
    PGRT_HIP(hipMemcpyAsync(&root_pairs, pairs.p + *root, sizeof(int), hipMemcpyDeviceToHost, stream));
    PGRT_HIP(hipStreamSynchronize(stream));
    const int slots = 2 + 2 * root_pairs;
    DevBuf<BvhNode> out;
    out.alloc((size_t)slots);
    PGRT_HIP(hipMemsetAsync(out.p, 0, sizeof(BvhNode) * (size_t)slots, stream));  // padding slots
    hipLaunchKernelGGL(k_lay_write, dim3(g), dim3(kB), 0, stream, nodes.p, n, depth.p, slot.p, out.p);
    PGRT_HIP(hipGetLastError());
    PGRT_HIP(hipStreamSynchronize(stream));
    nodes.swap(out);
    *root = 0;
    return slots;
}

}  // namespace pgrt
