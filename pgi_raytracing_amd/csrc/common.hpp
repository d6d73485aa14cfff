// common.hpp -- shared host/device definitions for libpgrt (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "pgrt.h"
#include "pgrt_detmath.h"

namespace pgrt {

// Error carried from deep inside the library to the C ABI (never crosses it).
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define PGRT_HIP(call)                                                                        \
    do {                                                                                      \
        hipError_t e_ = (call);                                                               \
        if (e_ != hipSuccess)                                                                 \
            throw ::pgrt::Error(PGRT_ERR_HIP, std::string(#call " failed: ") +                \
                                                  hipGetErrorString(e_) + " at " __FILE__ ":" + \
                                                  std::to_string(__LINE__));                  \
    } while (0)

#define PGRT_REQUIRE(cond, code, msg)                     \
    do {                                                  \
        if (!(cond)) throw ::pgrt::Error((code), (msg)); \
    } while (0)

// Device buffer owned by the context (RAII, no exceptions in the destructor).
template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    void alloc(size_t count) {
        if (count <= n && p) return;
        release();
        if (count == 0) count = 1;
        hipError_t e = hipMalloc(&p, count * sizeof(T));
        if (e != hipSuccess) {
            p = nullptr;
            throw Error(PGRT_ERR_OUT_OF_MEMORY, "hipMalloc of " + std::to_string(count * sizeof(T)) +
                                                    " bytes failed: " + hipGetErrorString(e));
        }
        n = count;
        static const bool log = getenv("PGRT_LOG_ALLOC") != nullptr;  // fault triage: address map
        if (log) fprintf(stderr, "pgrt alloc %p %zu\n", (void*)p, count * sizeof(T));
    }
    size_t bytes() const { return n * sizeof(T); }
    void swap(DevBuf& o) {
        std::swap(p, o.p);
        std::swap(n, o.n);
    }
};

// ---- device-side scene layout (HBM) -------------------------------------------------------

struct DevMaterial {  // 48 B, read through the scalar/vector cache
    float kd[3];
    float ks[3];
    float ns, ior;
    int type, tex;
    int pad[2];
};

struct DevTexture {
    int width, height, pitch, bpp;
    long long offset;  // into the texel pool
    long long size;    // pitch * height
};

struct DevLight {
    float pos[3], kd[3], ks[3];
};

// BVH2 node, 64 B: both child boxes live in the parent (Aila-Laine layout).
//   a = (c0.lo.x, c0.hi.x, c0.lo.y, c0.hi.y)   b = (c1.lo.x, c1.hi.x, c1.lo.y, c1.hi.y)
//   c = (c0.lo.z, c0.hi.z, c1.lo.z, c1.hi.z)   d = (child0, child1, -, -)
// child >= 0: internal node index; child < 0: leaf = 0x80000000 | (count-1) << 27 | first.
struct BvhNode {
    float4 a, b, c;
    int4 d;
};

constexpr int kLeafMaxTris = 4;
__host__ __device__ inline int leaf_encode(int first, int count) {
    return (int)(0x80000000u | ((unsigned)(count - 1) << 27) | (unsigned)first);
}
__host__ __device__ inline int leaf_first(int c) { return (int)((unsigned)c & 0x07ffffffu); }
__host__ __device__ inline int leaf_count(int c) { return (int)(((unsigned)c >> 27) & 0xfu) + 1; }

// 8-wide BVH node, 80 B (five 16-B loads): 8 child boxes quantized to 8 bits per plane
// relative to origin p with per-axis scale 2^e (conservative: floor / ceil).
//   p  = (origin.xyz, bits: e.x+127 | e.y+127 << 8 | e.z+127 << 16 | imask << 24)
//   m  = (child_base, tri_base, meta[0..3], meta[4..7])
//   qx = (lo.x[0..3], lo.x[4..7], hi.x[0..3], hi.x[4..7]) bytes, likewise qy, qz
// imask bit s: slot s is an internal node, stored at child_base + popc(imask below s).
// meta[s] of a leaf: 0x80 | (count - 1) << 5 | offset from tri_base (count <= 4, <= 32
// triangles per node, so a node's triangles fit one 32-bit mask); 0 = empty slot.
struct Bvh8Node {
    float4 p;
    uint4 m;
    uint4 qx, qy, qz;
};
__host__ __device__ inline unsigned wide_leaf_bits(unsigned meta) {  // the leaf's triangle mask
    return ((2u << ((meta >> 5) & 3u)) - 1u) << (meta & 31u);
}

// base + a 32-bit byte offset, zero-extended: a global load then takes the (wave-uniform) base as
// its scalar address operand and the offset as one VGPR -- no 64-bit address arithmetic per node or
// triangle.  Every BVH / triangle array of a scene stays below 4 GiB (scene.cpp checks the sizes).
template <class T>
__device__ __forceinline__ const T* at_bytes(const T* base, unsigned off) {
    return reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + off);
}

struct SceneView {  // kernel-argument view of the device scene
    const float4* tri;     // 3 x float4 per sorted triangle: (v0, orig id bits) (e1) (e2)
    const float4* tri_ng;  // per sorted triangle: its Ng = e2 x e1 (tri_normal), w = 0
    const BvhNode* nodes;
    int root;              // node index, or a leaf code for tiny scenes
    const Bvh8Node* nodes8;  // 8-wide BVH (root = node 0)
    const float4* tri8;      // triangles in 8-wide leaf order (same records as tri)
    int depth8;              // 8-wide BVH depth
    int group_max;           // queues of <= group_max rays: 8 lanes per ray over the 8-wide BVH
    int wide;
    int ntri;
    int depth;             // binary BVH depth (bounds the traversal stack)
    const float* attr;     // 16 floats per ORIGINAL triangle: n0 n1 n2 uv0 uv1 uv2, mat (bits)
    const unsigned char* prim_glass;  // per ORIGINAL triangle: 1 when its material is dielectric
    const DevMaterial* mats;
    const DevTexture* tex;
    int nmat, ntex;
    const unsigned char* texels;
    int env;
    int nlight;
    const DevLight* lights;
    // this launch's timeline slots (stamps.hpp; set per launch by the launcher), NULL = off
    unsigned long long* stamps;
};

struct CameraView {
    int width, height;
    float fy;
    float from[3];
    float m[9];  // row-major; columns x_c, y_c, z_c
};

inline int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }

}  // namespace pgrt
