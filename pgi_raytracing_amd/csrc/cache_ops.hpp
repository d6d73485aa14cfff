// cache_ops.hpp -- L2 policy of the frame's streaming data.
//
// The scene's traversal data (BVH nodes + triangle records, ~4 MB for the avenger proxy) and the
// shading tables are re-read by every launch of a frame; the ray queues, hit records, node records,
// shadow rays and the framebuffer are written once and read once (or never: the framebuffer).
// Measured on MI355X (tools/l2_persist_probe.hip, profiles/r4/l2_persist_probe_r4.txt): a table
// warmed into an XCD's 4 MiB L2 stays there across kernel boundaries (172 cycles per dependent
// load), but 64 MB of plain streaming stores OR plain streaming loads in between evict it (478
// cycles: an Infinity-Cache hit); the same 64 MB of write-through `sc1` stores leave it in place
// (172), `nt` stores and `nt` loads almost (174-279 from a 1 MB to a 3.9 MB table).  So the
// streaming outputs are stored with `sc1` (16-B per lane: the rate of a plain dwordx4 store) or
// `nt` (narrower stores: an `sc1` dword is one fabric write per lane), and the streaming inputs are
// loaded `nt` -- the traversal data of the deep, latency-bound levels then hits in L2.
// PGRT_STREAM_CACHE=0 (A/B builds): plain loads and stores.
#pragma once

#include <hip/hip_runtime.h>

#ifndef PGRT_STREAM_CACHE
#define PGRT_STREAM_CACHE 1
#endif
#ifndef PGRT_STREAM_ST
#define PGRT_STREAM_ST PGRT_STREAM_CACHE
#endif
#ifndef PGRT_STREAM_LD
#define PGRT_STREAM_LD PGRT_STREAM_CACHE
#endif

namespace pgrt {

typedef float pg_f4 __attribute__((ext_vector_type(4)));
typedef int pg_i4 __attribute__((ext_vector_type(4)));

// write-once 16-B records: write-through, the line leaves the XCD's L2.  The store is inline asm
// (no builtin carries sc1 on a plain global store), so the compiler's hazard recognizer does not
// see it: a VALU write of its data VGPRs right after it (the VMEM store-data hazard of stores
// wider than 8 bytes, 1 wait state on gfx9+) would change the stored value -- the asm carries its
// own s_nop.
__device__ __forceinline__ void st_stream(float4* p, float4 v) {
#if PGRT_STREAM_ST
    const pg_f4 w = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(w));
#else
    *p = v;
#endif
}
__device__ __forceinline__ void st_stream(int4* p, int4 v) {
#if PGRT_STREAM_ST
    const pg_i4 w = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(w));
#else
    *p = v;
#endif
}
// narrow write-once values: nontemporal
template <class T>
__device__ __forceinline__ void st_stream_nt(T* p, T v) {
#if PGRT_STREAM_ST
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}
// read-once streaming inputs: nontemporal loads
__device__ __forceinline__ float4 ld_stream(const float4* p) {
#if PGRT_STREAM_LD
    const pg_f4 v = __builtin_nontemporal_load(reinterpret_cast<const pg_f4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
#else
    return *p;
#endif
}
__device__ __forceinline__ int4 ld_stream(const int4* p) {
#if PGRT_STREAM_LD
    const pg_i4 v = __builtin_nontemporal_load(reinterpret_cast<const pg_i4*>(p));
    return make_int4(v.x, v.y, v.z, v.w);
#else
    return *p;
#endif
}
template <class T>
__device__ __forceinline__ T ld_stream_nt(const T* p) {
#if PGRT_STREAM_LD
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}

}  // namespace pgrt
