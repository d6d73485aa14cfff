// store_probe.hip -- are the streaming stores of cache_ops.hpp visible to the next kernel?
// For each store form: a kernel fills the array with a marker (plain stores) and reads it from
// every XCD (L2-resident copies everywhere), the writer kernel stores the values with the form
// under test, the checker kernel (different block -> element mapping) reads them with plain loads
// and counts mismatches.
// build: hipcc --offload-arch=gfx950 -O3 -o build/store_probe tools/store_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void prefill(float4* a, unsigned char* b, float* c, int n, unsigned* sink) {
    unsigned acc = 0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        a[i] = make_float4(-1, -1, -1, -1);
        b[i] = 0xee;
        c[i] = -1.0f;
    }
    __syncthreads();
    // every block reads everything: copies in every XCD's L2
    for (int i = threadIdx.x; i < n; i += blockDim.x) acc += (unsigned)a[i].x + b[i] + (unsigned)c[i];
    if (acc == 0x12345u) sink[0] = acc;
}

template <int MODE>
__global__ void writer(float4* a, unsigned char* b, float* c, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float v = (float)i;
        if (MODE == 0) {  // plain
            a[i] = make_float4(v, v + 1, v + 2, v + 3);
            b[i] = (unsigned char)(i & 255);
            c[i] = v;
        } else if (MODE == 1) {  // cache_ops.hpp: sc1 asm dwordx4, nt narrow
            const f4 w = {v, v + 1, v + 2, v + 3};
            float4* p = a + i;
            asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(w));
            __builtin_nontemporal_store((unsigned char)(i & 255), b + i);
            __builtin_nontemporal_store(v, c + i);
        } else if (MODE == 2) {  // sc1 asm dwordx4 only
            const f4 w = {v, v + 1, v + 2, v + 3};
            float4* p = a + i;
            asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(w));
            b[i] = (unsigned char)(i & 255);
            c[i] = v;
        } else {  // nt narrow only
            a[i] = make_float4(v, v + 1, v + 2, v + 3);
            __builtin_nontemporal_store((unsigned char)(i & 255), b + i);
            __builtin_nontemporal_store(v, c + i);
        }
    }
}

__global__ void checker(const float4* a, const unsigned char* b, const float* c, int n, unsigned* bad) {
    unsigned ba = 0, bb = 0, bc = 0;
    // reversed mapping: element i read by a different block than the one that wrote it
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        const int i = n - 1 - k;
        const float v = (float)i;
        const float4 x = a[i];
        ba += (x.x != v || x.y != v + 1 || x.z != v + 2 || x.w != v + 3);
        bb += (b[i] != (unsigned char)(i & 255));
        bc += (c[i] != v);
    }
    if (ba) atomicAdd(&bad[0], ba);
    if (bb) atomicAdd(&bad[1], bb);
    if (bc) atomicAdd(&bad[2], bc);
}

int main() {
    const int n = 1 << 20;
    float4* a;
    unsigned char* b;
    float* c;
    unsigned *bad, *sink;
    (void)hipMalloc(&a, n * sizeof(float4));
    (void)hipMalloc(&b, n);
    (void)hipMalloc(&c, n * sizeof(float));
    (void)hipMalloc(&bad, 16);
    (void)hipMalloc(&sink, 16);
    const char* names[] = {"plain", "sc1 x4 + nt narrow", "sc1 x4 only", "nt narrow only"};
    for (int mode = 0; mode < 4; ++mode) {
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipMemset(bad, 0, 16);
            hipLaunchKernelGGL(prefill, dim3(512), dim3(256), 0, 0, a, b, c, n, sink);
            if (mode == 0) hipLaunchKernelGGL(writer<0>, dim3(1024), dim3(256), 0, 0, a, b, c, n);
            if (mode == 1) hipLaunchKernelGGL(writer<1>, dim3(1024), dim3(256), 0, 0, a, b, c, n);
            if (mode == 2) hipLaunchKernelGGL(writer<2>, dim3(1024), dim3(256), 0, 0, a, b, c, n);
            if (mode == 3) hipLaunchKernelGGL(writer<3>, dim3(1024), dim3(256), 0, 0, a, b, c, n);
            hipLaunchKernelGGL(checker, dim3(777), dim3(256), 0, 0, a, b, c, n, bad);
            unsigned h[4];
            (void)hipMemcpy(h, bad, 16, hipMemcpyDeviceToHost);
            printf("%-20s rep %d: stale float4 %u, byte %u, float %u (of %d)\n", names[mode], rep, h[0], h[1], h[2], n);
        }
    }
    return 0;
}
