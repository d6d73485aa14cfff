// stamp_probe.hip -- what do the timeline stamps (stamps.hpp) cost a kernel that does not record?
// A grid-stride copy (the shape of k_export_counters / k_combine) with: no stamp code, the
// PGRT_STAMP_BEGIN / END macros and a NULL pointer, BEGIN only, END only, and a live pointer.
// Average device time of 200 back-to-back launches each (HIP events).
// build: hipcc --offload-arch=gfx950 -O3 -I pgi_raytracing_amd/csrc -o build/stamp_probe tools/stamp_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#include "stamps.hpp"

template <int MODE>
__global__ void copy_k(const uint4* __restrict__ src, uint4* __restrict__ dst, int n, unsigned long long* stamps) {
    if constexpr (MODE == 1 || MODE == 2 || MODE == 4) {
        PGRT_STAMP_BEGIN(stamps);
        for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) dst[i] = src[i];
        if constexpr (MODE != 2) PGRT_STAMP_END(stamps);
        (void)pgrt_stamp_t0_;
    } else if constexpr (MODE == 3) {
        const unsigned long long pgrt_stamp_t0_ = 0;
        for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) dst[i] = src[i];
        PGRT_STAMP_END(stamps);
    } else if constexpr (MODE == 5) {  // END indexing from blockIdx.x only
        const unsigned long long t0 = stamps ? wall_clock64() : 0ull;
        for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) dst[i] = src[i];
        if (stamps) {
            const unsigned long long t1 = wall_clock64();
            if (__lane_id() == 0)
                reinterpret_cast<ulonglong2*>(stamps)[blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)] =
                    make_ulonglong2(t0, t1);
        }
    } else {
        for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) dst[i] = src[i];
    }
}

template <int MODE>
float time_it(const uint4* src, uint4* dst, int n, int grid, unsigned long long* st) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(copy_k<MODE>, dim3(grid), dim3(256), 0, 0, src, dst, n, st);
    (void)hipEventRecord(a, 0);
    for (int r = 0; r < 200; ++r) hipLaunchKernelGGL(copy_k<MODE>, dim3(grid), dim3(256), 0, 0, src, dst, n, st);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1000.0f / 200;
}

int main() {
    const int n = 1 << 22;  // 64 MB
    uint4 *src, *dst;
    unsigned long long* st;
    (void)hipMalloc(&src, n * sizeof(uint4));
    (void)hipMalloc(&dst, n * sizeof(uint4));
    (void)hipMalloc(&st, (size_t)16384 * 4 * 16);
    (void)hipMemset(src, 1, n * sizeof(uint4));
    for (int grid : {64, 1024, 16384}) {
        for (int nn : {16384, n}) {
            printf("grid %5d n %8d: none %8.2f us  macros(null) %8.2f  begin-only %8.2f  end-only %8.2f  live %8.2f  x-only(null) %8.2f\n",
                   grid, nn, time_it<0>(src, dst, nn, grid, nullptr), time_it<1>(src, dst, nn, grid, nullptr),
                   time_it<2>(src, dst, nn, grid, nullptr), time_it<3>(src, dst, nn, grid, nullptr),
                   time_it<4>(src, dst, nn, grid, st), time_it<5>(src, dst, nn, grid, nullptr));
        }
    }
    return 0;
}
