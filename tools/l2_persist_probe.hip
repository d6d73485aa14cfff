// l2_persist_probe.hip -- does an XCD's L2 keep a table across kernel boundaries?
// One lane per block chases a random cycle of 128-B lines; pass 1 runs right after the
// preceding launch (cross-launch), pass 2 chases the same lines again inside the same launch
// (surely L2-resident).  Sequences:
//   cold      : 1 GiB memset, then chase             (pass 1 = MALL/HBM)
//   warm      : warm kernel reads the table on every XCD, then chase
//   warm+nop  : warm, an empty kernel, then chase
//   warm+str  : warm, a kernel streaming S MB of plain stores, then chase
//   warm+sc1  : warm, the same stream with sc1 stores (drop the line from L2), then chase
//   warm+nt / warm+ld / warm+ntld : nt stores, plain loads, nt loads of the same stream
// (the two passes of one launch are merged by the compiler: the figure is the first chase)
// build: hipcc --offload-arch=gfx950 -O3 -o build/l2_persist_probe tools/l2_persist_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <random>
#include <vector>

__device__ inline unsigned xcc_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 0xf;
}

__global__ void warm(const unsigned* __restrict__ t, int words, unsigned* sink) {
    unsigned acc = 0;
    for (int i = threadIdx.x * 32; i < words; i += blockDim.x * 32) acc += t[i];
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void nop_kernel(unsigned* sink) {
    if (threadIdx.x == 1000) sink[0] = 1;
}

__global__ void stream_stores(float4* dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = make_float4((float)i, 1.f, 2.f, 3.f);
}

__global__ void stream_sc1(float4* dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        typedef float f4 __attribute__((ext_vector_type(4)));
        const f4 v = {(float)i, 1.f, 2.f, 3.f};
        float4* p = dst + i;
        asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    }
}

__global__ void stream_loads(const float4* src, size_t n, float* sink) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = src[i];
        acc += v.x + v.w;
    }
    if (acc == 1234.5f) sink[0] = acc;
}

__global__ void stream_nt_loads(const float4* src, size_t n, float* sink) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        typedef float f4 __attribute__((ext_vector_type(4)));
        const f4 v = __builtin_nontemporal_load(reinterpret_cast<const f4*>(src) + i);
        acc += v.x + v.w;
    }
    if (acc == 1234.5f) sink[0] = acc;
}

__global__ void stream_nt_stores(float4* dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    {
        typedef float f4 __attribute__((ext_vector_type(4)));
        const f4 v = {(float)i, 1.f, 2.f, 3.f};
        __builtin_nontemporal_store(v, reinterpret_cast<f4*>(dst) + i);
    }
}

__global__ void chase(const unsigned* __restrict__ next, int steps, int stride, long long* out) {
    if (threadIdx.x != 0) return;
    unsigned start = (unsigned)(blockIdx.x * stride) * 32u;
    long long r[2];
    unsigned p = start;
    for (int pass = 0; pass < 2; ++pass) {
        p = start;
        const long long c0 = clock64();
        for (int i = 0; i < steps; ++i) p = next[p];
        const long long c1 = clock64();
        r[pass] = c1 - c0;
    }
    out[blockIdx.x * 4 + 0] = r[0];
    out[blockIdx.x * 4 + 1] = r[1];
    out[blockIdx.x * 4 + 2] = xcc_id();
    out[blockIdx.x * 4 + 3] = p;
}

int main() {
    const size_t max_bytes = 4u << 20;
    unsigned *d, *sink;
    long long* out;
    void* flush;
    float4* strm;
    const size_t flush_bytes = size_t(1) << 30;
    const size_t strm_bytes = size_t(64) << 20;
    (void)hipMalloc(&d, max_bytes);
    (void)hipMalloc(&sink, 64);
    (void)hipMalloc(&out, 64 * 4 * sizeof(long long));
    (void)hipMalloc(&flush, flush_bytes);
    (void)hipMalloc(&strm, strm_bytes);
    (void)hipMemset(strm, 0, strm_bytes);
    const size_t sizes[] = {1u << 20, 2u << 20, 3u << 20, (size_t)(3.8 * (1 << 20))};
    const char* names[] = {"cold", "warm", "warm+nop", "warm+st64MB", "warm+sc1st64MB", "warm+ntst64MB",
                           "warm+ld64MB", "warm+ntld64MB"};
    for (size_t bytes : sizes) {
        const size_t lines = bytes / 128;
        std::vector<unsigned> perm(lines);
        for (size_t i = 0; i < lines; ++i) perm[i] = (unsigned)i;
        std::mt19937 rng(7);
        std::shuffle(perm.begin(), perm.end(), rng);
        std::vector<unsigned> next(bytes / 4, 0);
        for (size_t i = 0; i < lines; ++i) next[perm[i] * 32] = perm[(i + 1) % lines] * 32;
        (void)hipMemcpy(d, next.data(), bytes, hipMemcpyHostToDevice);
        const int nblk = 16, steps = 512;
        for (int seq = 0; seq < 8; ++seq) {
            double tot = 0;
            const int reps = 3;
            for (int rep = 0; rep < reps; ++rep) {
                (void)hipMemset(flush, rep + 1, flush_bytes);
                (void)hipDeviceSynchronize();
                if (seq >= 1) hipLaunchKernelGGL(warm, dim3(8 * 32), dim3(256), 0, 0, d, (int)(bytes / 4), sink);
                if (seq == 2) hipLaunchKernelGGL(nop_kernel, dim3(256), dim3(64), 0, 0, sink);
                if (seq == 3) hipLaunchKernelGGL(stream_stores, dim3(2048), dim3(256), 0, 0, strm, strm_bytes / 16);
                if (seq == 4) hipLaunchKernelGGL(stream_sc1, dim3(2048), dim3(256), 0, 0, strm, strm_bytes / 16);
                if (seq == 5) hipLaunchKernelGGL(stream_nt_stores, dim3(2048), dim3(256), 0, 0, strm, strm_bytes / 16);
                if (seq == 6)
                    hipLaunchKernelGGL(stream_loads, dim3(2048), dim3(256), 0, 0, strm, strm_bytes / 16, (float*)sink);
                if (seq == 7)
                    hipLaunchKernelGGL(stream_nt_loads, dim3(2048), dim3(256), 0, 0, strm, strm_bytes / 16,
                                       (float*)sink);
                hipLaunchKernelGGL(chase, dim3(nblk), dim3(64), 0, 0, d, steps, (int)(lines / nblk), out);
                (void)hipDeviceSynchronize();
                std::vector<long long> h(nblk * 4);
                (void)hipMemcpy(h.data(), out, h.size() * sizeof(long long), hipMemcpyDeviceToHost);
                double p = 0;
                for (int b = 0; b < nblk; ++b) p += (double)(h[b * 4] + h[b * 4 + 1]) / steps;
                tot += p / nblk;
            }
            printf("table %5zu KB %-16s: %7.1f clk/load (first chase after the sequence, mean of %d)\n",
                   bytes >> 10, names[seq], tot / reps, reps);
        }
    }
    return 0;
}
