// latency_probe.hip -- dependent-load latency of one lane on gfx950 (calibrates the traversal
// step cost).  A random cyclic permutation of 128-B lines in a buffer of S bytes is chased by
// one lane; reports ns and shader-clock cycles per load.
// build: hipcc --offload-arch=gfx950 -O3 -o build/latency_probe tools/latency_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <random>
#include <vector>

__global__ void chase(const unsigned* __restrict__ next, int steps, unsigned* out, long long* t) {
    unsigned p = 0;
    const long long c0 = clock64();
    const long long w0 = wall_clock64();
    for (int i = 0; i < steps; ++i) p = next[p];
    const long long c1 = clock64();
    const long long w1 = wall_clock64();
    out[0] = p;
    t[0] = c1 - c0;
    t[1] = w1 - w0;
}

int main() {
    const size_t flush_bytes = size_t(1) << 30;
    void* flush;
    (void)hipMalloc(&flush, flush_bytes);
    const size_t sizes[] = {16u << 10, 256u << 10, 2u << 20, 8u << 20, 64u << 20, 1024u << 20};
    for (size_t bytes : sizes) {
        const size_t lines = bytes / 128;
        std::vector<unsigned> perm(lines);
        for (size_t i = 0; i < lines; ++i) perm[i] = (unsigned)i;
        std::mt19937 rng(1);
        std::shuffle(perm.begin(), perm.end(), rng);
        std::vector<unsigned> next(bytes / 4, 0);
        for (size_t i = 0; i < lines; ++i) next[perm[i] * 32] = perm[(i + 1) % lines] * 32;
        unsigned* d;
        unsigned* o;
        long long* t;
        (void)hipMalloc(&d, bytes);
        (void)hipMalloc(&o, 64);
        (void)hipMalloc(&t, 64);
        (void)hipMemcpy(d, next.data(), bytes, hipMemcpyHostToDevice);
        const int steps = 20000;
        // rep 0: after a 1 GiB streaming write elsewhere (cold: HBM); rep 1: right after rep 0
        // (same path: L2 / MALL warm)
        (void)hipMemset(flush, 1, flush_bytes);
        (void)hipDeviceSynchronize();
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(chase, dim3(1), dim3(1), 0, 0, d, steps, o, t);
            long long h[2];
            (void)hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
            printf("buffer %8zu KB %s: %7.1f ns/load %7.1f clk/load (clock %.2f GHz)\n", bytes >> 10,
                   rep ? "warm" : "cold", h[1] * 10.0 / steps, (double)h[0] / steps, (double)h[0] / (h[1] * 10.0));
        }
        (void)hipFree(d);
        (void)hipFree(o);
        (void)hipFree(t);
    }
    return 0;
}
