// How many kernels from different streams run at once?  N streams each launch one single-block
// kernel that spins for ~1 ms (wall_clock64); wall time / 1 ms = serialisation factor.
// hipcc --offload-arch=gfx950 -O2 -o build/stream_concurrency tools/stream_concurrency.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

__global__ void k_spin(long long ticks) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}

int main() {
    const long long ticks = 100000;  // wall_clock64 runs at 100 MHz: 1 ms
    for (int n : {1, 2, 3, 4, 6, 8, 12}) {
        std::vector<hipStream_t> s(n);
        for (auto& x : s) (void)hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipDeviceSynchronize();
            auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s[i], ticks);
            (void)hipDeviceSynchronize();
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            if (rep == 2) printf("streams %2d: %.2f ms (%.2f kernels at once)\n", n, ms, n / ms);
        }
        for (auto& x : s) (void)hipStreamDestroy(x);
    }
    return 0;
}
