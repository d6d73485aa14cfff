// d2h_probe.hip -- device-to-host bandwidth of the ways a C2 framebuffer (1920x1080 RGBA f32,
// 33.2 MB) can reach page-locked host memory: SDMA copies on 1 / 2 / 4 streams, row-band and
// tile-rectangle 2D copies, and a blit kernel storing straight into host-mapped memory (default /
// non-coherent pinned allocations).  Decides how pgrt's host-output frames move their pixels.
// build: hipcc --offload-arch=gfx950 -O3 -o build/d2h_probe tools/d2h_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            return 1;                                                               \
        }                                                                           \
    } while (0)

__global__ void blit(const float4* __restrict__ src, float4* __restrict__ dst, long long n) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    const int W = 1920, H = 1080;
    const size_t bytes = (size_t)W * H * 16;
    float4* dev;
    CK(hipMalloc(&dev, bytes));
    CK(hipMemset(dev, 1, bytes));
    float4 *host_def, *host_nc;
    CK(hipHostMalloc((void**)&host_def, bytes, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&host_nc, bytes, hipHostMallocNonCoherent | hipHostMallocMapped));
    hipStream_t st[4];
    for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timed = [&](const char* name, auto&& body) -> int {
        std::vector<double> ms;
        for (int rep = 0; rep < 12; ++rep) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, st[0]));
            for (int k = 1; k < 4; ++k) CK(hipStreamWaitEvent(st[k], e0, 0));
            if (body() != 0) return 1;
            for (int k = 1; k < 4; ++k) {
                hipEvent_t ek;
                CK(hipEventCreate(&ek));
                CK(hipEventRecord(ek, st[k]));
                CK(hipStreamWaitEvent(st[0], ek, 0));
                CK(hipEventDestroy(ek));
            }
            CK(hipEventRecord(e1, st[0]));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (rep >= 2) ms.push_back(t);
        }
        const double m = median(ms);
        printf("%-52s %8.3f ms  %6.1f GB/s\n", name, m, bytes / (m * 1e-3) / 1e9);
        return 0;
    };
    for (int pass = 0; pass < 2; ++pass) {
        printf("-- pass %d\n", pass);
        for (int ns : {1, 2, 4}) {
            char name[96];
            snprintf(name, sizeof name, "hipMemcpyAsync D2H, %d stream(s), pinned default", ns);
            if (timed(name, [&]() -> int {
                    const size_t part = bytes / ns;
                    for (int k = 0; k < ns; ++k)
                        CK(hipMemcpyAsync((char*)host_def + k * part, (char*)dev + k * part,
                                          k == ns - 1 ? bytes - k * part : part, hipMemcpyDeviceToHost, st[k]));
                    return 0;
                }))
                return 1;
        }
        if (timed("hipMemcpyAsync D2H, 1 stream, pinned non-coherent", [&]() -> int {
                CK(hipMemcpyAsync(host_nc, dev, bytes, hipMemcpyDeviceToHost, st[0]));
                return 0;
            }))
            return 1;
        // 17 row bands of 64 rows (one 2D copy each), round-robin over 2 streams
        if (timed("hipMemcpy2DAsync, 17 row bands, 2 streams", [&]() -> int {
                for (int b = 0; b * 64 < H; ++b) {
                    const int rows = std::min(64, H - b * 64);
                    CK(hipMemcpy2DAsync((char*)host_def + (size_t)b * 64 * W * 16, W * 16,
                                        (char*)dev + (size_t)b * 64 * W * 16, W * 16, W * 16, rows,
                                        hipMemcpyDeviceToHost, st[b & 1]));
                }
                return 0;
            }))
            return 1;
        // one 2D copy per 64x64 tile (510 copies), 2 streams
        if (timed("hipMemcpy2DAsync, 510 tiles 64x64, 2 streams", [&]() -> int {
                int k = 0;
                for (int ty = 0; ty * 64 < H; ++ty)
                    for (int tx = 0; tx * 64 < W; ++tx, ++k) {
                        const int rows = std::min(64, H - ty * 64), cols = std::min(64, W - tx * 64);
                        const size_t off = ((size_t)ty * 64 * W + (size_t)tx * 64) * 16;
                        CK(hipMemcpy2DAsync((char*)host_def + off, W * 16, (char*)dev + off, W * 16, cols * 16, rows,
                                            hipMemcpyDeviceToHost, st[k & 1]));
                    }
                return 0;
            }))
            return 1;
        for (int grid : {32, 64, 128, 256, 1024}) {
            for (int nc = 0; nc < 2; ++nc) {
                float4* hp;
                CK(hipHostGetDevicePointer((void**)&hp, nc ? (void*)host_nc : (void*)host_def, 0));
                char name[96];
                snprintf(name, sizeof name, "blit kernel -> host-mapped %s, grid %d", nc ? "non-coherent" : "default", grid);
                if (timed(name, [&]() -> int {
                        hipLaunchKernelGGL(blit, dim3(grid), dim3(256), 0, st[0], dev, hp, (long long)(bytes / 16));
                        return 0;
                    }))
                    return 1;
            }
        }
        // SDMA and a blit kernel at once (half each)
        {
            float4* hp;
            CK(hipHostGetDevicePointer((void**)&hp, (void*)host_def, 0));
            if (timed("half SDMA (1 stream) + half blit kernel (grid 1024)", [&]() -> int {
                    const size_t half = bytes / 2;
                    CK(hipMemcpyAsync(host_def, dev, half, hipMemcpyDeviceToHost, st[1]));
                    hipLaunchKernelGGL(blit, dim3(1024), dim3(256), 0, st[0], (const float4*)((char*)dev + half),
                                       (float4*)((char*)hp + half), (long long)(half / 16));
                    return 0;
                }))
                return 1;
        }
    }
    printf("d2h probe done\n");
    return 0;
}
