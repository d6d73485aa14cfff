// numa_probe.hip -- does the NUMA node of a page-locked host framebuffer decide its device-to-host
// bandwidth?  For one C2 framebuffer (33.2 MB RGBA f32): the process's CPU and allowed CPUs, the
// GPU's node (sysfs), then for hipHostMalloc memory and for mmap'd memory bound (mbind) to each
// node and registered with hipHostRegister: the node its pages landed on, SDMA (hipMemcpyAsync)
// and blit-kernel GB/s.  No libnuma: raw mbind / move_pages system calls.
// build: hipcc --offload-arch=gfx950 -O3 -o build/numa_probe tools/numa_probe.hip
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            fprintf(stderr, "%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            return 1;                                                                            \
        }                                                                                        \
    } while (0)

__global__ void blit(const float4* __restrict__ src, float4* __restrict__ dst, long long n) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

static int page_node(void* p) {
    void* pages[1] = {p};
    int status[1] = {-99};
    if (syscall(SYS_move_pages, 0, 1UL, pages, nullptr, status, 0) != 0) return -98;
    return status[0];
}

static int nodes_of(char* p, size_t bytes, int* hist, int nh) {
    for (int k = 0; k < nh; ++k) hist[k] = 0;
    for (size_t off = 0; off < bytes; off += (size_t)1 << 20) {
        const int n = page_node(p + off);
        if (n >= 0 && n < nh) ++hist[n];
    }
    return 0;
}

int main() {
    const int W = 1920, H = 1080;
    const size_t bytes = (size_t)W * H * 16;
    char bus[64] = {0};
    CK(hipDeviceGetPCIBusId(bus, sizeof bus, 0));
    for (char* c = bus; *c; ++c) *c = (char)tolower(*c);
    int gpu_node = -1;
    {
        char path[160];
        snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
        if (FILE* f = fopen(path, "r")) {
            if (fscanf(f, "%d", &gpu_node) != 1) gpu_node = -1;
            fclose(f);
        }
    }
    int nnodes = 0;
    for (int k = 0; k < 64; ++k) {
        char path[96];
        snprintf(path, sizeof path, "/sys/devices/system/node/node%d", k);
        if (access(path, F_OK) == 0) nnodes = k + 1;
    }
    cpu_set_t cs;
    CPU_ZERO(&cs);
    sched_getaffinity(0, sizeof cs, &cs);
    printf("gpu %s numa_node %d; host nodes %d; running on cpu %d; allowed cpus %d\n", bus, gpu_node, nnodes,
           sched_getcpu(), CPU_COUNT(&cs));
    float4* dev;
    CK(hipMalloc(&dev, bytes));
    CK(hipMemset(dev, 1, bytes));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto measure = [&](const char* name, char* host) -> int {
        int hist[16];
        nodes_of(host, bytes, hist, 16);
        float4* hp;
        CK(hipHostGetDevicePointer((void**)&hp, host, 0));
        double best[2] = {0, 0};
        for (int mode = 0; mode < 2; ++mode) {
            std::vector<double> ms;
            for (int rep = 0; rep < 10; ++rep) {
                CK(hipEventRecord(e0, st));
                if (mode == 0)
                    CK(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, st));
                else
                    hipLaunchKernelGGL(blit, dim3(256), dim3(256), 0, st, dev, hp, (long long)(bytes / 16));
                CK(hipEventRecord(e1, st));
                CK(hipEventSynchronize(e1));
                float t;
                CK(hipEventElapsedTime(&t, e0, e1));
                if (rep >= 2) ms.push_back(t);
            }
            std::sort(ms.begin(), ms.end());
            best[mode] = bytes / (ms[ms.size() / 2] * 1e-3) / 1e9;
        }
        printf("%-40s pages/MB on node:", name);
        for (int k = 0; k < std::max(nnodes, 1) && k < 16; ++k) printf(" %d", hist[k]);
        printf("   SDMA %6.1f GB/s   blit %6.1f GB/s\n", best[0], best[1]);
        return 0;
    };
    {
        char* h;
        CK(hipHostMalloc((void**)&h, bytes, hipHostMallocDefault));
        if (measure("hipHostMalloc default", h)) return 1;
        CK(hipHostFree(h));
    }
    {
        char* h;
        CK(hipHostMalloc((void**)&h, bytes, hipHostMallocNumaUser));
        if (measure("hipHostMalloc NumaUser", h)) return 1;
        CK(hipHostFree(h));
    }
    for (int node = 0; node < nnodes && node < 8; ++node) {
        char* h = (char*)mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (h == MAP_FAILED) return 1;
        unsigned long mask[4] = {0, 0, 0, 0};
        mask[node / 64] = 1UL << (node % 64);
        const long rc = syscall(SYS_mbind, h, bytes, 2 /*MPOL_BIND*/, mask, 256UL, 0U);
        memset(h, 0, bytes);  // first touch under the policy
        CK(hipHostRegister(h, bytes, hipHostRegisterMapped));
        char name[64];
        snprintf(name, sizeof name, "mmap + mbind(node %d)%s + register", node, rc ? " FAILED" : "");
        if (measure(name, h)) return 1;
        CK(hipHostUnregister(h));
        munmap(h, bytes);
    }
    printf("numa probe done\n");
    return 0;
}
