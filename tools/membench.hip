// membench.hip -- calibration microbenchmarks for the sort/merge kernel design (not product
// code): streaming copy bandwidth by access width, and a tile-local digit scatter.
// build: hipcc --offload-arch=gfx950 -O3 -o build/membench tools/membench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)

template <typename T>
__global__ void copy_kernel(const T* __restrict__ in, T* __restrict__ out, uint64_t n) {
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = in[i];
}

// per block: a tile of 4096 u64 read coalesced (8 B/lane), written as runs of 16 (random run order)
__global__ void runs_kernel(const uint64_t* __restrict__ in, uint64_t* __restrict__ out, uint64_t n,
                            const uint32_t* __restrict__ perm, int runlen) {
    uint64_t base = (uint64_t)blockIdx.x * 4096;
    for (int i = threadIdx.x; i < 4096; i += 256) {
        uint64_t k = base + i;
        if (k >= n) break;
        uint32_t run = i / runlen, off = i % runlen;
        uint64_t dst = (uint64_t)perm[(base / runlen + run) % (n / runlen)] * runlen + off;
        out[dst] = in[k];
    }
}

int main() {
    const uint64_t n = 100000000ull;   // 0.8 GB of u64
    uint64_t *a, *b;
    uint32_t* perm;
    CK(hipMalloc(&a, n * 8));
    CK(hipMalloc(&b, n * 8));
    CK(hipMemset(a, 1, n * 8));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto time = [&](auto launch, double bytes, const char* name) {
        for (int w = 0; w < 2; w++) launch();
        hipEventRecord(e0);
        const int it = 10;
        for (int r = 0; r < it; r++) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-40s %8.3f ms  %8.1f GB/s\n", name, ms / it, bytes / (ms / it * 1e-3) / 1e9);
    };
    for (int g : {1024, 2048, 4096, 8192, 16384}) {
        char nm[64];
        snprintf(nm, 64, "copy u32 (4B/lane) grid %d", g);
        time([&] { hipLaunchKernelGGL(copy_kernel<uint32_t>, dim3(g), dim3(256), 0, 0, (const uint32_t*)a, (uint32_t*)b, 2 * n); }, 16.0 * n, nm);
        snprintf(nm, 64, "copy u64 (8B/lane) grid %d", g);
        time([&] { hipLaunchKernelGGL(copy_kernel<uint64_t>, dim3(g), dim3(256), 0, 0, a, b, n); }, 16.0 * n, nm);
        snprintf(nm, 64, "copy u128 (16B/lane) grid %d", g);
        time([&] { hipLaunchKernelGGL(copy_kernel<ulonglong2>, dim3(g), dim3(256), 0, 0, (const ulonglong2*)a, (ulonglong2*)b, n / 2); }, 16.0 * n, nm);
    }
    // runs scatter
    std::vector<uint32_t> hp(n / 8);
    for (uint64_t i = 0; i < hp.size(); i++) hp[i] = (uint32_t)((i * 2654435761ull) % hp.size());
    CK(hipMalloc(&perm, hp.size() * 4));
    for (int rl : {8, 16, 32, 64}) {
        std::vector<uint32_t> q(n / rl);
        for (uint64_t i = 0; i < q.size(); i++) q[i] = (uint32_t)((i * 2654435761ull) % q.size());
        CK(hipMemcpy(perm, q.data(), q.size() * 4, hipMemcpyHostToDevice));
        char nm[64];
        snprintf(nm, 64, "scatter runs of %d u64", rl);
        time([&] { hipLaunchKernelGGL(runs_kernel, dim3((unsigned)((n + 4095) / 4096)), dim3(256), 0, 0, a, b, n, perm, rl); }, 16.0 * n, nm);
    }
    return 0;
}
