// readbench.hip -- calibration (not product code): read-only streaming bandwidth of the access
// shapes the scan kernels use, over 0.8 GB and 6.4 GB of u64.
// build: hipcc --offload-arch=gfx950 -O3 -o build/readbench tools/readbench.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)

// grid-stride, each thread ITEMS x 16-B loads per iteration
template <int ITEMS>
__global__ void __launch_bounds__(512) rd_stride(const uint64_t* __restrict__ in, uint64_t n, unsigned long long* out) {
    uint64_t acc = 0;
    const uint64_t T = 512ull * ITEMS * 2, stride = (uint64_t)gridDim.x * T;
    for (uint64_t t = (uint64_t)blockIdx.x * T; t < n; t += stride) {
        ulonglong2 x[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            uint64_t i = t + (uint64_t)j * 1024 + 2ull * threadIdx.x;
            x[j] = i + 1 < n ? *reinterpret_cast<const ulonglong2*>(in + i) : ulonglong2{0, 0};
        }
#pragma unroll
        for (int j = 0; j < ITEMS; j++) acc ^= x[j].x + x[j].y;
    }
    if (acc == 0x123456789ull) atomicAdd(out, 1ull);
}

// one tile per block
template <int ITEMS>
__global__ void __launch_bounds__(512) rd_tile(const uint64_t* __restrict__ in, uint64_t n, unsigned long long* out) {
    uint64_t acc = 0;
    const uint64_t t = (uint64_t)blockIdx.x * 512ull * ITEMS * 2;
    ulonglong2 x[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        uint64_t i = t + (uint64_t)j * 1024 + 2ull * threadIdx.x;
        x[j] = i + 1 < n ? *reinterpret_cast<const ulonglong2*>(in + i) : ulonglong2{0, 0};
    }
#pragma unroll
    for (int j = 0; j < ITEMS; j++) acc ^= x[j].x + x[j].y;
    if (acc == 0x123456789ull) atomicAdd(out, 1ull);
}

int main() {
    const uint64_t N = 800000000ull;
    uint64_t* a;
    unsigned long long* o;
    CK(hipMalloc(&a, N * 8));
    CK(hipMalloc(&o, 8));
    CK(hipMemset(a, 1, N * 8));
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
        printf("%-44s %8.3f ms  %8.1f GB/s\n", name, ms / it, bytes / (ms / it * 1e-3) / 1e9);
    };
    for (uint64_t n : {N / 8, N}) {
        char nm[96];
        for (int g : {512, 1024, 2048, 4096}) {
            snprintf(nm, sizeof nm, "stride4 grid %d n %llu", g, (unsigned long long)n);
            time([&] { hipLaunchKernelGGL(rd_stride<4>, dim3(g), dim3(512), 0, 0, a, n, o); }, 8.0 * n, nm);
            snprintf(nm, sizeof nm, "stride8 grid %d n %llu", g, (unsigned long long)n);
            time([&] { hipLaunchKernelGGL(rd_stride<8>, dim3(g), dim3(512), 0, 0, a, n, o); }, 8.0 * n, nm);
        }
        snprintf(nm, sizeof nm, "tile4 n %llu", (unsigned long long)n);
        time([&] { hipLaunchKernelGGL(rd_tile<4>, dim3((n + 4095) / 4096), dim3(512), 0, 0, a, n, o); }, 8.0 * n, nm);
        snprintf(nm, sizeof nm, "tile8 n %llu", (unsigned long long)n);
        time([&] { hipLaunchKernelGGL(rd_tile<8>, dim3((n + 8191) / 8192), dim3(512), 0, 0, a, n, o); }, 8.0 * n, nm);
    }
    return 0;
}
