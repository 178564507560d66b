// gatherbench.hip -- calibration for the random-gather kernels (take, key gathers, checksums):
// out[i] = src[idx[i]] with idx a pseudo-random map, by element width, source size (Infinity
// Cache-resident or not) and gathers in flight per thread.  Tuning aid, not product code.
// build: hipcc --offload-arch=gfx950 -O3 -o build/gatherbench tools/gatherbench.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            printf("HIP %s\n", hipGetErrorString(e));                          \
            return 1;                                                          \
        }                                                                      \
    } while (0)

__global__ void make_idx(uint32_t* idx, uint64_t n, uint64_t range) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        uint64_t h = (i + 0x9E3779B97F4A7C15ull) * 0xbf58476d1ce4e5b9ull;
        h ^= h >> 31;
        idx[i] = (uint32_t)(h % range);
    }
}

// K gathers per thread, their loads issued before any is used; 16-B index loads when K % 4 == 0
template <typename T, int K>
__global__ void __launch_bounds__(256) gather_kernel(const T* __restrict__ src, const uint32_t* __restrict__ idx,
                                                     uint64_t n, T* __restrict__ out) {
    const uint64_t base = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * K;
    if (base + K > n) return;
    uint32_t ix[K];
    if (K % 4 == 0) {
#pragma unroll
        for (int q = 0; q < K / 4; q++) {
            uint4 v = *reinterpret_cast<const uint4*>(idx + base + 4 * q);
            ix[4 * q] = v.x; ix[4 * q + 1] = v.y; ix[4 * q + 2] = v.z; ix[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < K; q++) ix[q] = idx[base + q];
    }
    T v[K];
#pragma unroll
    for (int q = 0; q < K; q++) v[q] = src[ix[q]];
#pragma unroll
    for (int q = 0; q < K; q++) out[base + q] = v[q];
}

int main() {
    const uint64_t n = 46600000;   // C3's join outputs
    uint32_t* idx;
    uint64_t *src, *out;
    const uint64_t maxsrc = 100000000;
    CK(hipMalloc(&idx, n * 4));
    CK(hipMalloc(&src, maxsrc * 8));
    CK(hipMalloc(&out, n * 8));
    CK(hipMemset(src, 1, maxsrc * 8));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto time = [&](auto launch, const char* name) {
        for (int w = 0; w < 2; w++) launch();
        hipEventRecord(e0);
        const int it = 10;
        for (int r = 0; r < it; r++) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-44s %8.3f ms  %6.2f ps/elem\n", name, ms / it, ms / it * 1e9 / n);
    };
    for (uint64_t range : {8000000ull, 46600000ull, 100000000ull}) {
        hipLaunchKernelGGL(make_idx, dim3((n + 255) / 256), dim3(256), 0, 0, idx, n, range);
        char nm[96];
#define RUN(T, K)                                                                                                  \
        snprintf(nm, sizeof nm, "%s gather, src %5.0f MB, %d in flight", sizeof(T) == 4 ? "u32" : "u64",          \
                 range * sizeof(T) / 1e6, K);                                                                      \
        time([&] { hipLaunchKernelGGL((gather_kernel<T, K>), dim3((unsigned)(n / K / 256)), dim3(256), 0, 0,     \
                                      (const T*)src, idx, n, (T*)out); }, nm);
        RUN(uint32_t, 1) RUN(uint32_t, 4) RUN(uint32_t, 8) RUN(uint32_t, 16)
        RUN(uint64_t, 1) RUN(uint64_t, 4) RUN(uint64_t, 8)
    }
    return 0;
}
