// Micro-benchmark: the cost of the plan's random gathers under three HBM layouts of a relation.
//   col     -- the columnar layout: key = c0[r] (u64), later val = c2[r] (u64) in a second pass
//   col2    -- both columns in ONE kernel (two random line fetches per row)
//   rm32    -- a row-major u32 copy, 16 B per row: key and value from one 16 B slot
//   rm64    -- a row-major u64 copy, 32 B per row
// n rows of a 100M-row relation chosen at random (a hash of the index), 46.6M of them (C3's J2).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__device__ inline uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__global__ void init_kernel(uint64_t* c0, uint64_t* c1, uint64_t* c2, uint32_t* rm32, uint64_t* rm64, uint64_t N) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < N; i += (uint64_t)gridDim.x * 256) {
        const uint64_t a = hash32((uint32_t)i) % N, b = hash32((uint32_t)i ^ 0x5555u) % N,
                       d = hash32((uint32_t)i * 3u + 7u);
        c0[i] = a; c1[i] = b; c2[i] = d;
        reinterpret_cast<uint4*>(rm32)[i] = make_uint4((uint32_t)a, (uint32_t)b, (uint32_t)d, 0u);
        rm64[4 * i] = a; rm64[4 * i + 1] = b; rm64[4 * i + 2] = d; rm64[4 * i + 3] = 0;
    }
}

// P > 1: the rows partitioned into P ranges of the rowid space (partition p's rows contiguous)
__global__ void rows_kernel(uint32_t* rows, uint64_t n, uint64_t N, uint32_t P) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint32_t r = hash32((uint32_t)i * 2654435761u + 12345u) % (uint32_t)(N / P);
        const uint32_t p = (uint32_t)(i * P / n);
        rows[i] = p * (uint32_t)(N / P) + r;
    }
}

constexpr uint64_t N32 = 100000000ull;
template <int MODE>
__global__ void __launch_bounds__(256) gather_kernel(const uint64_t* __restrict__ c0, const uint64_t* __restrict__ c2,
                                                     const uint32_t* __restrict__ rm32, const uint64_t* __restrict__ rm64,
                                                     const uint32_t* __restrict__ rows, uint64_t n,
                                                     uint64_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    const uint64_t stride = (uint64_t)gridDim.x * 256 * 4;
    for (uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 4; i + 3 < n; i += stride) {
        const uint4 r = *reinterpret_cast<const uint4*>(rows + i);
        const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
        uint64_t k[4];
        uint32_t v[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (MODE == 0) { k[j] = c0[rr[j]]; v[j] = 0; }
            if (MODE == 1) { k[j] = 0; v[j] = (uint32_t)c2[rr[j]]; }
            if (MODE == 2) { k[j] = c0[rr[j]]; v[j] = (uint32_t)c2[rr[j]]; }
            if (MODE == 3) { const uint2 x = *reinterpret_cast<const uint2*>(rm32 + 4ull * rr[j]);
                             const uint32_t y = rm32[4ull * rr[j] + 2]; k[j] = x.x; v[j] = y; }
            if (MODE == 4) { k[j] = rm64[4ull * rr[j]]; v[j] = (uint32_t)rm64[4ull * rr[j] + 2]; }
            if (MODE == 5) { k[j] = rm32[rr[j]]; v[j] = 0; }                       // u32 column (rm32 reused as one)
            if (MODE == 6) { k[j] = rm32[rr[j]]; v[j] = rm32[N32 + rr[j]]; }        // two u32 columns
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (MODE != 1) keys[i + j] = k[j];
            if (MODE != 0) vals[i + j] = v[j];
        }
    }
}

int main() {
    const uint64_t N = 100000000ull, n = 46600000ull;
    uint64_t *c0, *c1, *c2, *rm64, *keys;
    uint32_t *rm32, *rows, *vals;
    CK(hipMalloc(&c0, N * 8)); CK(hipMalloc(&c1, N * 8)); CK(hipMalloc(&c2, N * 8));
    CK(hipMalloc(&rm32, N * 16)); CK(hipMalloc(&rm64, N * 32));
    CK(hipMalloc(&rows, n * 4)); CK(hipMalloc(&keys, n * 8)); CK(hipMalloc(&vals, n * 4));
    init_kernel<<<4096, 256>>>(c0, c1, c2, rm32, rm64, N);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const char* names[7] = {"col key only", "col value only", "col key+value (1 kernel)", "rm32 key+value",
                            "rm64 key+value", "u32 col key only", "u32 col key+value"};
    const int grid = 4096;
    for (uint32_t P : {1u, 4u, 16u, 64u, 256u}) {
        rows_kernel<<<4096, 256>>>(rows, n, N, P);
        CK(hipDeviceSynchronize());
        for (int mode = 0; mode < 7; mode++) {
            std::vector<float> ts;
            for (int rep = 0; rep < 6; rep++) {
                CK(hipEventRecord(a));
                switch (mode) {
                    case 0: gather_kernel<0><<<grid, 256>>>(c0, c2, rm32, rm64, rows, n, keys, vals); break;
                    case 1: gather_kernel<1><<<grid, 256>>>(c0, c2, rm32, rm64, rows, n, keys, vals); break;
                    case 2: gather_kernel<2><<<grid, 256>>>(c0, c2, rm32, rm64, rows, n, keys, vals); break;
                    case 3: gather_kernel<3><<<grid, 256>>>(c0, c2, rm32, rm64, rows, n, keys, vals); break;
                    case 4: gather_kernel<4><<<grid, 256>>>(c0, c2, rm32, rm64, rows, n, keys, vals); break;
                    case 5: gather_kernel<5><<<grid, 256>>>(c0, c2, rm32, rm64, rows, n, keys, vals); break;
                    case 6: gather_kernel<6><<<grid, 256>>>(c0, c2, rm32, rm64, rows, n, keys, vals); break;
                }
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                if (rep) ts.push_back(ms);
            }
            std::sort(ts.begin(), ts.end());
            printf("P %4u  %-28s median %.3f ms  min %.3f ms\n", P, names[mode], ts[ts.size() / 2], ts[0]);
        }
    }
    return 0;
}
