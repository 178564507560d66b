// gatherbench2.hip -- does an XCD-local bucketed gather beat a random one?  checksum-style
// sum of src[idx[i]] over 46.6 M indices into a 100 M-row u64 column: (a) indices random over
// the whole column, (b) indices grouped into B buckets of the row range (as one radix pass over
// the rowids' high bits would leave them), each bucket's gathers done by the blocks of ONE XCD
// (blockIdx % 8) so its 800/B MB slice of the column stays in that XCD's L2.  Tuning aid only.
// build: hipcc --offload-arch=gfx950 -O3 -o build/gatherbench2 tools/gatherbench2.hip
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

__device__ inline uint64_t mix(uint64_t i) {
    uint64_t h = (i + 0x9E3779B97F4A7C15ull) * 0xbf58476d1ce4e5b9ull;
    return h ^ (h >> 31);
}

// random: idx[i] uniform in [0, range); bucketed: segment s = i / seg holds indices of bucket s
__global__ void make_idx(uint32_t* idx, uint64_t n, uint64_t range, uint32_t nb) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t h = mix(i);
    if (nb <= 1) { idx[i] = (uint32_t)(h % range); return; }
    const uint64_t seg = (n + nb - 1) / nb, bw = (range + nb - 1) / nb;
    const uint64_t s = i / seg;
    uint64_t v = s * bw + h % bw;
    idx[i] = (uint32_t)(v < range ? v : range - 1);
}

__global__ void __launch_bounds__(256) sum_random(const uint64_t* __restrict__ col, const uint32_t* __restrict__ rows,
                                                  uint64_t n, unsigned long long* out) {
    uint64_t s = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256 * 8;
    for (uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 8; i + 7 < n; i += stride) {
        uint4 a = *reinterpret_cast<const uint4*>(rows + i);
        uint4 b = *reinterpret_cast<const uint4*>(rows + i + 4);
        s += col[a.x] + col[a.y] + col[a.z] + col[a.w] + col[b.x] + col[b.y] + col[b.z] + col[b.w];
    }
    __shared__ uint64_t red[4];
    for (int o = 32; o; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(out, (unsigned long long)(red[0] + red[1] + red[2] + red[3]));
}

// XCD x = blockIdx % 8 takes segments x, x + 8, ...; its blocks split each segment
__global__ void __launch_bounds__(256) sum_bucketed(const uint64_t* __restrict__ col,
                                                    const uint32_t* __restrict__ rows, uint64_t n, uint32_t nb,
                                                    unsigned long long* out) {
    const uint32_t x = blockIdx.x & 7, l = blockIdx.x >> 3, per = gridDim.x >> 3;
    const uint64_t seg = (n + nb - 1) / nb;
    uint64_t s = 0;
    for (uint32_t b = x; b < nb; b += 8) {
        const uint64_t lo = b * seg, hi = lo + seg < n ? lo + seg : n;
        for (uint64_t i = lo + ((uint64_t)l * 256 + threadIdx.x) * 8; i < hi; i += (uint64_t)per * 256 * 8) {
            if (i + 7 < hi) {
                uint4 a = *reinterpret_cast<const uint4*>(rows + i);
                uint4 c = *reinterpret_cast<const uint4*>(rows + i + 4);
                s += col[a.x] + col[a.y] + col[a.z] + col[a.w] + col[c.x] + col[c.y] + col[c.z] + col[c.w];
            } else {
                for (uint64_t k = i; k < hi; k++) s += col[rows[k]];
            }
        }
    }
    __shared__ uint64_t red[4];
    for (int o = 32; o; o >>= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(out, (unsigned long long)(red[0] + red[1] + red[2] + red[3]));
}

int main() {
    const uint64_t n = 46600000, range = 100000000;
    uint32_t* idx;
    uint64_t* src;
    unsigned long long* out;
    CK(hipMalloc(&idx, n * 4));
    CK(hipMalloc(&src, range * 8));
    CK(hipMalloc(&out, 8));
    CK(hipMemset(src, 1, range * 8));
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
        printf("%-52s %8.3f ms  %6.2f ps/elem\n", name, ms / it, ms / it * 1e9 / n);
    };
    char nm[96];
    hipLaunchKernelGGL(make_idx, dim3((n + 255) / 256), dim3(256), 0, 0, idx, n, range, 1u);
    for (unsigned g : {2048u, 4096u, 8192u}) {
        snprintf(nm, sizeof nm, "random, grid %u", g);
        time([&] { hipLaunchKernelGGL(sum_random, dim3(g), dim3(256), 0, 0, src, idx, n, out); }, nm);
    }
    for (uint32_t nb : {128u, 256u, 512u, 1024u, 2048u}) {
        hipLaunchKernelGGL(make_idx, dim3((n + 255) / 256), dim3(256), 0, 0, idx, n, range, nb);
        for (unsigned g : {1024u, 2048u, 4096u}) {
            snprintf(nm, sizeof nm, "bucketed %4u (%.2f MB slices), grid %u", nb, range * 8.0 / nb / 1e6, g);
            time([&] { hipLaunchKernelGGL(sum_bucketed, dim3(g), dim3(256), 0, 0, src, idx, n, nb, out); }, nm);
        }
        snprintf(nm, sizeof nm, "bucketed %4u, plain grid-stride (no XCD map)", nb);
        time([&] { hipLaunchKernelGGL(sum_random, dim3(4096), dim3(256), 0, 0, src, idx, n, out); }, nm);
    }
    CK(hipDeviceSynchronize());
    return 0;
}
