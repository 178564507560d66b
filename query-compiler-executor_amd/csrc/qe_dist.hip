// qe_dist.hip -- primitives of the key-partitioned multi-GPU plan.
//
// Each rank owns a rowid slice of every relation (base columns replicated, so rowid gathers
// stay local).  Before each join the rows of both sides are hash-partitioned on the join key,
// dest = fmix64(key) % nparts, into contiguous per-destination segments of caller-provided
// send buffers; the caller moves them with one RCCL all-to-all per array (torch.distributed,
// backend "nccl" = RCCL over xGMI), then joins its own bucket locally with the single-GPU
// sort + merge kernels.  Checksums are added mod 2^64 and all-reduced.
#include <algorithm>

#include "qe_device.h"
#include "qe_internal.h"

namespace qe {

__host__ __device__ __forceinline__ uint64_t fmix64(uint64_t k) {   // murmur3 finaliser
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

constexpr int PB = 256;                 // block
constexpr int P_ITEMS = 8;
constexpr int PTILE = PB * P_ITEMS;     // rows per block
constexpr int PMAX = 64;                // max destinations
constexpr int PNW = PB / 64;

__global__ void __launch_bounds__(PB) part_count_kernel(const uint64_t* __restrict__ keys, uint64_t n, uint32_t nparts,
                                                        uint32_t* __restrict__ table /*[nblocks][nparts]*/) {
    __shared__ uint32_t h[PMAX];
    for (int i = threadIdx.x; i < PMAX; i += PB) h[i] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * PTILE;
#pragma unroll
    for (int j = 0; j < P_ITEMS; j++) {
        uint64_t i = base + (uint64_t)j * PB + threadIdx.x;
        if (i < n) atomicAdd(&h[fmix64(keys[i]) % nparts], 1u);
    }
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < nparts; p += PB) table[(uint64_t)blockIdx.x * nparts + p] = h[p];
}

// column-major exclusive scan of the [nblocks][nparts] table: offset of (block, dest) in the
// send buffer, destination segments contiguous; totals[p] = rows for dest p.  One block.
__global__ void __launch_bounds__(1024) part_scan_kernel(uint32_t* __restrict__ table, uint32_t nblocks,
                                                         uint32_t nparts, uint64_t* __restrict__ totals) {
    __shared__ uint64_t wsum[16];
    __shared__ uint64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t p = 0; p < nparts; p++) {
        uint64_t start = carry;
        for (uint32_t b0 = 0; b0 < nblocks; b0 += 1024) {
            uint32_t b = b0 + threadIdx.x;
            uint64_t x = b < nblocks ? table[(uint64_t)b * nparts + p] : 0;
            uint64_t inc = wave_incl_scan_u64(x);
            if (lane_id() == 63) wsum[wave_id()] = inc;
            __syncthreads();
            uint64_t add = carry;
            for (int w = 0; w < wave_id(); w++) add += wsum[w];
            if (b < nblocks) table[(uint64_t)b * nparts + p] = (uint32_t)(inc - x + add);   // rows < 2^32
            __syncthreads();
            if (threadIdx.x == 1023) carry = add + inc;
            __syncthreads();
        }
        if (threadIdx.x == 0) totals[p] = carry - start;
        __syncthreads();
    }
}

// rowid columns travel by value in the kernel arguments: pointers loaded from a device array
// would be generic (FLAT loads / stores)
struct PartCols {
    const uint32_t* in[4];
    uint32_t* out[4];
};

// stable scatter: element order is kept inside every destination segment
template <int NC>
__global__ void __launch_bounds__(PB) part_scatter_kernel(const uint64_t* __restrict__ keys, uint64_t n,
                                                          uint32_t nparts, const uint32_t* __restrict__ table,
                                                          PartCols pc, uint64_t* __restrict__ okeys) {
    __shared__ uint32_t cnt[P_ITEMS][PNW][PMAX];   // (step, wave, dest) counts -> exclusive prefix
    const int w = wave_id(), l = lane_id();
    const uint64_t lt = lanemask_lt();
    const uint64_t base = (uint64_t)blockIdx.x * PTILE;
    uint32_t dest[P_ITEMS], rank[P_ITEMS];
    uint64_t key[P_ITEMS];
#pragma unroll
    for (int j = 0; j < P_ITEMS; j++) {
        uint64_t i = base + (uint64_t)j * PB + threadIdx.x;
        bool ok = i < n;
        key[j] = ok ? keys[i] : 0;
        dest[j] = ok ? (uint32_t)(fmix64(key[j]) % nparts) : PMAX;
        uint32_t r = 0;
        for (uint32_t p = 0; p < nparts; p++) {
            uint64_t m = __ballot(dest[j] == p);
            if (dest[j] == p) r = (uint32_t)__popcll(m & lt);
            if (l == 0) cnt[j][w][p] = (uint32_t)__popcll(m);
        }
        rank[j] = r;
    }
    __syncthreads();
    // exclusive prefix over (step, wave) for each destination, starting at the block's offset
    for (uint32_t p = threadIdx.x; p < nparts; p += PB) {
        uint32_t run = table[(uint64_t)blockIdx.x * nparts + p];
        for (int j = 0; j < P_ITEMS; j++)
            for (int ww = 0; ww < PNW; ww++) {
                uint32_t c = cnt[j][ww][p];
                cnt[j][ww][p] = run;
                run += c;
            }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < P_ITEMS; j++) {
        uint64_t i = base + (uint64_t)j * PB + threadIdx.x;
        if (i < n) {
            uint32_t o = cnt[j][w][dest[j]] + rank[j];
            okeys[o] = key[j];
#pragma unroll
            for (int c = 0; c < NC; c++) pc.out[c][o] = pc.in[c][i];
        }
    }
}

__global__ void __launch_bounds__(256) iota_kernel(uint32_t* __restrict__ out, uint64_t start, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (uint32_t)(start + i);
}

__global__ void __launch_bounds__(256) take_u32_kernel(const uint32_t* __restrict__ src, const uint32_t* __restrict__ idx,
                                                       uint64_t n, uint32_t* __restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = src[idx[i]];
}

__global__ void __launch_bounds__(256) add_u32_kernel(uint32_t* __restrict__ a, uint64_t n, uint32_t add) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] += add;
}

}  // namespace qe

using namespace qe;

extern "C" {

int qe_partition(qe_ctx* c, const uint64_t* keys, uint64_t n, const uint32_t* const* cols, int ncols,
                 uint32_t nparts, uint64_t* counts, uint64_t* out_keys, uint32_t* const* out_cols) {
    QE_API_BEGIN(c)
    if (nparts < 1 || nparts > (uint32_t)PMAX) throw Error(QE_EINVAL, "nparts must be in [1, 64]");
    if (ncols < 0 || ncols > 4) throw Error(QE_EINVAL, "at most 4 rowid columns per partition call");
    if (n >= 0xFFFFFFFFull) throw Error(QE_EINVAL, "partition input too large");
    for (uint32_t p = 0; p < nparts; p++) counts[p] = 0;
    if (n == 0) return 0;
    const uint32_t nb = (uint32_t)((n + PTILE - 1) / PTILE);
    uint32_t* table = dalloc_t<uint32_t>(c, (uint64_t)nb * nparts);
    uint64_t* d_tot = dalloc_t<uint64_t>(c, nparts);
    PartCols pc{};
    for (int i = 0; i < ncols; i++) {
        pc.in[i] = cols[i];
        pc.out[i] = out_cols[i];
    }
    {
        Timed t(c, "partition", (8.0 + 4.0 * ncols) * 2.0 * n + 8.0 * n);
        hipLaunchKernelGGL(part_count_kernel, dim3(nb), dim3(PB), 0, c->stream, keys, n, nparts, table);
        QE_HIP(hipGetLastError());
        hipLaunchKernelGGL(part_scan_kernel, dim3(1), dim3(1024), 0, c->stream, table, nb, nparts, d_tot);
        QE_HIP(hipGetLastError());
        switch (ncols) {
#define QE_PS(NC)                                                                                              \
    case NC:                                                                                                   \
        hipLaunchKernelGGL(part_scatter_kernel<NC>, dim3(nb), dim3(PB), 0, c->stream, keys, n, nparts, table, \
                           pc, out_keys);                                                                      \
        break;
            QE_PS(0) QE_PS(1) QE_PS(2) QE_PS(3) QE_PS(4)
#undef QE_PS
        }
        QE_HIP(hipGetLastError());
    }
    QE_HIP(hipMemcpyAsync(counts, d_tot, nparts * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    QE_HIP(hipStreamSynchronize(c->stream));
    dfree(c, table);
    dfree(c, d_tot);
    return 0;
    QE_API_END(c)
}

int qe_filter_scan_range(qe_ctx* c, qe_col col, uint64_t start, uint64_t end, char op, uint64_t v, qe_list* out) {
    QE_API_BEGIN(c)
    if (end > col.n || start > end) throw Error(QE_EINVAL, "bad row range");
    if (op != '=' && op != '<' && op != '>') throw Error(QE_EINVAL, "Wrong operator");
    const uint64_t n = end - start;
    out->d = dalloc_t<uint32_t>(c, std::max<uint64_t>(n, 1));
    out->cap = n;
    out->n = filter_scan(c, col.d + start, n, op, v, out->d);
    if (start && out->n) {
        hipLaunchKernelGGL(add_u32_kernel, dim3(grid_for(out->n, 256)), dim3(256), 0, c->stream, out->d, out->n,
                           (uint32_t)start);
        QE_HIP(hipGetLastError());
    }
    out->flags = QE_LIST_DISTINCT;
    return 0;
    QE_API_END(c)
}

int qe_iota(qe_ctx* c, uint64_t start, uint64_t n, qe_list* out) {
    QE_API_BEGIN(c)
    out->d = dalloc_t<uint32_t>(c, std::max<uint64_t>(n, 1));
    out->n = out->cap = n;
    out->flags = QE_LIST_DISTINCT;
    if (n) {
        hipLaunchKernelGGL(iota_kernel, dim3(grid_for(n, 256)), dim3(256), 0, c->stream, out->d, start, n);
        QE_HIP(hipGetLastError());
    }
    return 0;
    QE_API_END(c)
}

int qe_take_u32(qe_ctx* c, const uint32_t* src, const qe_list* idx, qe_list* out) {
    QE_API_BEGIN(c)
    const uint64_t n = idx->n;
    out->d = dalloc_t<uint32_t>(c, std::max<uint64_t>(n, 1));
    out->n = out->cap = n;
    out->flags = 0;
    if (n) {
        Timed t(c, "take_u32", 12.0 * n);
        hipLaunchKernelGGL(take_u32_kernel, dim3(grid_for(n, 256)), dim3(256), 0, c->stream, src, idx->d, n, out->d);
        QE_HIP(hipGetLastError());
    }
    return 0;
    QE_API_END(c)
}

int qe_join_indices(qe_ctx* c, const uint64_t* keysA, uint64_t nA, const uint64_t* keysB, uint64_t nB, qe_list* ia,
                    qe_list* ib) {
    QE_API_BEGIN(c)
    qe_pairs A{const_cast<uint64_t*>(keysA), nullptr, nullptr, nA, 0, 0, QE_PAIRS_DISTINCT, 0};
    qe_pairs B{const_cast<uint64_t*>(keysB), nullptr, nullptr, nB, 0, 0, QE_PAIRS_DISTINCT, 0};
    int rc = qe_sort_pairs(c, &A);
    if (rc == 0) rc = qe_sort_pairs(c, &B);
    if (rc == 0) rc = qe_merge_join(c, &A, &B, ia, ib);
    qe_pairs_free(c, &A);
    qe_pairs_free(c, &B);
    return rc;
    QE_API_END(c)
}

int qe_sync_stream_ptr(qe_ctx* c, void** stream) {
    if (!c) return QE_EINVAL;
    *stream = (void*)c->stream;
    return 0;
}

}  // extern "C"
