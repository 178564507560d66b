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


// ---- local bucket select: the hash bucket `part` of a replicated base column ----------------------
// Base columns are replicated on every rank, so a join side that is a whole base
// relation is bucketed by one scan of the column instead of an exchange: rank g keeps the rows
// with fmix64(key) % nparts == g -- exactly the rows the exchange would have delivered to it.
// Unordered compaction (the bucket is sorted next): per (step, wave) survivor runs are ranked with
// ballots, the block reserves its range with one atomic, every wave writes its runs contiguously.
// Keys listed in `heavy` (sorted, skew path) are left out of every bucket.
constexpr int BS_B = 512;
constexpr int BS_ITEMS = 4;                 // x 2 keys per 16-B load
constexpr int BS_TILE = BS_B * BS_ITEMS * 2;
constexpr int BS_NW = BS_B / 64;
constexpr int HEAVY_MAX = 1024;

__device__ __forceinline__ int heavy_find(const uint64_t* h, uint32_t nh, uint64_t k) {
    // lower bound over the sorted heavy list (LDS); -1 when absent
    uint32_t lo = 0, len = nh;
    while (len > 0) {
        uint32_t half = len >> 1;
        bool go = h[lo + half] < k;
        lo = go ? lo + half + 1 : lo;
        len = go ? len - half - 1 : half;
    }
    return (lo < nh && h[lo] == k) ? (int)lo : -1;
}

__global__ void __launch_bounds__(BS_B) bucket_select_kernel(const uint64_t* __restrict__ keys, uint64_t n,
                                                             uint32_t nparts, uint32_t part,
                                                             const uint64_t* __restrict__ heavy, uint32_t nheavy,
                                                             uint64_t* __restrict__ okeys, uint32_t* __restrict__ ovals,
                                                             uint64_t cap, unsigned long long* __restrict__ counter) {
    __shared__ uint64_t s_heavy[HEAVY_MAX];
    __shared__ uint32_t s_cnt[BS_ITEMS * 2 * BS_NW];
    __shared__ uint64_t s_base;
    for (uint32_t i = threadIdx.x; i < nheavy; i += BS_B) s_heavy[i] = heavy[i];
    const int w = wave_id(), l = lane_id();
    const uint64_t lt = lanemask_lt();
    const uint64_t tile = (uint64_t)blockIdx.x * BS_TILE;
    uint64_t k[BS_ITEMS][2];
#pragma unroll
    for (int j = 0; j < BS_ITEMS; j++) {
        const uint64_t i = tile + (uint64_t)j * (BS_B * 2) + (uint64_t)threadIdx.x * 2;
        if (i + 1 < n) {
            ulonglong2 x = *reinterpret_cast<const ulonglong2*>(keys + i);
            k[j][0] = x.x;
            k[j][1] = x.y;
        } else {
            k[j][0] = i < n ? keys[i] : 0;
            k[j][1] = 0;
        }
    }
    __syncthreads();   // s_heavy
    bool f[BS_ITEMS][2];
    uint32_t rank[BS_ITEMS][2];
#pragma unroll
    for (int j = 0; j < BS_ITEMS; j++) {
        const uint64_t i = tile + (uint64_t)j * (BS_B * 2) + (uint64_t)threadIdx.x * 2;
#pragma unroll
        for (int v = 0; v < 2; v++) {
            bool ok = i + v < n && (uint32_t)(fmix64(k[j][v]) % nparts) == part;
            if (ok && nheavy) ok = heavy_find(s_heavy, nheavy, k[j][v]) < 0;
            f[j][v] = ok;
            uint64_t m = __ballot(ok);
            rank[j][v] = (uint32_t)__popcll(m & lt);
            if (l == 0) s_cnt[(j * 2 + v) * BS_NW + w] = (uint32_t)__popcll(m);
        }
    }
    __syncthreads();
    if (w == 0) {
        constexpr int NC = BS_ITEMS * 2 * BS_NW;
        uint32_t c = l < NC ? s_cnt[l] : 0;
        uint32_t inc = wave_incl_scan_u32(c);
        uint32_t total = (uint32_t)__shfl((int)inc, NC - 1, 64);
        if (l < NC) s_cnt[l] = inc - c;
        if (l == 0) s_base = total ? atomicAdd(counter, (unsigned long long)total) : 0;
    }
    __syncthreads();
    const uint64_t base = s_base;
#pragma unroll
    for (int j = 0; j < BS_ITEMS; j++) {
        const uint64_t i = tile + (uint64_t)j * (BS_B * 2) + (uint64_t)threadIdx.x * 2;
#pragma unroll
        for (int v = 0; v < 2; v++) {
            const uint64_t o = base + s_cnt[(j * 2 + v) * BS_NW + w] + rank[j][v];
            if (f[j][v] && o < cap) {   // an overfull bucket is counted, not written, and re-run
                okeys[o] = k[j][v];
                ovals[o] = (uint32_t)(i + v);
            }
        }
    }
}

// ---- heavy-key statistics over a row range (skew path) ---------------------------------------------
// counts[h] += #rows with key heavy[h]; wsum += sum of vals[row] * weights[h] over those rows (mod 2^64).
__global__ void __launch_bounds__(BS_B) heavy_stats_kernel(const uint64_t* __restrict__ keys,
                                                           const uint64_t* __restrict__ vals, uint64_t start,
                                                           uint64_t end, const uint64_t* __restrict__ heavy,
                                                           uint32_t nheavy, const uint64_t* __restrict__ weights,
                                                           unsigned long long* __restrict__ counts,
                                                           unsigned long long* __restrict__ wsum) {
    __shared__ uint64_t s_heavy[HEAVY_MAX];
    __shared__ uint32_t s_cnt[HEAVY_MAX];
    __shared__ uint64_t s_red[BS_NW];
    for (uint32_t i = threadIdx.x; i < nheavy; i += BS_B) {
        s_heavy[i] = heavy[i];
        s_cnt[i] = 0;
    }
    __syncthreads();
    const uint64_t tile = start + (uint64_t)blockIdx.x * BS_TILE;
    uint64_t acc = 0;
#pragma unroll
    for (int j = 0; j < BS_ITEMS * 2; j++) {
        const uint64_t i = tile + (uint64_t)j * BS_B + threadIdx.x;
        if (i < end) {
            const int h = heavy_find(s_heavy, nheavy, keys[i]);
            if (h >= 0) {
                atomicAdd(&s_cnt[h], 1u);
                if (weights) acc += vals[i] * weights[h];
            }
        }
    }
    if (weights) {
        acc = wave_sum_u64(acc);
        if (lane_id() == 0) s_red[wave_id()] = acc;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nheavy; i += BS_B)
        if (s_cnt[i]) atomicAdd(&counts[i], (unsigned long long)s_cnt[i]);
    if (weights && threadIdx.x == 0) {
        uint64_t t = 0;
        for (int x = 0; x < BS_NW; x++) t += s_red[x];
        if (t) atomicAdd(wsum, (unsigned long long)t);
    }
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

int qe_bucket_select(qe_ctx* c, qe_col col, uint32_t nparts, uint32_t part, const uint64_t* heavy, uint32_t nheavy,
                     qe_pairs* out) {
    QE_API_BEGIN(c)
    if (nparts < 1 || part >= nparts) throw Error(QE_EINVAL, "bad bucket");
    if (nheavy > (uint32_t)HEAVY_MAX) throw Error(QE_EINVAL, "at most 1024 heavy keys");
    if (col.n >= 0xFFFFFFFFull) throw Error(QE_EINVAL, "column too large for 32-bit rowids");
    for (uint32_t i = 1; i < nheavy; i++)
        if (heavy[i - 1] >= heavy[i]) throw Error(QE_EINVAL, "heavy keys must be sorted and distinct");
    *out = qe_pairs{};
    const uint64_t n = col.n;
    // capacity: the whole column when nparts == 1, else the expected bucket + a generous margin
    // (the count is checked below; an overfull bucket re-runs with full capacity)
    uint64_t cap = nparts == 1 ? n : std::min<uint64_t>(n, n / nparts + n / (4 * nparts) + 65536);
    uint64_t* d_heavy = nullptr;
    if (nheavy) {
        d_heavy = dalloc_t<uint64_t>(c, nheavy);
        QE_HIP(hipMemcpyAsync(d_heavy, heavy, nheavy * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
    }
    unsigned long long* d_cnt = reinterpret_cast<unsigned long long*>(c->d_scratch);
    const unsigned nb = grid_for(n, BS_TILE);
    for (int attempt = 0; attempt < 2; attempt++) {
        out->key = dalloc_t<uint64_t>(c, std::max<uint64_t>(cap, 1));
        out->val = dalloc_t<uint32_t>(c, std::max<uint64_t>(cap, 1));
        QE_HIP(hipMemsetAsync(d_cnt, 0, sizeof(uint64_t), c->stream));
        if (n) {
            Timed t(c, "bucket_select", 8.0 * n);
            hipLaunchKernelGGL(bucket_select_kernel, dim3(nb), dim3(BS_B), 0, c->stream, col.d, n, nparts, part,
                               d_heavy, nheavy, out->key, out->val, cap, d_cnt);
            QE_HIP(hipGetLastError());
        }
        const uint64_t m = read_u64(c, reinterpret_cast<uint64_t*>(d_cnt));
        if (m <= cap) {
            out->n = m;
            break;
        }
        dfree(c, out->key);
        dfree(c, out->val);
        if (attempt == 1) throw Error(QE_EINVAL, "internal: bucket larger than its column");
        cap = n;
    }
    if (c->prof && !c->pending.empty()) c->pending.back().bytes += 12.0 * out->n;
    out->owns = 3;
    out->flags = QE_PAIRS_DISTINCT;
    if (d_heavy) dfree(c, d_heavy);
    return 0;
    QE_API_END(c)
}

int qe_heavy_stats(qe_ctx* c, qe_col keys, uint64_t start, uint64_t end, const uint64_t* heavy, uint32_t nheavy,
                   qe_col vals, const uint64_t* weights, uint64_t* counts, uint64_t* wsum) {
    QE_API_BEGIN(c)
    if (end > keys.n || start > end) throw Error(QE_EINVAL, "bad row range");
    if (nheavy > (uint32_t)HEAVY_MAX) throw Error(QE_EINVAL, "at most 1024 heavy keys");
    if (weights && (!vals.d || vals.n < end)) throw Error(QE_EINVAL, "weighted sum needs a value column");
    for (uint32_t i = 1; i < nheavy; i++)
        if (heavy[i - 1] >= heavy[i]) throw Error(QE_EINVAL, "heavy keys must be sorted and distinct");
    if (wsum) *wsum = 0;
    if (counts)
        for (uint32_t i = 0; i < nheavy; i++) counts[i] = 0;
    if (nheavy == 0 || end == start) return 0;
    // device block: [heavy | weights | counts | wsum]
    uint64_t* d = dalloc_t<uint64_t>(c, 3 * (uint64_t)nheavy + 1);
    QE_HIP(hipMemcpyAsync(d, heavy, nheavy * 8, hipMemcpyHostToDevice, c->stream));
    if (weights) QE_HIP(hipMemcpyAsync(d + nheavy, weights, nheavy * 8, hipMemcpyHostToDevice, c->stream));
    QE_HIP(hipMemsetAsync(d + 2 * nheavy, 0, (nheavy + 1) * 8, c->stream));
    {
        const uint64_t n = end - start;
        Timed t(c, "heavy_stats", 8.0 * n);
        hipLaunchKernelGGL(heavy_stats_kernel, dim3(grid_for(n, BS_TILE)), dim3(BS_B), 0, c->stream, keys.d,
                           vals.d, start, end, d, nheavy, weights ? d + nheavy : nullptr,
                           reinterpret_cast<unsigned long long*>(d + 2 * nheavy),
                           reinterpret_cast<unsigned long long*>(d + 3 * nheavy));
        QE_HIP(hipGetLastError());
    }
    std::vector<uint64_t> h(nheavy + 1);
    QE_HIP(hipMemcpyAsync(h.data(), d + 2 * nheavy, (nheavy + 1) * 8, hipMemcpyDeviceToHost, c->stream));
    QE_HIP(hipStreamSynchronize(c->stream));
    if (counts)
        for (uint32_t i = 0; i < nheavy; i++) counts[i] = h[i];
    if (wsum) *wsum = h[nheavy];
    dfree(c, d);
    return 0;
    QE_API_END(c)
}

int qe_sync_stream_ptr(qe_ctx* c, void** stream) {
    if (!c) return QE_EINVAL;
    *stream = (void*)c->stream;
    return 0;
}

}  // extern "C"
