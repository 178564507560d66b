// qe_dist.hip -- primitives of the key-partitioned multi-GPU plan.
//
// Each rank owns a rowid slice of every relation (base columns replicated, so rowid gathers
// stay local).  Before each join the rows of both sides are hash-partitioned on the join key,
// dest = part_of(key) = (hi32(mix(key)) * nparts) >> 32, into contiguous per-destination segments of caller-provided
// send buffers; the caller moves them with one RCCL all-to-all per array (torch.distributed,
// backend "nccl" = RCCL over xGMI), then joins its own bucket locally with the single-GPU
// sort + merge kernels.  Checksums are added mod 2^64 and all-reduced.
#include <algorithm>

#include <algorithm>
#include <vector>

#include <chrono>

#include "qe_device.h"
#include "qe_internal.h"

namespace qe {

// destination of a key: one xor-shift-multiply mix (splitmix64's first round), its high half
// scaled to [0, nparts) by a multiply -- a few VALU ops per key.  (murmur3's full finaliser plus
// a 64-bit modulo -- a software division on gfx950 -- made the 8-way bucket scan ALU-bound.)
__host__ __device__ __forceinline__ uint32_t part_of(uint64_t k, uint32_t nparts) {
    const uint64_t h = (k ^ (k >> 29)) * 0xbf58476d1ce4e5b9ull;
    return (uint32_t)(((h >> 32) * (uint64_t)nparts) >> 32);
}

constexpr int PMAX = 64;                // max destinations
constexpr int PB = 512;                 // block
constexpr int P_ITEMS = 8;              // rows per thread (strided by PB: coalesced)
constexpr int PTILE = PB * P_ITEMS;     // rows per tile
constexpr int PNW = PB / 64;

// lanes of this wave holding the same destination (match-any from log2(nparts) ballots)
__device__ __forceinline__ uint64_t dest_peers(uint32_t d, bool ok, int dbits) {
    uint64_t peers = __ballot(ok);
    for (int b = 0; b < dbits; b++) {
        const bool bit = (d >> b) & 1u;
        const uint64_t mm = __ballot(bit);
        peers &= bit ? mm : ~mm;
    }
    return peers;
}

// rows per destination: per-wave match-any, one LDS add per (wave, item, distinct dest), one
// global add per (block, dest)
// KI: the keys' width in memory (u32: a side gathered as u32 keys, PreHist::k32) -- the destination
// is the value's, whatever the width (part_of of the value widened)
template <typename KI>
__global__ void __launch_bounds__(PB) part_count_kernel(const KI* __restrict__ keys, uint64_t n, uint32_t nparts,
                                                        int dbits, unsigned long long* __restrict__ counts) {
    // a capped grid (one global add per (block, dest): ~88 adds per us per word) walking tiles of
    // PTILE x 2 rows, 16-B loads, the next tile's loads issued before this one is counted
    __shared__ uint32_t h[PMAX];
    for (int i = threadIdx.x; i < PMAX; i += PB) h[i] = 0;
    __syncthreads();
    const int l = lane_id();
    constexpr uint64_t T2 = 2ull * PTILE;
    const uint64_t stride = (uint64_t)gridDim.x * T2;
    auto load = [&](uint64_t tile, uint64_t (&k)[P_ITEMS][2]) {
#pragma unroll
        for (int j = 0; j < P_ITEMS; j++) {
            const uint64_t i = tile + (uint64_t)j * (2 * PB) + 2ull * threadIdx.x;
            if (i + 1 < n) {
                if constexpr (sizeof(KI) == 8) {
                    ulonglong2 x = *reinterpret_cast<const ulonglong2*>(keys + i);
                    k[j][0] = x.x;
                    k[j][1] = x.y;
                } else {
                    uint2 x = *reinterpret_cast<const uint2*>(keys + i);
                    k[j][0] = x.x;
                    k[j][1] = x.y;
                }
            } else {
                k[j][0] = i < n ? keys[i] : 0;
                k[j][1] = 0;
            }
        }
    };
    uint64_t k[P_ITEMS][2], kn[P_ITEMS][2];
    uint64_t tile = (uint64_t)blockIdx.x * T2;
    if (tile < n) load(tile, k);
    for (; tile < n; tile += stride) {
        if (tile + stride < n) load(tile + stride, kn);
#pragma unroll
        for (int j = 0; j < P_ITEMS; j++) {
#pragma unroll
            for (int v = 0; v < 2; v++) {
                const uint64_t i = tile + (uint64_t)j * (2 * PB) + 2ull * threadIdx.x + v;
                const bool ok = i < n;
                const uint32_t d = ok ? part_of(k[j][v], nparts) : 0;
                const uint64_t peers = dest_peers(d, ok, dbits);
                if (ok && l == __ffsll((unsigned long long)peers) - 1) atomicAdd(&h[d], (uint32_t)__popcll(peers));
            }
        }
#pragma unroll
        for (int j = 0; j < P_ITEMS; j++) {
            k[j][0] = kn[j][0];
            k[j][1] = kn[j][1];
        }
    }
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < nparts; p += PB)
        if (h[p]) atomicAdd(&counts[p], (unsigned long long)h[p]);
}

// rowid columns travel by value in the kernel arguments: pointers loaded from a device array
// would be generic (FLAT loads / stores)
struct PartCols {
    const uint32_t* in[4];
    uint32_t* out[4];
};

// scatter: a tile is ranked by destination in registers (match-any + per-wave LDS counters),
// staged in LDS in destination order, each destination's range in the send buffer reserved with
// one atomic on its cursor (cursor[d] starts at d's segment start), and written as runs of
// ~PTILE / nparts rows.  Order inside a segment is not kept (the receiver sorts).
// KI / KO: the keys' width in and out (KO = u32: keys below 2^32 leave as 4 B -- half the key bytes
// of the send buffer, the link and the receive buffer)
template <int NC, typename KI = uint64_t, typename KO = uint64_t>
__global__ void __launch_bounds__(PB) part_scatter_kernel(const KI* __restrict__ keys, uint64_t n,
                                                          uint32_t nparts, int dbits,
                                                          unsigned long long* __restrict__ cursor, PartCols pc,
                                                          KO* __restrict__ okeys) {
    __shared__ uint64_t s_key[PTILE];
    __shared__ uint32_t s_col[NC > 0 ? NC : 1][PTILE];
    __shared__ uint8_t s_dest[PTILE];
    __shared__ uint32_t whist[PNW][PMAX];
    __shared__ uint32_t toff[PMAX + 1];
    __shared__ uint64_t gbase[PMAX];
    const int w = wave_id(), l = lane_id();
    const uint64_t lt = lanemask_lt();
    const uint64_t tile = (uint64_t)blockIdx.x * PTILE;
    for (int i = threadIdx.x; i < PNW * PMAX; i += PB) (&whist[0][0])[i] = 0;
    uint64_t k[P_ITEMS];
    uint32_t cv[NC > 0 ? NC : 1][P_ITEMS];
#pragma unroll
    for (int j = 0; j < P_ITEMS; j++) {
        const uint64_t i = tile + (uint64_t)j * PB + threadIdx.x;
        const bool ok = i < n;
        k[j] = ok ? keys[i] : 0;
#pragma unroll
        for (int c = 0; c < NC; c++) cv[c][j] = ok ? pc.in[c][i] : 0;
    }
    __syncthreads();   // whist cleared
    uint32_t dst[P_ITEMS], rank[P_ITEMS];
#pragma unroll
    for (int j = 0; j < P_ITEMS; j++) {      // items in order: the wave's LDS counters stay exact
        const uint64_t i = tile + (uint64_t)j * PB + threadIdx.x;
        const bool ok = i < n;
        const uint32_t d = ok ? part_of(k[j], nparts) : 0;
        const uint64_t peers = dest_peers(d, ok, dbits);
        const int leader = peers ? __ffsll((unsigned long long)peers) - 1 : 0;
        uint32_t old = 0;
        if (ok && l == leader) {
            old = whist[w][d];
            whist[w][d] = old + (uint32_t)__popcll(peers);
        }
        old = (uint32_t)__shfl((int)old, leader, 64);
        dst[j] = ok ? d : PMAX;
        rank[j] = old + (uint32_t)__popcll(peers & lt);
    }
    __syncthreads();
    // per destination: exclusive prefix over waves, tile total; then a scan over destinations
    uint32_t tot = 0;
    if (threadIdx.x < PMAX) {
        const uint32_t d = threadIdx.x;
#pragma unroll
        for (int ww = 0; ww < PNW; ww++) {
            const uint32_t c = whist[ww][d];
            whist[ww][d] = tot;
            tot += c;
        }
        const uint32_t inc = wave_incl_scan_u32(tot);   // threads 0..63 = wave 0
        toff[d] = inc - tot;
        if (d == PMAX - 1) toff[PMAX] = inc;
        if (tot && d < nparts) gbase[d] = atomicAdd(&cursor[d], (unsigned long long)tot);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < P_ITEMS; j++) {
        if (dst[j] < PMAX) {
            const uint32_t pos = toff[dst[j]] + whist[w][dst[j]] + rank[j];
            s_key[pos] = k[j];
            s_dest[pos] = (uint8_t)dst[j];
#pragma unroll
            for (int c = 0; c < NC; c++) s_col[c][pos] = cv[c][j];
        }
    }
    __syncthreads();
    const uint32_t total = toff[PMAX];
    for (uint32_t i = threadIdx.x; i < total; i += PB) {
        const uint32_t d = s_dest[i];
        const uint64_t o = gbase[d] + (i - toff[d]);
        okeys[o] = (KO)s_key[i];
#pragma unroll
        for (int c = 0; c < NC; c++) pc.out[c][o] = s_col[c][i];
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
// with part_of(key, nparts) == g -- exactly the rows the exchange would have delivered to it.
// Unordered compaction (the bucket is sorted next).  A block walks sub-tiles of 4096 rows
// (grid-stride, the next sub-tile's loads in flight while this one is ranked), ranks survivors
// with ballots and appends them to an LDS stage of BS_CAP (key, rowid) pairs; a full stage is
// flushed as one contiguous run, its range reserved with ONE atomic.  (An atomic per sub-tile
// serialises on the counter: ~88 per us on one word, 200 k sub-tiles at 8e8 rows = 2.3 ms.)
// Keys listed in `heavy` (sorted, skew path) are left out of every bucket.
#ifndef QE_BS_B
#define QE_BS_B 256
#endif
#ifndef QE_BS_ITEMS
#define QE_BS_ITEMS 4
#endif
constexpr int BS_B = QE_BS_B;
constexpr int BS_ITEMS = QE_BS_ITEMS;       // x 2 keys per 16-B load
constexpr int BS_TILE = BS_B * BS_ITEMS * 2;
constexpr int BS_NW = BS_B / 64;
constexpr int BS_CAP = BS_TILE;             // staged survivors (a sub-tile's worst case): 12 B each
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

__device__ __forceinline__ void bs_load(const uint64_t* __restrict__ keys, uint64_t n, uint64_t tile,
                                        uint64_t (&k)[BS_ITEMS][2]) {
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
}

__global__ void __launch_bounds__(BS_B) bucket_select_kernel(const uint64_t* __restrict__ keys, uint64_t n,
                                                             uint32_t nparts, uint32_t part,
                                                             const uint64_t* __restrict__ heavy, uint32_t nheavy,
                                                             uint64_t* __restrict__ okeys, uint32_t* __restrict__ ovals,
                                                             uint64_t cap, unsigned long long* __restrict__ counter,
                                                             const uint64_t* __restrict__ vals) {
    __shared__ uint64_t s_key[BS_CAP];
    __shared__ uint32_t s_row[BS_CAP];
    extern __shared__ uint64_t s_heavy[];   // nheavy words (dynamic: no LDS when there are none)
    __shared__ uint32_t s_cnt[BS_ITEMS * 2 * BS_NW];
    __shared__ uint32_t s_total;
    __shared__ uint64_t s_base;
    constexpr int NC = BS_ITEMS * 2 * BS_NW;
    static_assert(NC <= 64, "one wave scans the (item, slot, wave) counts");
    for (uint32_t i = threadIdx.x; i < nheavy; i += BS_B) s_heavy[i] = heavy[i];
    const int w = wave_id(), l = lane_id();
    const uint64_t lt = lanemask_lt();
    const uint64_t nsub = (n + BS_TILE - 1) / BS_TILE;
    uint32_t fill = 0;   // block-uniform
    uint64_t k[BS_ITEMS][2], kn[BS_ITEMS][2];
    uint64_t sub = blockIdx.x;
    if (sub < nsub) bs_load(keys, n, sub * BS_TILE, k);
    __syncthreads();   // s_heavy
    for (; sub < nsub; sub += gridDim.x) {
        const uint64_t tile = sub * BS_TILE;
        const uint64_t nxt = sub + gridDim.x;
        if (nxt < nsub) bs_load(keys, n, nxt * BS_TILE, kn);
        bool f[BS_ITEMS][2];
        uint32_t rank[BS_ITEMS][2];
#pragma unroll
        for (int j = 0; j < BS_ITEMS; j++) {
            const uint64_t i = tile + (uint64_t)j * (BS_B * 2) + (uint64_t)threadIdx.x * 2;
#pragma unroll
            for (int v = 0; v < 2; v++) {
                bool ok = i + v < n && part_of(k[j][v], nparts) == part;
                if (ok && nheavy) ok = heavy_find(s_heavy, nheavy, k[j][v]) < 0;
                f[j][v] = ok;
                const uint64_t m = __ballot(ok);
                rank[j][v] = (uint32_t)__popcll(m & lt);
                if (l == 0) s_cnt[(j * 2 + v) * BS_NW + w] = (uint32_t)__popcll(m);
            }
        }
        __syncthreads();
        if (w == 0) {
            const uint32_t c = l < NC ? s_cnt[l] : 0;
            const uint32_t inc = wave_incl_scan_u32(c);
            if (l < NC) s_cnt[l] = inc - c;
            if (l == NC - 1) s_total = inc;
        }
        __syncthreads();
        const uint32_t total = s_total;
        if (fill + total > (uint32_t)BS_CAP) {          // block-uniform: flush the stage
            if (threadIdx.x == 0) s_base = atomicAdd(counter, (unsigned long long)fill);
            __syncthreads();
            const uint64_t base = s_base;
            for (uint32_t i = threadIdx.x; i < fill; i += BS_B)
                if (base + i < cap) {                    // an overfull bucket is counted, not written
                    okeys[base + i] = s_key[i];
                    ovals[base + i] = s_row[i];
                }
            __syncthreads();
            fill = 0;
        }
#pragma unroll
        for (int j = 0; j < BS_ITEMS; j++) {
            const uint64_t i = tile + (uint64_t)j * (BS_B * 2) + (uint64_t)threadIdx.x * 2;
#pragma unroll
            for (int v = 0; v < 2; v++)
                if (f[j][v]) {
                    const uint32_t o = fill + s_cnt[(j * 2 + v) * BS_NW + w] + rank[j][v];
                    s_key[o] = k[j][v];
                    s_row[o] = vals ? (uint32_t)vals[i + v] : (uint32_t)(i + v);   // a value column's low word, or the rowid
                }
        }
        fill += total;
        __syncthreads();                                 // s_cnt / s_total reused next sub-tile
#pragma unroll
        for (int j = 0; j < BS_ITEMS; j++) {
            k[j][0] = kn[j][0];
            k[j][1] = kn[j][1];
        }
    }
    if (fill) {
        if (threadIdx.x == 0) s_base = atomicAdd(counter, (unsigned long long)fill);
        __syncthreads();
        const uint64_t base = s_base;
        for (uint32_t i = threadIdx.x; i < fill; i += BS_B)
            if (base + i < cap) {
                okeys[base + i] = s_key[i];
                ovals[base + i] = s_row[i];
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

// exclusive scan of the (<= 64) destination counts into the scatter cursors, on the device
__global__ void part_starts_kernel(const unsigned long long* __restrict__ cnt, unsigned long long* __restrict__ cursor,
                                   uint32_t nparts) {
    if (threadIdx.x == 0) {
        unsigned long long run = 0;
        for (uint32_t p = 0; p < nparts; p++) {
            cursor[p] = run;
            run += cnt[p];
        }
    }
}

void partition_dev(qe_ctx* c, const uint64_t* keys, uint64_t n, const uint32_t* const* cols, int ncols,
                   uint32_t nparts, unsigned long long* d_cnt, uint64_t* out_keys, uint32_t* const* out_cols,
                   const uint32_t* keys32, bool out32) {
    if (nparts < 1 || nparts > (uint32_t)PMAX) throw Error(QE_EINVAL, "nparts must be in [1, 64]");
    if (ncols < 0 || ncols > 4) throw Error(QE_EINVAL, "at most 4 rowid columns per partition call");
    if (n >= 0xFFFFFFFFull) throw Error(QE_EINVAL, "partition input too large");
    QE_HIP(hipMemsetAsync(d_cnt, 0, PMAX * sizeof(uint64_t), c->stream));
    if (n == 0) return;
    int dbits = 0;
    while ((1u << dbits) < nparts) dbits++;
    const uint32_t nb = (uint32_t)((n + PTILE - 1) / PTILE);
    PartCols pc{};
    for (int i = 0; i < ncols; i++) {
        pc.in[i] = cols[i];
        pc.out[i] = out_cols[i];
    }
    const double kin = keys32 ? 4.0 : 8.0, kout = out32 ? 4.0 : 8.0;
    {
        Timed t(c, "partition_count", kin * n);
        if (keys32)
            hipLaunchKernelGGL(part_count_kernel<uint32_t>, dim3(std::min<uint32_t>(nb, 1024)), dim3(PB), 0, c->stream,
                               keys32, n, nparts, dbits, d_cnt);
        else
            hipLaunchKernelGGL(part_count_kernel<uint64_t>, dim3(std::min<uint32_t>(nb, 1024)), dim3(PB), 0, c->stream,
                               keys, n, nparts, dbits, d_cnt);
        QE_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(part_starts_kernel, dim3(1), dim3(64), 0, c->stream, d_cnt, d_cnt + PMAX, nparts);
    QE_HIP(hipGetLastError());
    {
        Timed t(c, "partition", (kin + kout + 8.0 * ncols) * n);
        uint32_t* ok32 = reinterpret_cast<uint32_t*>(out_keys);
        switch (ncols) {
#define QE_PS(NC)                                                                                                 \
    case NC:                                                                                                      \
        if (keys32 && out32)                                                                                      \
            hipLaunchKernelGGL((part_scatter_kernel<NC, uint32_t, uint32_t>), dim3(nb), dim3(PB), 0, c->stream,    \
                               keys32, n, nparts, dbits, d_cnt + PMAX, pc, ok32);                                 \
        else if (out32)                                                                                           \
            hipLaunchKernelGGL((part_scatter_kernel<NC, uint64_t, uint32_t>), dim3(nb), dim3(PB), 0, c->stream,    \
                               keys, n, nparts, dbits, d_cnt + PMAX, pc, ok32);                                   \
        else                                                                                                      \
            hipLaunchKernelGGL((part_scatter_kernel<NC>), dim3(nb), dim3(PB), 0, c->stream, keys, n, nparts,       \
                               dbits, d_cnt + PMAX, pc, out_keys);                                                \
        break;
            QE_PS(0) QE_PS(1) QE_PS(2) QE_PS(3) QE_PS(4)
#undef QE_PS
        }
        QE_HIP(hipGetLastError());
    }
}

}  // namespace qe

using namespace qe;

extern "C" {

int qe_partition(qe_ctx* c, const uint64_t* keys, uint64_t n, const uint32_t* const* cols, int ncols,
                 uint32_t nparts, uint64_t* counts, uint64_t* out_keys, uint32_t* const* out_cols) {
    QE_API_BEGIN(c)
    unsigned long long* d_cnt = dalloc_t<unsigned long long>(c, 2 * PMAX);   // [counts | cursors]
    partition_dev(c, keys, n, cols, ncols, nparts, d_cnt, out_keys, out_cols);
    QE_HIP(hipMemcpyAsync(counts, d_cnt, nparts * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    QE_HIP(hipStreamSynchronize(c->stream));   // the caller hands the buffers to RCCL next
    dfree(c, d_cnt);
    uint64_t run = 0;
    for (uint32_t p = 0; p < nparts; p++) run += counts[p];
    if (run != n) throw Error(QE_EINVAL, "internal: partition counts do not add up");
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

int qe_filter_scan2_range(qe_ctx* c, qe_col col1, char op1, uint64_t v1, qe_col col2, char op2, uint64_t v2,
                          uint64_t start, uint64_t end, qe_list* out) {
    QE_API_BEGIN(c)
    if (end > col1.n || end > col2.n || start > end) throw Error(QE_EINVAL, "bad row range");
    const uint64_t n = end - start;
    out->d = dalloc_t<uint32_t>(c, std::max<uint64_t>(n, 1));
    out->cap = n;
    out->n = filter_scan2(c, col1.d + start, op1, v1, col2.d + start, op2, v2, n, out->d);
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
    bucket_select_dev(c, col, nparts, part, heavy, nheavy, nullptr, out);
    return 0;
    QE_API_END(c)
}

int qe_partition_columns(qe_ctx* c, uint32_t nparts, uint32_t part) {
    QE_API_BEGIN(c)
    if (nparts < 1 || part >= nparts) throw Error(QE_EINVAL, "part out of range");
    drop_partitions(c);
    if (nparts == 1) return 0;   // (one rank reads the columns themselves)
    // nothing is selected here: a column's bucket is made the first time the partitioned plan reads
    // it as a whole base join side (e_base_side) and cached until the relations are dropped -- a
    // column that is never a partitioned join key (a payload, or a broadcast join's base side)
    // never holds one, and no allocation can fail at load
    c->bparts_n = nparts;
    c->bparts_p = part;
    return 0;
    QE_API_END(c)
}

}  // extern "C"

namespace qe {

// every run longer than thr in a sorted sample: its key and length (first element of the run
// only; a binary search finds the end), appended through one counter (runs that long are few)
__global__ void __launch_bounds__(256) heavy_runs_kernel(const uint64_t* __restrict__ s, uint64_t n, uint64_t thr,
                                                         unsigned long long* __restrict__ cnt, uint64_t* __restrict__ okey,
                                                         uint64_t* __restrict__ olen, uint32_t cap) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n || i + thr >= n) return;
    const uint64_t k = s[i];
    if ((i > 0 && s[i - 1] == k) || s[i + thr] != k) return;
    uint64_t lo = i + thr, hi = n;   // s[lo] == k; s[hi] != k or hi == n
    while (lo + 1 < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (s[mid] == k) lo = mid;
        else hi = mid;
    }
    const unsigned long long slot = atomicAdd(cnt, 1ull);
    if (slot < cap) {
        okey[slot] = k;
        olen[slot] = lo + 1 - i;
    }
}

std::vector<uint64_t> heavy_keys_dev(qe_ctx* c, const qe_col* cols, int ncols, uint64_t sample, uint64_t div,
                                     uint32_t maxk) {
    constexpr uint32_t CAP = 4096;
    std::vector<std::pair<double, uint64_t>> cand;   // (sample frequency, key)
    for (int ci = 0; ci < ncols; ci++) {
        const uint64_t m = std::min<uint64_t>(sample, cols[ci].n);
        const uint64_t thr = m / std::max<uint64_t>(div, 1);
        if (m == 0 || thr + 1 >= m) continue;
        SortOut so = radix_sort_u64(c, cols[ci].d, nullptr, m, false, nullptr, false);
        const uint64_t* sorted = static_cast<const uint64_t*>(so.keys);
        uint64_t* d = dalloc_t<uint64_t>(c, 2 * (uint64_t)CAP + 1);
        unsigned long long* d_cnt = reinterpret_cast<unsigned long long*>(d + 2 * CAP);
        hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(64), 0, c->stream, (uint64_t*)d_cnt, 1);
        QE_HIP(hipGetLastError());
        hipLaunchKernelGGL(heavy_runs_kernel, dim3(grid_for(m, 256)), dim3(256), 0, c->stream, sorted, m, thr, d_cnt, d,
                           d + CAP, CAP);
        QE_HIP(hipGetLastError());
        const uint64_t got = std::min<uint64_t>(read_u64(c, reinterpret_cast<uint64_t*>(d_cnt)), CAP);
        std::vector<uint64_t> h(2 * (size_t)CAP);
        if (got) {
            QE_HIP(hipMemcpyAsync(h.data(), d, got * 8, hipMemcpyDeviceToHost, c->stream));
            QE_HIP(hipMemcpyAsync(h.data() + CAP, d + CAP, got * 8, hipMemcpyDeviceToHost, c->stream));
            QE_HIP(hipStreamSynchronize(c->stream));
        }
        for (uint64_t i = 0; i < got; i++) cand.emplace_back((double)h[CAP + i] / (double)m, h[i]);
        dfree(c, d);
        if (so.keys_new) dfree(c, so.keys);
        if (so.vals_new) dfree(c, so.vals);
    }
    // the most frequent first (a key heavy on both sides counts with its larger frequency), then
    // the kept ones sorted ascending -- the same list on every rank (replicated columns)
    std::sort(cand.begin(), cand.end(), [](const auto& a, const auto& b) {
        return a.first != b.first ? a.first > b.first : a.second < b.second;
    });
    std::vector<uint64_t> keys;
    for (const auto& x : cand) {
        if (keys.size() >= maxk) break;
        if (std::find(keys.begin(), keys.end(), x.second) == keys.end()) keys.push_back(x.second);
    }
    std::sort(keys.begin(), keys.end());
    return keys;
}

void bucket_select_dev(qe_ctx* c, qe_col col, uint32_t nparts, uint32_t part, const uint64_t* heavy, uint32_t nheavy,
                       const uint64_t* vals, qe_pairs* out) {
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
    // grid-stride over sub-tiles with exactly the resident blocks (a second round of blocks would
    // run behind the first on a fraction of the CUs)
    static int cus = 0;
    int per_cu = 0;
    const size_t dyn = (size_t)nheavy * sizeof(uint64_t);
    if (!cus) QE_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
    QE_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, bucket_select_kernel, BS_B, dyn));
    const unsigned nb = grid_for(n, BS_TILE, (unsigned)std::max(1, cus * std::max(1, per_cu)));
    for (int attempt = 0; attempt < 2; attempt++) {
        out->key = dalloc_t<uint64_t>(c, std::max<uint64_t>(cap, 1));
        out->val = dalloc_t<uint32_t>(c, std::max<uint64_t>(cap, 1));
        hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(64), 0, c->stream, (uint64_t*)d_cnt, 1);
        QE_HIP(hipGetLastError());
        if (n) {
            Timed t(c, "bucket_select", 8.0 * n);
            hipLaunchKernelGGL(bucket_select_kernel, dim3(nb), dim3(BS_B), dyn, c->stream, col.d, n, nparts, part,
                               d_heavy, nheavy, out->key, out->val, cap, d_cnt, vals);
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
    add_bytes(c, "bucket_select", 12.0 * out->n + (vals ? 8.0 * n : 0.0));
    out->owns = 3;
    out->flags = vals ? 0 : QE_PAIRS_DISTINCT;
    if (d_heavy) dfree(c, d_heavy);
}

}  // namespace qe

extern "C" {

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
