// qe_agg.hip -- the aggregate join of two base columns (C5).
//
// The query's last join, whose two lists only print_sums reads (src/utilities.c:197-224), is
// never materialised: for R row i with c_i partners in S, the R list holds rowid i exactly c_i
// times, so its checksum over column V is sum_i V[i] * c_i (mod 2^64), and the list length is
// P = sum_i c_i.  The reference builds the lists (src/join.c:325-392, its DArray caps them at
// INT32_MAX: src/DArray.h:14-15); the faithful executor's merge path computes the same numbers
// from sorted (key, rowid) pairs and then gathers V by rowid (random 8-B reads).  Here each
// side is sorted once as (key field << 32 | V[i]) words -- the select column rides where the
// rowid would -- and ONE merge-path pass over both sorted sides yields c_i for every row of both
// sides and the three sums, all streaming:
//
//   * the merged order of R and S (R first on equal keys) is cut into tiles of AG_T elements
//     (merge path: a binary search per boundary); a key whose merged run crosses a tile boundary
//     gets its global counts there (galloping searches around the boundary, both sides);
//   * a tile loads its R and S ranges (coalesced words) and keeps the key fields in LDS; every
//     other key's run lies wholly inside the tile, and two merge walks of the tile (R first, then
//     S first on equal keys; one stretch of AG_ITEMS merged elements per thread) give each row
//     the lower and upper bound of its key in the other range: the partner count;
//   * per-tile partial sums, then one small reduction: one host read of (P, sumR, sumS).
//
// HBM traffic: the sorted words once (8 B per row of both sides) + the split table.
#include "qe_device.h"
#include "qe_internal.h"

namespace qe {

#ifndef QE_AG_NT
#define QE_AG_NT 256
#endif
#ifndef QE_AG_ITEMS
#define QE_AG_ITEMS 16
#endif
constexpr int AG_NT = QE_AG_NT;
constexpr int AG_ITEMS = QE_AG_ITEMS;
constexpr int AG_T = AG_NT * AG_ITEMS;   // merged elements per tile

__device__ __forceinline__ uint32_t kf(uint64_t w) { return (uint32_t)(w >> 32); }

// the run of key k in sorted a[0..n) that contains (or starts at) position p, where every key
// before p is <= k and every key from p on is >= k: [first, end), by galloping outwards from p
__device__ __forceinline__ void g_run(const uint64_t* __restrict__ a, uint64_t n, uint64_t p, uint32_t k, uint64_t* first,
                                      uint64_t* end) {
    // backwards: smallest i <= p with a[i..p) all == k
    uint64_t lo = p, step = 1;
    while (lo > 0 && kf(a[lo - 1]) == k) {
        const uint64_t nl = lo >= step ? lo - step : 0;
        if (kf(a[nl]) == k) {
            lo = nl;
            step <<= 1;
        } else {   // a[nl] < k <= a[lo-1] = k: the run starts in (nl, lo)
            uint64_t l2 = nl + 1, h2 = lo;
            while (l2 < h2) {
                const uint64_t mid = l2 + (h2 - l2) / 2;
                if (kf(a[mid]) < k) l2 = mid + 1;
                else h2 = mid;
            }
            lo = l2;
            break;
        }
    }
    // forwards: first i >= p with a[i] > k
    uint64_t hi = p;
    step = 1;
    while (hi < n && kf(a[hi]) == k) {
        const uint64_t nh = hi + step < n ? hi + step : n;
        if (nh < n && kf(a[nh]) == k) {
            hi = nh + 1;
            step <<= 1;
        } else {   // a[hi] == k, a[nh] > k (or nh == n): the run ends in (hi, nh]
            uint64_t l2 = hi + 1, h2 = nh;
            while (l2 < h2) {
                const uint64_t mid = l2 + (h2 - l2) / 2;
                if (kf(a[mid]) <= k) l2 = mid + 1;
                else h2 = mid;
            }
            hi = l2;
            break;
        }
    }
    *first = lo;
    *end = hi;
}

// boundary t (0..nt): ra[t] = number of R rows among the first d = min(t * AG_T, nR + nS) merged
// elements (R first on equal keys); for 0 < t < nt also the key of merged element d and its
// global run lengths in R and S
__global__ void __launch_bounds__(256) ag_split_kernel(const uint64_t* __restrict__ R, uint64_t nR,
                                                       const uint64_t* __restrict__ S, uint64_t nS, uint32_t nt,
                                                       uint64_t* __restrict__ ra, uint32_t* __restrict__ bkey,
                                                       uint32_t* __restrict__ bcR, uint32_t* __restrict__ bcS) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t > nt) return;
    const uint64_t m = nR + nS;
    const uint64_t d = (uint64_t)t * AG_T < m ? (uint64_t)t * AG_T : m;
    // largest a with R[a-1] <= S[d-a]: binary search over a in [max(0, d - nS), min(d, nR)]
    uint64_t lo = d > nS ? d - nS : 0, hi = d < nR ? d : nR;
    while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;   // take R[mid] before S[d - mid - 1]?
        if (kf(R[mid]) <= kf(S[d - mid - 1])) lo = mid + 1;
        else hi = mid;
    }
    const uint64_t a = lo, b = d - a;
    ra[t] = a;
    if (t == 0 || t == nt) return;
    uint32_t k;
    if (a < nR && (b >= nS || kf(R[a]) <= kf(S[b]))) k = kf(R[a]);
    else k = kf(S[b]);
    uint64_t f0, e0, f1, e1;
    g_run(R, nR, a, k, &f0, &e0);
    g_run(S, nS, b, k, &f1, &e1);
    bkey[t] = k;
    bcR[t] = (uint32_t)(e0 - f0);
    bcS[t] = (uint32_t)(e1 - f1);
}

// LDS index with one pad word per 32: the walks' threads start ~8-16 words apart, which without
// padding lands a wave's accesses on a few banks
__device__ __forceinline__ uint32_t pd(uint32_t i) { return i + (i >> 5); }

// One thread's stretch [d, e) of the tile's merged order, walked twice at once: R first on
// equal keys (chain A) and S first (chain B), each chain placed by its own merge-path search in
// LDS.  Every element taken learns how many elements of the other side precede it -- chain A: an
// R row #S < k, an S row #R <= k; chain B: an R row #S <= k, an S row #R < k -- so the two give
// each row the lower and upper bound of its key in the other range.  The chains are independent
// (16-bit bounds, lo[] and hi[]): their LDS latencies overlap.
// keys[] holds the R range at [0, na) and the S range at [na, na + nb) (padded indices).
__device__ __forceinline__ void merge_walks(const uint32_t* keys, uint32_t na, uint32_t nb, uint32_t d, uint32_t e,
                                            uint16_t* blo, uint16_t* bhi) {
    uint32_t la = d > nb ? d - nb : 0, ha = d < na ? d : na;
    uint32_t lb = la, hb = ha;
#pragma unroll
    for (int it = 0; it < 13; it++) {   // 13 halvings cover AG_T <= 4096 (static_assert below)
        if (la < ha) {
            const uint32_t mid = (la + ha) >> 1;
            if (keys[pd(mid)] <= keys[pd(na + d - mid - 1)]) la = mid + 1;
            else ha = mid;
        }
        if (lb < hb) {
            const uint32_t mid = (lb + hb) >> 1;
            if (keys[pd(mid)] < keys[pd(na + d - mid - 1)]) lb = mid + 1;
            else hb = mid;
        }
    }
    uint32_t aA = la, bA = d - la, aB = lb, bB = d - lb;
    uint32_t kaA = aA < na ? keys[pd(aA)] : 0, kbA = bA < nb ? keys[pd(na + bA)] : 0;
    uint32_t kaB = aB < na ? keys[pd(aB)] : 0, kbB = bB < nb ? keys[pd(na + bB)] : 0;
    for (uint32_t p = d; p < e; p++) {
        const bool tA = aA < na && (bA >= nb || kaA <= kbA);
        const bool tB = aB < na && (bB >= nb || kaB < kbB);
        blo[pd(tA ? aA : na + bA)] = (uint16_t)(tA ? bA : aA);   // R: #S < k; S: #R <= k
        bhi[pd(tB ? aB : na + bB)] = (uint16_t)(tB ? bB : aB);   // R: #S <= k; S: #R < k
        aA += tA ? 1u : 0u;
        bA += tA ? 0u : 1u;
        aB += tB ? 1u : 0u;
        bB += tB ? 0u : 1u;
        const uint32_t nA = tA ? aA : na + bA, nB = tB ? aB : na + bB;
        const uint32_t kA = (tA ? aA < na : bA < nb) ? keys[pd(nA)] : 0;
        const uint32_t kB = (tB ? aB < na : bB < nb) ? keys[pd(nB)] : 0;
        kaA = tA ? kA : kaA;
        kbA = tA ? kbA : kA;
        kaB = tB ? kB : kaB;
        kbB = tB ? kbB : kB;
    }
}

#ifdef QE_DIAG_STAMPS
__device__ uint64_t g_ag_stamps[STAMP_TILES * STAMP_SLOTS];
#endif

// the words of tile t (its R range, then its S range) into registers, striped over the block
__device__ __forceinline__ void ag_load(const uint64_t* __restrict__ R, const uint64_t* __restrict__ S, uint64_t m,
                                        const uint64_t* __restrict__ ra, uint32_t t, uint64_t* w, uint32_t* na_out,
                                        uint32_t* tot_out) {
    const uint64_t d0 = (uint64_t)t * AG_T, d1 = d0 + AG_T < m ? d0 + AG_T : m;
    const uint64_t a0 = ra[t], a1 = ra[t + 1];
    const uint64_t b0 = d0 - a0;
    const uint32_t na = (uint32_t)(a1 - a0), tot = (uint32_t)(d1 - d0);
#pragma unroll
    for (int j = 0; j < AG_ITEMS; j++) {
        const uint32_t i = (uint32_t)j * AG_NT + threadIdx.x;
        w[j] = i < na ? R[a0 + i] : (i < tot ? S[b0 + (i - na)] : 0);
    }
    *na_out = na;
    *tot_out = tot;
}

// Persistent: each workgroup takes tiles blockIdx.x, + gridDim.x, ...; the next tile's words are
// loaded while the current tile is walked and summed (its HBM latency hides behind LDS work),
// and the sums stay in registers until the last tile: partial[block] = (pairs, sum of R vals x
// S counts, sum of S vals x R counts)
__global__ void __launch_bounds__(AG_NT) ag_tile_kernel(const uint64_t* __restrict__ R, uint64_t nR,
                                                        const uint64_t* __restrict__ S, uint64_t nS, uint32_t nt,
                                                        const uint64_t* __restrict__ ra, const uint32_t* __restrict__ bkey,
                                                        const uint32_t* __restrict__ bcR, const uint32_t* __restrict__ bcS,
                                                        uint64_t* __restrict__ partial) {
    static_assert(AG_T <= 4096, "13 merge-path halvings, 16-bit in-tile bounds");
    __shared__ uint32_t keys[AG_T + AG_T / 32];   // R range then S range (padded indices, pd)
    __shared__ uint16_t blo[AG_T + AG_T / 32];    // per element: bounds of its key in the other range
    __shared__ uint16_t bhi[AG_T + AG_T / 32];
    __shared__ uint64_t red[3][AG_NT / 64];
    const uint64_t m = nR + nS;
    uint64_t pairs = 0, sr = 0, ss = 0;
    uint64_t w[AG_ITEMS], wn[AG_ITEMS];
    uint32_t na = 0, tot = 0, nan = 0, totn = 0;
    uint32_t t = blockIdx.x;
    if (t < nt) ag_load(R, S, m, ra, t, w, &na, &tot);
    for (; t < nt; t += gridDim.x) {
        QE_STAMP(g_ag_stamps, t, 0);
        const uint32_t nb = tot - na;
#pragma unroll
        for (int j = 0; j < AG_ITEMS; j++) {
            const uint32_t i = (uint32_t)j * AG_NT + threadIdx.x;
            if (i < tot) keys[pd(i)] = kf(w[j]);
        }
        __syncthreads();
        QE_STAMP(g_ag_stamps, t, 1);
        const uint32_t tn = t + gridDim.x;
        if (tn < nt) ag_load(R, S, m, ra, tn, wn, &nan, &totn);   // in flight during the walks
        // boundary keys: a key equal to one of these may run past the tile -- global counts;
        // every other key's run lies wholly inside the tile and the walks count its partners
        const bool hasL = t > 0, hasR = t + 1 < nt;
        const uint32_t kL = hasL ? bkey[t] : 0, kR = hasR ? bkey[t + 1] : 0;
        const uint32_t lR = hasL ? bcR[t] : 0, lS = hasL ? bcS[t] : 0;
        const uint32_t rR = hasR ? bcR[t + 1] : 0, rS = hasR ? bcS[t + 1] : 0;
        const uint32_t e0 = threadIdx.x * AG_ITEMS < tot ? threadIdx.x * AG_ITEMS : tot;
        const uint32_t e1 = e0 + AG_ITEMS < tot ? e0 + AG_ITEMS : tot;
        merge_walks(keys, na, nb, e0, e1, blo, bhi);
        __syncthreads();
        QE_STAMP(g_ag_stamps, t, 2);
#pragma unroll
        for (int j = 0; j < AG_ITEMS; j++) {
            const uint32_t i = (uint32_t)j * AG_NT + threadIdx.x;
            if (i >= tot) continue;
            const uint32_t k = kf(w[j]);
            const uint32_t v = (uint32_t)w[j];
            const bool isR = i < na;
            const uint32_t lo = blo[pd(i)], hi = bhi[pd(i)];
            uint32_t c = isR ? hi - lo : lo - hi;   // partners in the other side
            if (hasL && k == kL) c = isR ? lS : lR;
            else if (hasR && k == kR) c = isR ? rS : rR;
            if (isR) {
                pairs += c;
                sr += (uint64_t)v * c;
            } else {
                ss += (uint64_t)v * c;
            }
        }
        __syncthreads();   // keys / bounds are rewritten for the next tile
        QE_STAMP(g_ag_stamps, t, 3);
#pragma unroll
        for (int j = 0; j < AG_ITEMS; j++) w[j] = wn[j];
        na = nan;
        tot = totn;
    }
    pairs = wave_sum_u64(pairs);
    sr = wave_sum_u64(sr);
    ss = wave_sum_u64(ss);
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[0][wv] = pairs;
        red[1][wv] = sr;
        red[2][wv] = ss;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        uint64_t sum = 0;
#pragma unroll
        for (int q = 0; q < AG_NT / 64; q++) sum += red[threadIdx.x][q];
        partial[(uint64_t)blockIdx.x * 3 + threadIdx.x] = sum;
    }
}

__global__ void __launch_bounds__(1024) ag_reduce_kernel(const uint64_t* __restrict__ partial, uint32_t nt,
                                                         uint64_t* __restrict__ out) {
    __shared__ uint64_t red[3][16];
    uint64_t s[3] = {0, 0, 0};
    for (uint32_t t = threadIdx.x; t < nt; t += 1024)
#pragma unroll
        for (int q = 0; q < 3; q++) s[q] += partial[(uint64_t)t * 3 + q];
#pragma unroll
    for (int q = 0; q < 3; q++) s[q] = wave_sum_u64(s[q]);
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int q = 0; q < 3; q++) red[q][threadIdx.x >> 6] = s[q];
    __syncthreads();
    if (threadIdx.x < 3) {
        uint64_t v = 0;
        for (int q = 0; q < 16; q++) v += red[threadIdx.x][q];
        out[threadIdx.x] = v;
    }
}

// ---- the bucketed aggregate join ---------------------------------------------------------------
// Both sides' (key field << 32 | value) words partitioned into the 2^15 buckets of the field's top
// bits (partition_words_kv: the two-level sort's two global passes, no per-bucket sort); inside a
// bucket a key is its field's L low bits, a dense domain of 2^L values counted in LDS.  Per bucket
// (one workgroup):  cnt <- S's key counts;  R rows: pairs += cnt[k], sumR += valR * cnt[k];
// cnt <- R's key counts;  S rows: sumS += valS * cnt[k].  Two reads of each side's words, no
// merge, no search.  A bucket side beyond AB_BIG rows (a Zipf head key) goes to the giant path:
// many workgroups per bucket, counts pre-aggregated in LDS per chunk and added to a per-bucket
// global count table.  Counting takes ONE LDS atomic per wave for the lanes whose key equals the
// first valid lane's (a head key fills whole waves), one per lane otherwise.
constexpr int AB_NT = 1024, AB_U = 8;
#ifndef QE_AB_BIG
#define QE_AB_BIG (1u << 18)
#endif
constexpr uint32_t AB_BIG = QE_AB_BIG;
constexpr uint32_t AB_CHUNK = 1u << 16;   // giant path: rows per workgroup

__device__ __forceinline__ uint32_t ab_val(uint64_t w, uint32_t dmask) { return (uint32_t)(w >> 32) & dmask; }

// NT: the rows' last read (non-temporal loads: MI355X_MICROARCH "nt-weights"; the aggregate last
// join's words measured 0.26 -> 0.239 ms per C3 query that way, profiles/r06ze_c3_bench.log)
#ifndef QE_AB_NT
#define QE_AB_NT 1   // (build knob, A/B: 0 = default-policy loads on the second read too)
#endif
template <bool NT = false>
__device__ __forceinline__ uint64_t ab_ld(const uint64_t* p) {
    if constexpr (NT && QE_AB_NT) return __builtin_nontemporal_load(p);
    else return *p;
}

template <bool NT = false>
__device__ __forceinline__ void ab_count(const uint64_t* __restrict__ w, uint32_t m, uint32_t dmask,
                                         uint32_t* __restrict__ cnt) {
    const int l = lane_id();
    for (uint32_t i0 = threadIdx.x; i0 < m; i0 += AB_NT * AB_U) {   // (block-uniform trip count: i0 - tid)
        uint64_t x[AB_U];
#pragma unroll
        for (int u = 0; u < AB_U; u++) {
            const uint32_t i = i0 + (uint32_t)u * AB_NT;
            x[u] = i < m ? ab_ld<NT>(&w[i]) : 0;
        }
#pragma unroll
        for (int u = 0; u < AB_U; u++) {
            const uint32_t i = i0 + (uint32_t)u * AB_NT;
            const bool valid = i < m;
            const uint32_t v = ab_val(x[u], dmask);
            const uint64_t vb = __ballot(valid);
            if (!vb) continue;
            const int leader = __ffsll((unsigned long long)vb) - 1;
            const uint32_t v0 = (uint32_t)__shfl((int)v, leader, 64);
            const uint64_t same = __ballot(valid && v == v0);
            if (valid) {
                if (v != v0) atomicAdd(&cnt[v], 1u);
                else if (l == leader) atomicAdd(&cnt[v0], (uint32_t)__popcll(same));
            }
        }
    }
}

// rows of w[0..m): a0 += cnt[k], a1 += (u32) value * cnt[k]
template <bool NT = false>
__device__ __forceinline__ void ab_lookup(const uint64_t* __restrict__ w, uint32_t m, uint32_t dmask,
                                          const uint32_t* __restrict__ cnt, uint64_t& a0, uint64_t& a1) {
    for (uint32_t i0 = threadIdx.x; i0 < m; i0 += AB_NT * AB_U) {
        uint64_t x[AB_U];
#pragma unroll
        for (int u = 0; u < AB_U; u++) {
            const uint32_t i = i0 + (uint32_t)u * AB_NT;
            x[u] = i < m ? ab_ld<NT>(&w[i]) : 0;
        }
#pragma unroll
        for (int u = 0; u < AB_U; u++) {
            const uint32_t i = i0 + (uint32_t)u * AB_NT;
            if (i < m) {
                const uint64_t c = cnt[ab_val(x[u], dmask)];
                a0 += c;
                a1 += (uint64_t)(uint32_t)x[u] * c;
            }
        }
    }
}

__device__ __forceinline__ void ab_zero(uint32_t* cnt, uint32_t D) {
    for (uint32_t v = threadIdx.x * 4; v < D; v += AB_NT * 4) *reinterpret_cast<uint4*>(cnt + v) = make_uint4(0, 0, 0, 0);
}

// block sum of three u64 -> out[0..2] (plain stores, thread 0)
__device__ __forceinline__ void ab_reduce3(uint64_t a0, uint64_t a1, uint64_t a2, uint64_t* __restrict__ out,
                                           bool atomic) {
    __shared__ uint64_t red[AB_NT / 64][3];
    a0 = wave_sum_u64(a0);
    a1 = wave_sum_u64(a1);
    a2 = wave_sum_u64(a2);
    if (lane_id() == 0) {
        red[wave_id()][0] = a0;
        red[wave_id()][1] = a1;
        red[wave_id()][2] = a2;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        uint64_t t = 0;
        for (int w = 0; w < AB_NT / 64; w++) t += red[w][threadIdx.x];
        if (atomic) atomicAdd(reinterpret_cast<unsigned long long*>(out + threadIdx.x), (unsigned long long)t);
        else out[threadIdx.x] = t;
    }
}

// one workgroup per bucket; a giant bucket is listed (b, mR, mS) for the giant path
__global__ void __launch_bounds__(AB_NT) ab_bucket_kernel(const uint64_t* __restrict__ wR, const uint32_t* __restrict__ bsR,
                                                          const uint64_t* __restrict__ wS, const uint32_t* __restrict__ bsS,
                                                          int L, uint64_t* __restrict__ part, uint32_t* __restrict__ big,
                                                          unsigned long long* __restrict__ nbig) {
    __shared__ uint32_t cnt[1u << 15];
    const uint32_t b = blockIdx.x;
    const uint32_t r0 = bsR[b], mR = bsR[b + 1] - r0, s0 = bsS[b], mS = bsS[b + 1] - s0;
    if (mR == 0 || mS == 0) {
        if (threadIdx.x < 3) part[(uint64_t)b * 3 + threadIdx.x] = 0;
        return;
    }
    if (mR > AB_BIG || mS > AB_BIG) {
        if (threadIdx.x < 3) part[(uint64_t)b * 3 + threadIdx.x] = 0;
        if (threadIdx.x == 0) {
            const unsigned long long k = atomicAdd(nbig, 1ull);
            big[3 * k] = b;
            big[3 * k + 1] = mR;
            big[3 * k + 2] = mS;
        }
        return;
    }
    const uint32_t D = 1u << L, dmask = D - 1u;
    const uint64_t* __restrict__ bR = wR + r0;
    const uint64_t* __restrict__ bS = wS + s0;
    uint64_t pairs = 0, sR = 0, sS = 0, dummy = 0;
    ab_zero(cnt, D);
    __syncthreads();
    ab_count(bS, mS, dmask, cnt);
    __syncthreads();
    ab_lookup(bR, mR, dmask, cnt, pairs, sR);
    __syncthreads();
    ab_zero(cnt, D);
    __syncthreads();
    ab_count<true>(bR, mR, dmask, cnt);   // (each side's second and last read)
    __syncthreads();
    ab_lookup<true>(bS, mS, dmask, cnt, dummy, sS);
    ab_reduce3(pairs, sR, sS, part + (uint64_t)b * 3, false);
}

// giant path, counting: workgroup (x, g) counts rows [x * AB_CHUNK, ...) of giant g's side in LDS
// and adds the nonzero counts to g's global table
__global__ void __launch_bounds__(AB_NT) ab_big_count_kernel(const uint64_t* __restrict__ w, const uint32_t* __restrict__ bs,
                                                             const uint32_t* __restrict__ big, int side, int L,
                                                             uint32_t* __restrict__ gcnt) {
    __shared__ uint32_t cnt[1u << 15];
    const uint32_t g = blockIdx.y, b = big[3 * g], m = big[3 * g + 1 + side];
    const uint32_t c0 = blockIdx.x * AB_CHUNK;
    if (c0 >= m) return;
    const uint32_t mc = m - c0 < AB_CHUNK ? m - c0 : AB_CHUNK;
    const uint32_t D = 1u << L, dmask = D - 1u;
    ab_zero(cnt, D);
    __syncthreads();
    ab_count(w + bs[b] + c0, mc, dmask, cnt);
    __syncthreads();
    uint32_t* __restrict__ gc = gcnt + (uint64_t)g * D;
    for (uint32_t v = threadIdx.x; v < D; v += AB_NT)
        if (cnt[v]) atomicAdd(&gc[v], cnt[v]);
}

// giant path, lookups against g's global table: acc[0] += counts (with_pairs), acc[1 + side] +=
// value * count
__global__ void __launch_bounds__(AB_NT) ab_big_look_kernel(const uint64_t* __restrict__ w, const uint32_t* __restrict__ bs,
                                                            const uint32_t* __restrict__ big, int side, int L,
                                                            const uint32_t* __restrict__ gcnt, int with_pairs,
                                                            uint64_t* __restrict__ acc) {
    const uint32_t g = blockIdx.y, b = big[3 * g], m = big[3 * g + 1 + side];
    const uint32_t c0 = blockIdx.x * AB_CHUNK;
    if (c0 >= m) return;
    const uint32_t mc = m - c0 < AB_CHUNK ? m - c0 : AB_CHUNK;
    const uint32_t D = 1u << L, dmask = D - 1u;
    uint64_t a0 = 0, a1 = 0;
    ab_lookup(w + bs[b] + c0, mc, dmask, gcnt + (uint64_t)g * D, a0, a1);
    ab_reduce3(with_pairs ? a0 : 0, side == 0 ? a1 : 0, side == 1 ? a1 : 0, acc, true);
}

__global__ void __launch_bounds__(256) ab_sum3_kernel(const uint64_t* __restrict__ part, uint32_t nb,
                                                      uint64_t* __restrict__ out) {
    const uint32_t k = blockIdx.x;
    uint64_t t = 0;
    for (uint32_t b = threadIdx.x; b < nb; b += 256) t += part[(uint64_t)b * 3 + k];
    t = wave_sum_u64(t);
    __shared__ uint64_t red[4];
    if (lane_id() == 0) red[wave_id()] = t;
    __syncthreads();
    if (threadIdx.x == 0) out[k] += red[0] + red[1] + red[2] + red[3];
}

static bool agg_buckets_on() {
    static bool on = [] {   // tuning knob: QE_AGG_BUCKETS=0 keeps the sort + merge-path counting form
        const char* s = getenv("QE_AGG_BUCKETS");
        return !(s && s[0] == '0');
    }();
    return on;
}

// out = {pairs, sumR, sumS} (values as AggSide: none -> the caller zeroes that sum)
static void join_aggregate_buckets(qe_ctx* c, const AggSide& R, const AggSide& S, int lo, int nb, uint64_t out[3]) {
    constexpr uint32_t NB = 1u << AGG_BUCKET_BITS;
    const int L = nb - AGG_BUCKET_BITS;
    uint64_t *wR = nullptr, *wS = nullptr;
    uint32_t *bsR = nullptr, *bsS = nullptr;
    partition_words_kv(c, R.keys, R.v64, R.v32, R.n, lo, nb, &wR, &bsR);
    partition_words_kv(c, S.keys, S.v64, S.v32, S.n, lo, nb, &wS, &bsS);
    uint64_t* part = dalloc_t<uint64_t>(c, (size_t)NB * 3);
    uint32_t* big = dalloc_t<uint32_t>(c, (size_t)NB * 3);
    uint64_t* d = dalloc_t<uint64_t>(c, 4);   // [pairs, sumR, sumS, giant buckets]
    hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(64), 0, c->stream, (uint64_t*)d, 4);
    QE_HIP(hipGetLastError());
    {
        Timed t(c, "agg_count", 8.0 * 2.0 * (double)(R.n + S.n));
        hipLaunchKernelGGL(ab_bucket_kernel, dim3(NB), dim3(AB_NT), 0, c->stream, wR, bsR, wS, bsS, L, part, big,
                           reinterpret_cast<unsigned long long*>(d + 3));
        QE_HIP(hipGetLastError());
        hipLaunchKernelGGL(ab_sum3_kernel, dim3(3), dim3(256), 0, c->stream, part, NB, d);
        QE_HIP(hipGetLastError());
    }
    uint64_t h[4];
    read_words(c, d, h, 4);
    const uint32_t ng = (uint32_t)h[3];
    if (ng) {   // the giant buckets (Zipf head keys): many workgroups each
        std::vector<uint32_t> bl(3 * (size_t)ng);
        QE_HIP(hipMemcpyAsync(bl.data(), big, bl.size() * 4, hipMemcpyDeviceToHost, c->stream));
        QE_HIP(hipStreamSynchronize(c->stream));
        uint32_t mx[2] = {1, 1};
        for (uint32_t g = 0; g < ng; g++)
            for (int sd = 0; sd < 2; sd++) mx[sd] = std::max(mx[sd], bl[3 * g + 1 + sd]);
        const size_t D = (size_t)1 << L;
        uint32_t* gc = dalloc_t<uint32_t>(c, (size_t)ng * D);
        Timed t(c, "agg_big", 0.0);   // (its bytes are counted in agg_count)
        for (int phase = 0; phase < 2; phase++) {
            const int cs = phase == 0 ? 1 : 0, ls = phase == 0 ? 0 : 1;   // count side, lookup side
            const uint64_t* wc = cs ? wS : wR;
            const uint32_t* bc = cs ? bsS : bsR;
            const uint64_t* wl = ls ? wS : wR;
            const uint32_t* bl_ = ls ? bsS : bsR;
            QE_HIP(hipMemsetAsync(gc, 0, (size_t)ng * D * 4, c->stream));
            hipLaunchKernelGGL(ab_big_count_kernel, dim3((mx[cs] + AB_CHUNK - 1) / AB_CHUNK, ng), dim3(AB_NT), 0, c->stream,
                               wc, bc, big, cs, L, gc);
            QE_HIP(hipGetLastError());
            hipLaunchKernelGGL(ab_big_look_kernel, dim3((mx[ls] + AB_CHUNK - 1) / AB_CHUNK, ng), dim3(AB_NT), 0, c->stream,
                               wl, bl_, big, ls, L, gc, phase == 0 ? 1 : 0, d);
            QE_HIP(hipGetLastError());
        }
        read_words(c, d, h, 3);
        dfree(c, gc);
    }
    out[0] = h[0];
    out[1] = h[1];
    out[2] = h[2];
    for (void* p : {(void*)wR, (void*)wS, (void*)bsR, (void*)bsS, (void*)part, (void*)big, (void*)d}) dfree(c, p);
}

// OR / AND of a column: the load-time statistics of a relation column, else one pass
static void col_bits(qe_ctx* c, const uint64_t* d, uint64_t n, uint64_t kb[2]) {
    for (const Relation& r : c->rels)
        for (size_t j = 0; j < r.cols.size(); j++)
            if (r.cols[j] == d && r.rows == n && j < r.kor.size()) {
                kb[0] = r.kor[j];
                kb[1] = r.kand[j];
                return;
            }
    key_bits_u64(c, d, n, kb);
}

}  // namespace qe

#ifdef QE_DIAG_STAMPS
extern "C" int qe_diag_stamps_ag(uint64_t* out, uint64_t n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(qe::g_ag_stamps), n * 8) == hipSuccess ? 0 : -2;
}
#endif

namespace qe {

void join_aggregate_sides(qe_ctx* c, const AggSide& R, const AggSide& S, uint64_t out[3]) {
    const uint64_t nR = R.n, nS = S.n;
    out[0] = out[1] = out[2] = 0;
    if (nR == 0 || nS == 0) return;
    if (nR >= 0xFFFFFFFFull || nS >= 0xFFFFFFFFull) throw Error(QE_ENOTSUP, "aggregate join side beyond 2^32 rows");
    const uint64_t vary = (R.kb[0] | S.kb[0]) & ~(R.kb[1] & S.kb[1]);
    int lo = 0, nb = 0;
    if (vary) {
        lo = __builtin_ctzll(vary);
        nb = 64 - __builtin_clzll(vary) - lo;
    }
    // (bits outside the field are equal in every key of both sides: comparing fields is exact)
    if (nb > 32) throw Error(QE_ENOTSUP, "aggregate join keys vary in more than 32 bits");
    if (agg_buckets_on() && nb > AGG_BUCKET_BITS && nb <= AGG_BUCKET_BITS + 15 && nR + nS >= (1ull << 22)) {
        join_aggregate_buckets(c, R, S, lo, nb, out);   // two partition passes per side, LDS counting
        if (!R.v64 && !R.v32) out[1] = 0;
        if (!S.v64 && !S.v32) out[2] = 0;
        return;
    }
    uint64_t* wR = sort_words_kv64(c, R.keys, R.v64, nR, lo, nb, R.v32);
    uint64_t* wS = sort_words_kv64(c, S.keys, S.v64, nS, lo, nb, S.v32);
    const uint64_t m = nR + nS;
    const uint32_t nt = (uint32_t)((m + AG_T - 1) / AG_T);
    uint64_t* ra = dalloc_t<uint64_t>(c, (uint64_t)nt + 1);
    uint32_t* bk = dalloc_t<uint32_t>(c, (uint64_t)nt + 1);
    uint32_t* bcR = dalloc_t<uint32_t>(c, (uint64_t)nt + 1);
    uint32_t* bcS = dalloc_t<uint32_t>(c, (uint64_t)nt + 1);
    // persistent tile kernel: as many workgroups as stay resident
    static int resident = [&] {
        int ncu = 0, per = 0;
        QE_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device));
        QE_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, ag_tile_kernel, AG_NT, 0));
        return std::max(ncu, 1) * std::max(per, 1);
    }();
    const uint32_t grid = std::max<uint32_t>(1, std::min<uint32_t>(nt, (uint32_t)resident));
    uint64_t* partial = dalloc_t<uint64_t>(c, (uint64_t)grid * 3);
    uint64_t* d_out = c->d_scratch + 48;   // [pairs, sum R, sum S]
    {
        Timed t(c, "agg_split", 0);
        hipLaunchKernelGGL(ag_split_kernel, dim3((nt + 1 + 255) / 256), dim3(256), 0, c->stream, wR, nR, wS, nS, nt, ra, bk,
                           bcR, bcS);
        QE_HIP(hipGetLastError());
    }
    {
        Timed t(c, "agg_count", 8.0 * (double)m);
        hipLaunchKernelGGL(ag_tile_kernel, dim3(grid), dim3(AG_NT), 0, c->stream, wR, nR, wS, nS, nt, ra, bk, bcR, bcS,
                           partial);
        QE_HIP(hipGetLastError());
        hipLaunchKernelGGL(ag_reduce_kernel, dim3(1), dim3(1024), 0, c->stream, partial, grid, d_out);
        QE_HIP(hipGetLastError());
    }
    read_words(c, d_out, out, 3);
    if (!R.v64 && !R.v32) out[1] = 0;   // (the words carried row indices)
    if (!S.v64 && !S.v32) out[2] = 0;
    for (void* p : {(void*)wR, (void*)wS, (void*)ra, (void*)bk, (void*)bcR, (void*)bcS, (void*)partial}) dfree(c, p);
}

}  // namespace qe

using namespace qe;

extern "C" int qe_join_aggregate(qe_ctx* c, qe_col keyR, qe_col valR, qe_col keyS, qe_col valS, uint64_t* out) {
    QE_API_BEGIN(c)
    if (!out) throw Error(QE_EINVAL, "null output");
    if (!keyR.d || !keyS.d) throw Error(QE_EINVAL, "null key column");
    if ((valR.d && valR.n != keyR.n) || (valS.d && valS.n != keyS.n))
        throw Error(QE_EINVAL, "value column length differs from its key column");
    out[0] = out[1] = out[2] = 0;
    if (keyR.n == 0 || keyS.n == 0) return 0;
    if (keyR.n >= 0xFFFFFFFFull || keyS.n >= 0xFFFFFFFFull) throw Error(QE_ENOTSUP, "aggregate join side beyond 2^32 rows");
    AggSide R{keyR.d, valR.d, nullptr, keyR.n, {0, 0}}, S{keyS.d, valS.d, nullptr, keyS.n, {0, 0}};
    col_bits(c, keyR.d, keyR.n, R.kb);
    col_bits(c, keyS.d, keyS.n, S.kb);
    for (const qe_col* v : {&valR, &valS}) {
        if (!v->d) continue;
        uint64_t vb[2];
        col_bits(c, v->d, v->n, vb);
        if (vb[0] >> 32) throw Error(QE_ENOTSUP, "aggregate join value column beyond 32 bits");
    }
    join_aggregate_sides(c, R, S, out);
    return 0;
    QE_API_END(c)
}
