// qe_join.hip -- merge join, payload propagation, gathers and checksums on gfx950.
//
// merge join (reference join_relations, src/join.c:325-392) on sorted inputs:
//   mj_partition -- one binary search pair per R tile: the S window [lo, hi) the tile can match
//   mj_fused     -- per tile: R keys + the S window staged in LDS, each thread bounds its 8
//                   consecutive R keys' matches with interleaved branchless binary searches,
//                   block scan, decoupled lookback for the tile's output offset (published
//                   before the pairs are staged in LDS), one coalesced store of the tile's pairs
//   mj_tile<0>   -- the same walk, tile match count -> global exclusive scan (tile_scan): the
//                   exact two-pass form when the output outgrows the single pass's buffers
//   mj_tile<1>   -- recompute, block scan, then a load-balanced expansion: output slot o of the
//                   tile finds its R element by binary search over the tile's prefix sums, so
//                   every write of outR/outS is coalesced whatever the fan-out
// Output order = key, then R order, then S order: exactly the reference's nested loop.
// Unsorted inputs (possible in the reference's state machine) take
// merge_sequential, an exact parallel form of the literal two-pointer loop, so results stay
// identical there too.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>

#include "qe_device.h"
#include "qe_internal.h"

namespace qe {

// 512 threads x 8 = 4096 R rows per tile with an 8192-key S window: half the tiles (and lookbacks
// and window searches) of 256 x 8, at three tiles per CU for 32-bit keys -- same-box A/B
// 1.10 -> 0.98 ms per 1e8 x 1e8 join
#ifndef QE_MJB
#define QE_MJB 512
#endif
#ifndef QE_MJ_WIN
#define QE_MJ_WIN 8192
#endif
constexpr int MJB = QE_MJB;               // threads per merge tile
constexpr int MJ_ITEMS = 8;
constexpr int MJ_TILE = MJB * MJ_ITEMS;   // 4096 R elements per tile
constexpr int MJ_WIN = QE_MJ_WIN;         // S keys staged in LDS (64 KiB as u64, 32 KiB as u32)
// a tile with more pairs than this is not emitted by its own workgroup: it is listed and
// expanded afterwards by mj_heavy_prep + mj_heavy_emit, MJ_HEAVY_CHUNK pairs per workgroup
// (a skewed key can put 1e8 pairs in one tile)
constexpr uint64_t MJ_HEAVY_DEFER = 1ull << 20;
constexpr uint64_t MJ_HEAVY_CHUNK = 1ull << 16;

// MJF_* flags: qe_internal.h

template <class F>
__device__ __forceinline__ uint64_t lower_bound_f(uint64_t lo, uint64_t hi, uint64_t key, F at) {
    while (lo < hi) {
        uint64_t mid = lo + ((hi - lo) >> 1);
        if (at(mid) < key) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
template <class F>
__device__ __forceinline__ uint64_t upper_bound_f(uint64_t lo, uint64_t hi, uint64_t key, F at) {
    while (lo < hi) {
        uint64_t mid = lo + ((hi - lo) >> 1);
        if (at(mid) <= key) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// zero_a / zero_b (nullable): result words of the merge that follows, cleared here instead of by
// two memset launches
// Each R tile's S window [lower_bound(first key), upper_bound(last key)).  ONE WAVE per tile, both
// searches 64-ary: every step the lanes probe 64 evenly spaced keys of the remaining range and a
// ballot narrows it 64-fold -- ~4 dependent loads for 10^7 keys instead of the ~2 x 23 of a
// thread-serial binary search pair (round 4: ~24 us per C4 merge, latency-bound).
__device__ __forceinline__ uint64_t wave_bound(const uint64_t* __restrict__ sk, uint64_t nS, uint64_t key, bool upper) {
    const int l = lane_id();
    uint64_t lo = 0, hi = nS;   // the first index whose key is not below (upper: not at or below) key is in [lo, hi]
    for (;;) {   // (wave-uniform)
        const uint64_t n = hi - lo;
        if (n <= 64) {
            bool p = false;
            if ((uint64_t)l < n) {
                const uint64_t v = sk[lo + (uint64_t)l];
                p = upper ? v <= key : v < key;
            }
            return lo + (uint64_t)__popcll(__ballot(p));
        }
        const uint64_t step = (n + 63) / 64, idx = lo + (uint64_t)l * step;
        bool p = false;
        if (idx < hi) {
            const uint64_t v = sk[idx];
            p = upper ? v <= key : v < key;
        }
        const uint64_t c = (uint64_t)__popcll(__ballot(p));   // probes 0 .. c-1 hold
        const uint64_t nv = (n + step - 1) / step;              // probes inside [lo, hi)
        const uint64_t nlo = c ? lo + (c - 1) * step + 1 : lo;
        const uint64_t nhi = c < nv ? lo + c * step : hi;
        lo = nlo;
        hi = nhi;
    }
}

__global__ void __launch_bounds__(256) mj_partition(const uint64_t* __restrict__ rk, uint64_t nR,
                                                    const uint64_t* __restrict__ sk, uint64_t nS, uint32_t ntiles,
                                                    uint64_t* __restrict__ win, uint64_t* zero_a, uint64_t* zero_b) {
    const uint32_t t = blockIdx.x * 4u + (uint32_t)wave_id();
    if (t == 0 && lane_id() == 0) {
        if (zero_a) *zero_a = 0;
        if (zero_b) *zero_b = 0;
    }
    if (t >= ntiles) return;   // (wave-uniform)
    const uint64_t first = (uint64_t)t * MJ_TILE;
    const uint64_t last = std::min<uint64_t>(nR, first + MJ_TILE) - 1;
    const uint64_t lb = wave_bound(sk, nS, rk[first], false), ub = wave_bound(sk, nS, rk[last], true);
    if (lane_id() == 0) {
        win[2 * t] = lb;
        win[2 * t + 1] = ub;
    }
}

// exclusive scan of `n` uint64 counts in place, single block (n = tiles, small); total -> *total
__global__ void __launch_bounds__(1024) tile_scan_kernel(uint64_t* __restrict__ v, uint64_t n, uint64_t* total) {
    __shared__ uint64_t wsum[16];
    __shared__ uint64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint64_t base = 0; base < n; base += 1024) {
        uint64_t i = base + threadIdx.x;
        uint64_t x = i < n ? v[i] : 0;
        uint64_t inc = wave_incl_scan_u64(x);
        if (lane_id() == 63) wsum[wave_id()] = inc;
        __syncthreads();
        uint64_t add = carry;
        for (int w = 0; w < wave_id(); w++) add += wsum[w];
        if (i < n) v[i] = inc - x + add;
        __syncthreads();
        if (threadIdx.x == 1023) carry = add + inc;
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry;
}

// the same scan for long arrays: chunk sums, one block over them (tile_scan_kernel), then every
// chunk rescanned from its base -- the single block walked 1024 values per step and took ~0.8 ms
// per C4 seq_merge candidate count (profiles/r03_c4_timeline.txt)
constexpr uint32_t SCAN_PER = 8, SCAN_CH = 1024 * SCAN_PER;
__global__ void __launch_bounds__(1024) chunk_sum_u64_kernel(const uint64_t* __restrict__ v, uint64_t n,
                                                             uint64_t* __restrict__ part) {
    __shared__ uint64_t wsum[16];
    const uint64_t i0 = (uint64_t)blockIdx.x * SCAN_CH + (uint64_t)threadIdx.x * SCAN_PER;
    uint64_t s = 0;
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER; k++) s += i0 + k < n ? v[i0 + k] : 0ull;
    const uint64_t inc = wave_incl_scan_u64(s);
    if (lane_id() == 63) wsum[wave_id()] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int w = 0; w < 16; w++) t += wsum[w];
        part[blockIdx.x] = t;
    }
}

__global__ void __launch_bounds__(1024) chunk_scan_u64_kernel(uint64_t* __restrict__ v, uint64_t n,
                                                              const uint64_t* __restrict__ part) {
    __shared__ uint64_t wsum[16];
    const uint64_t i0 = (uint64_t)blockIdx.x * SCAN_CH + (uint64_t)threadIdx.x * SCAN_PER;
    uint64_t x[SCAN_PER], s = 0;
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER; k++) {
        x[k] = i0 + k < n ? v[i0 + k] : 0ull;
        s += x[k];
    }
    const uint64_t inc = wave_incl_scan_u64(s);
    if (lane_id() == 63) wsum[wave_id()] = inc;
    __syncthreads();
    uint64_t run = part[blockIdx.x] + inc - s;
    for (int w = 0; w < wave_id(); w++) run += wsum[w];
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER; k++) {
        if (i0 + k < n) v[i0 + k] = run;
        run += x[k];
    }
}

// exclusive scan of n u64 in place on the ctx stream; the total lands in *total (device)
static void scan_u64(qe_ctx* c, uint64_t* v, uint64_t n, uint64_t* total) {
    if (n <= 4 * SCAN_CH) {
        hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, c->stream, v, n, total);
        QE_HIP(hipGetLastError());
        return;
    }
    const uint64_t nb = (n + SCAN_CH - 1) / SCAN_CH;
    uint64_t* part = dalloc_t<uint64_t>(c, nb);
    hipLaunchKernelGGL(chunk_sum_u64_kernel, dim3((unsigned)nb), dim3(1024), 0, c->stream, v, n, part);
    QE_HIP(hipGetLastError());
    hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, c->stream, part, nb, total);
    QE_HIP(hipGetLastError());
    hipLaunchKernelGGL(chunk_scan_u64_kernel, dim3((unsigned)nb), dim3(1024), 0, c->stream, v, n, part);
    QE_HIP(hipGetLastError());
    dfree(c, part);
}

// S window and output staging are XOR-swizzled: thread t's walk reads S near 8t and its emitted
// run starts near 8t, so unswizzled the lanes of a wave would hit 4 (u64) / 8 (u32) banks.
// Both swizzles permute within aligned groups of 8, so linear sweeps stay conflict-free.
__device__ __forceinline__ uint32_t sw64(uint32_t i) { return i ^ ((i >> 5) & 7u); }
__device__ __forceinline__ uint32_t sw32(uint32_t o) { return o ^ ((o >> 6) & 7u); }

// R keys live in LDS with one pad slot per 8: thread t walks elements 8t..8t+7, and without the
// pad the 32 lanes of a ds_read_b64 group would hit 4 banks (8-way conflict)
__device__ __forceinline__ uint32_t rpad(uint32_t e) { return e + (e >> 3); }

// KT = uint64_t: keys as they are.  KT = uint32_t: key - (the tile's first R key): every key a tile
// touches lies in [first R key, last R key] (the S window is bounded by those), so when R's
// varying bits are all below bit 32 the tile works on 32-bit offsets -- one-op compares in the
// VALU-bound walk, half the LDS bytes, and (with a 1.5x output stage) 4 workgroups per CU.
template <typename KT, int OUTCAP, int WIN = MJ_WIN>
struct MJSharedG {
    using Key = KT;
    static constexpr int kOutCap = OUTCAP;   // pairs a balanced tile stages in LDS
    static constexpr int kWin = WIN;         // S keys a tile stages in LDS (a wider window: global walk)
    static_assert(WIN % MJB == 0, "the window is staged MJB keys per round");
    KT r[MJ_TILE + MJ_TILE / 8];
    union {                       // the S window is dead once every thread has walked (a barrier
        KT s[WIN];                // separates the walk from the emission's use of the space)
        struct {
            uint32_t lo[MJ_TILE];     // window-relative S start per R element
            uint32_t off[MJ_TILE];    // tile-relative output offset per R element
        };
        struct {
            uint32_t oR[OUTCAP];      // a balanced tile's pairs, staged for coalesced stores
            uint32_t oS[OUTCAP];
        };
    };
    uint64_t red[MJB / 64];
    uint64_t excl;
    uint32_t flag;
    uint32_t ticket;
};
using MJShared64 = MJSharedG<uint64_t, 2 * MJ_TILE>;
// 1.375 pairs per R row staged (with 256-thread tiles: 31.8 KiB of LDS, FIVE workgroups per CU
// against four at 1.5) -- more tiles in flight to cover the lookback wait (stamps: ~6 us of a
// ~26 us tile)
#ifndef QE_MJ32_OUTCAP
#define QE_MJ32_OUTCAP (11 * MJ_TILE / 8)
#endif
// S window of the 32-bit tile, tunable separately from the 64-bit one.  A 4096-row R tile spans
// |S|/|R| x 4096 S keys, so one of C3's joins (|S|/|R| ~ 2.15) puts ~8800 behind each tile --
// past 8192 -- and walks S in global memory.  A 12288-key window (48 KiB, still two workgroups
// per CU) was measured against 8192 on one box (C3 mj_fused 2.98 vs 2.95 ms per query, end to
// end 20.0 vs 20.0 ms): no gain -- the wider staging costs what the LDS walk saves -- so 8192 stays
#ifndef QE_MJ32_WIN
#define QE_MJ32_WIN MJ_WIN
#endif
using MJShared32 = MJSharedG<uint32_t, QE_MJ32_OUTCAP, QE_MJ32_WIN>;
// 1.0625 pairs per R row (256-thread tiles: 26.0 KiB, SIX workgroups per CU) -- for |S| <= |R|,
// where the mean fan-out per R row is at most ~1 (C3's joins: 3.19 -> 3.00 ms per query, same-box
// A/B); a tile with more pairs takes the binary-search emission
using MJShared32s = MJSharedG<uint32_t, 17 * MJ_TILE / 16>;

// bank swizzle of the S window for the key width (sw64: u64 slots, sw32: u32 slots)
template <typename KT>
__device__ __forceinline__ uint32_t swz(uint32_t i) {
    if constexpr (sizeof(KT) == 8) return sw64(i);
    else return sw32(i);
}

// stage the tile's R keys and (when it fits) its S window in LDS.  Every load of the tile is
// issued before the first LDS store: 24 independent loads in flight per thread instead of one
// (a load -> store loop leaves ~6 KB in flight per CU, a quarter of what HBM needs).
template <class SH>
__device__ __forceinline__ void mj_stage(SH& sh, const uint64_t* rk, uint64_t base, uint32_t tn,
                                         const uint64_t* sk, uint64_t wlo, uint64_t wn, uint64_t kbase) {
    using KT = typename SH::Key;
    if (threadIdx.x == 0) sh.flag = 0;
    constexpr int RS = MJ_TILE / MJB, SS = SH::kWin / MJB;
    uint64_t rr[RS], ss[SS];
    const uint32_t t = threadIdx.x;
    if (tn == MJ_TILE) {   // base is a multiple of MJ_TILE: 16-B aligned pairs
        const uint4* r4 = reinterpret_cast<const uint4*>(rk + base);
#pragma unroll
        for (int k = 0; k < RS / 2; k++) {
            uint4 v = r4[t + k * MJB];
            rr[2 * k] = ((uint64_t)v.y << 32) | v.x;
            rr[2 * k + 1] = ((uint64_t)v.w << 32) | v.z;
        }
    } else {
#pragma unroll
        for (int k = 0; k < RS / 2; k++) {
            uint32_t i = 2 * (t + k * MJB);
            rr[2 * k] = i < tn ? rk[base + i] : 0;
            rr[2 * k + 1] = i + 1 < tn ? rk[base + i + 1] : 0;
        }
    }
    const bool sw = wn <= (uint64_t)SH::kWin;
    if (sw) {
#pragma unroll
        for (int k = 0; k < SS; k++) {
            uint32_t i = t + k * MJB;
            ss[k] = i < wn ? sk[wlo + i] : 0;
        }
    }
#pragma unroll
    for (int k = 0; k < RS / 2; k++) {
        uint32_t i = 2 * (t + k * MJB);
        if (i < tn) sh.r[rpad(i)] = (KT)(rr[2 * k] - kbase);
        if (i + 1 < tn) sh.r[rpad(i + 1)] = (KT)(rr[2 * k + 1] - kbase);
    }
    if (sw) {
#pragma unroll
        for (int k = 0; k < SS; k++) {
            uint32_t i = t + k * MJB;
            if (i < wn) sh.s[swz<KT>(i)] = (KT)(ss[k] - kbase);
        }
    }
    __syncthreads();
}

// each thread finds [lo, hi) in the S window for its MJ_ITEMS consecutive R keys:
//   1. the thread's range [a, b) = [lower_bound(first key), upper_bound(last key)): two
//      interleaved binary searches over the window;
//   2. MJ_ITEMS independent branchless lower-bound searches inside [a, b) -- a few elements for
//      a balanced join -- all in flight together;
//   3. upper bounds by MJ_PROBE independent equality probes past each lower bound (a binary
//      search only for a run of equal S keys longer than that).
// The walk is VALU-bound (64-bit compares), so the work per key is what this minimises; no
// divergent walk loop, ~log2(window) + log2(b - a) dependent LDS round trips.
// IN_LDS is a template parameter on purpose: a run-time choice between sh.s and sk inside the
// accessor compiles to a pointer select and FLAT loads (global-path latency for LDS data).
constexpr uint32_t MJ_PROBE = 2;
template <bool IN_LDS, class SH>
__device__ __forceinline__ uint64_t mj_walk_t(const SH& sh, const uint64_t* sk, uint64_t wlo, uint64_t wn64,
                                              uint32_t tn, uint64_t kbase, uint32_t (&cnt)[MJ_ITEMS],
                                              uint32_t (&lo_rel)[MJ_ITEMS]) {
    using KT = typename SH::Key;
    const uint32_t wn = (uint32_t)wn64;   // window-relative positions: nS < 2^32
    auto S = [&](uint32_t i) -> KT {
        if constexpr (IN_LDS) return sh.s[swz<KT>(i)];
        else return (KT)(sk[wlo + i] - kbase);
    };
    const uint32_t e0 = threadIdx.x * MJ_ITEMS;
    const uint32_t nv = tn > e0 ? (tn - e0 < (uint32_t)MJ_ITEMS ? tn - e0 : (uint32_t)MJ_ITEMS) : 0u;
#pragma unroll
    for (int j = 0; j < MJ_ITEMS; j++) {
        cnt[j] = 0;
        lo_rel[j] = 0;
    }
    if (nv == 0) return 0;
    KT key[MJ_ITEMS];
#pragma unroll
    for (int j = 0; j < MJ_ITEMS; j++) key[j] = sh.r[rpad(e0 + ((uint32_t)j < nv ? (uint32_t)j : nv - 1))];
    const KT klast = key[MJ_ITEMS - 1];   // = the last valid key (padded above)
    uint32_t a = 0, an = wn, b = 0, bn = wn;
    while (an | bn) {
        if (an) {
            const uint32_t h = an >> 1;
            if (S(a + h) < key[0]) {
                a += h + 1;
                an -= h + 1;
            } else {
                an = h;
            }
        }
        if (bn) {
            const uint32_t h = bn >> 1;
            if (S(b + h) <= klast) {
                b += h + 1;
                bn -= h + 1;
            } else {
                bn = h;
            }
        }
    }
    if (key[0] == klast) {   // one key for all of the thread's rows (inside a skewed key's run):
        uint64_t tsum = 0;    // [a, b) is already its S run
#pragma unroll
        for (int j = 0; j < MJ_ITEMS; j++) {
            if ((uint32_t)j < nv) {
                cnt[j] = b - a;
                lo_rel[j] = a;
                tsum += b - a;
            }
        }
        return tsum;
    }
    uint32_t lo[MJ_ITEMS], ln[MJ_ITEMS];
#pragma unroll
    for (int j = 0; j < MJ_ITEMS; j++) {
        lo[j] = a;
        ln[j] = b - a;
    }
    for (uint32_t rem = b - a; rem; rem >>= 1) {   // ceil(log2(b - a + 1)) rounds
#pragma unroll
        for (int j = 0; j < MJ_ITEMS; j++) {
            if (ln[j]) {
                const uint32_t h = ln[j] >> 1;
                if (S(lo[j] + h) < key[j]) {
                    lo[j] += h + 1;
                    ln[j] -= h + 1;
                } else {
                    ln[j] = h;
                }
            }
        }
    }
    uint32_t hi[MJ_ITEMS];
    bool open[MJ_ITEMS];
#pragma unroll
    for (int j = 0; j < MJ_ITEMS; j++) {
        hi[j] = lo[j];
        open[j] = true;
    }
#pragma unroll
    for (uint32_t q = 0; q < MJ_PROBE; q++) {
#pragma unroll
        for (int j = 0; j < MJ_ITEMS; j++) {
            if (open[j]) {
                if (hi[j] < b && S(hi[j]) == key[j]) hi[j]++;
                else open[j] = false;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < MJ_ITEMS; j++) {   // a run longer than the probes: binary search
        if (open[j] && hi[j] < b && S(hi[j]) == key[j]) {
            uint32_t hn = b - hi[j];
            while (hn) {
                const uint32_t h = hn >> 1;
                if (S(hi[j] + h) <= key[j]) {
                    hi[j] += h + 1;
                    hn -= h + 1;
                } else {
                    hn = h;
                }
            }
        }
    }
    uint64_t tsum = 0;
#pragma unroll
    for (int j = 0; j < MJ_ITEMS; j++) {
        if ((uint32_t)j < nv) {
            cnt[j] = hi[j] - lo[j];
            lo_rel[j] = lo[j];
            tsum += cnt[j];
        }
    }
    return tsum;
}

template <class SH>
__device__ __forceinline__ uint64_t mj_walk(const SH& sh, const uint64_t* sk, uint64_t wlo, uint64_t wn,
                                            uint32_t tn, uint64_t kbase, uint32_t (&cnt)[MJ_ITEMS],
                                            uint32_t (&lo_rel)[MJ_ITEMS]) {
    if (wn <= (uint64_t)SH::kWin) return mj_walk_t<true>(sh, sk, wlo, wn, tn, kbase, cnt, lo_rel);
    // a window beyond LDS: inside a skewed key's run.  When the whole R tile holds one key the
    // window [lower_bound(first), upper_bound(last)) IS that key's S run -- every row matches all
    // of it, no search (the per-thread global binary searches cost ~24 dependent HBM round trips)
    if (tn && sh.r[rpad(0)] == sh.r[rpad(tn - 1)]) {
        const uint32_t e0 = threadIdx.x * MJ_ITEMS;
        uint64_t tsum = 0;
#pragma unroll
        for (int j = 0; j < MJ_ITEMS; j++) {
            const bool v = e0 + (uint32_t)j < tn;
            cnt[j] = v ? (uint32_t)wn : 0u;
            lo_rel[j] = 0;
            tsum += v ? wn : 0;
        }
        return tsum;
    }
    return mj_walk_t<false>(sh, sk, wlo, wn, tn, kbase, cnt, lo_rel);
}

// per-row match counts, output-distinctness flags, optional driver-count annotation
template <class SH>
__device__ __forceinline__ uint32_t mj_annotate_rows(const SH& sh, const uint64_t* rk, const uint32_t* rv,
                                                     uint64_t nR, uint64_t base, uint32_t tn, uint64_t kbase,
                                                     const uint32_t (&cnt)[MJ_ITEMS], uint32_t* match,
                                                     uint32_t* annot) {
    uint32_t myflag = 0;
    const uint32_t e0 = threadIdx.x * MJ_ITEMS;
    const bool full = e0 + MJ_ITEMS <= tn;
    if (match && full) {   // this thread's 8 counts: two 16-B stores
        *reinterpret_cast<uint4*>(match + base + e0) = make_uint4(cnt[0], cnt[1], cnt[2], cnt[3]);
        *reinterpret_cast<uint4*>(match + base + e0 + 4) = make_uint4(cnt[4], cnt[5], cnt[6], cnt[7]);
    }
#pragma unroll
    for (int j = 0; j < MJ_ITEMS; j++) {
        uint32_t e = e0 + j;
        if (e >= tn) continue;
        uint32_t c = cnt[j];
        if (c > 1) myflag |= MJF_R_FANOUT;
        if (match && !full) match[base + e] = c;
        if (c > 0) {
            const uint64_t key = kbase + sh.r[rpad(e)];   // back to the full key
            const uint64_t nxt = e + 1 < tn ? kbase + sh.r[rpad(e + 1)] : (base + e + 1 < nR ? rk[base + e + 1] : ~key);
            if (nxt == key) myflag |= MJF_S_DUP;
            if (annot) annot[rv ? rv[base + e] : (uint32_t)(base + e)] = c;
        }
    }
    return myflag;
}

template <class SH>
__device__ __forceinline__ void mj_publish_flags(SH& sh, uint32_t myflag, uint32_t* flags) {
    if (myflag) atomicOr(&sh.flag, myflag);
    __syncthreads();
    if (threadIdx.x == 0 && sh.flag) {
        uint32_t seen = __hip_atomic_load(flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (sh.flag & ~seen) atomicOr(flags, sh.flag);   // one word for the grid: no hot-spot
    }
}

// block-exclusive offsets of the per-thread sums; returns this thread's start, sets *btotal
template <class SH>
__device__ __forceinline__ uint64_t mj_block_scan(SH& sh, uint64_t tsum, uint64_t* btotal) {
    uint64_t inc = wave_incl_scan_u64(tsum);
    if (lane_id() == 63) sh.red[wave_id()] = inc;
    __syncthreads();
    uint64_t add = 0, tot = 0;
    for (int w = 0; w < MJB / 64; w++) {
        if (w < wave_id()) add += sh.red[w];
        tot += sh.red[w];
    }
    *btotal = tot;
    return inc - tsum + add;
}

// A balanced tile (pairs fit the LDS output stage: 2 per R row for u64 keys, 1.5 for u32) builds
// its pairs in LDS -- tile-local offsets only, so this runs while the tile's lookback is in
// flight -- and stores them as one coalesced run.
template <class SH>
__device__ __forceinline__ bool mj_balanced(uint64_t btotal) { return btotal <= (uint64_t)SH::kOutCap; }

template <class SH>
__device__ __forceinline__ void mj_stage_out(SH& sh, const uint32_t* rv, uint64_t base, uint32_t tn,
                                             uint64_t run, const uint32_t (&cnt)[MJ_ITEMS],
                                             const uint32_t (&lo_rel)[MJ_ITEMS]) {
    const uint32_t e0 = threadIdx.x * MJ_ITEMS;
    uint32_t r[MJ_ITEMS];
    if (rv && e0 + MJ_ITEMS <= tn) {
        uint4 a = *reinterpret_cast<const uint4*>(rv + base + e0);
        uint4 b = *reinterpret_cast<const uint4*>(rv + base + e0 + 4);
        r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w;
        r[4] = b.x; r[5] = b.y; r[6] = b.z; r[7] = b.w;
    } else {
#pragma unroll
        for (int j = 0; j < MJ_ITEMS; j++)
            r[j] = e0 + j < tn ? (rv ? rv[base + e0 + j] : (uint32_t)(base + e0 + j)) : 0;
    }
#pragma unroll
    for (int j = 0; j < MJ_ITEMS; j++) {
        if (e0 + j >= tn) continue;
        for (uint32_t k = 0; k < cnt[j]; k++) {
            const uint32_t o = sw32((uint32_t)run + k);
            sh.oR[o] = r[j];
            sh.oS[o] = lo_rel[j] + k;   // window-relative; S payloads gathered at store time
        }
        run += cnt[j];
    }
}

// after a barrier: [gofs, gofs + btotal) <- the staged pairs, four independent S-payload loads in
// flight per thread per round (the window is read in order, so each round's loads coalesce)
template <class SH>
__device__ __forceinline__ void mj_store_out(const SH& sh, const uint32_t* sv, uint64_t wlo, uint64_t btotal,
                                             uint64_t gofs, uint32_t* outR, uint32_t* outS) {
    const uint32_t bt = (uint32_t)btotal;
    for (uint32_t i0 = threadIdx.x; i0 < bt; i0 += 4 * MJB) {
        uint32_t v[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            uint32_t i = i0 + q * MJB;
            uint64_t sidx = wlo + (i < bt ? sh.oS[sw32(i)] : 0);
            v[q] = i < bt ? (sv ? sv[sidx] : (uint32_t)sidx) : 0;
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            uint32_t i = i0 + q * MJB;
            if (i < bt) {
                outR[gofs + i] = sh.oR[sw32(i)];
                outS[gofs + i] = v[q];
            }
        }
    }
}

// a heavy tile: load-balanced expansion (every output slot finds its R row by binary search)
template <class SH>
__device__ __forceinline__ void mj_emit_heavy(SH& sh, const uint32_t* rv, const uint32_t* sv, uint64_t base,
                                              uint32_t tn, uint64_t wlo, uint64_t run, uint64_t btotal, uint64_t gofs,
                                              const uint32_t (&cnt)[MJ_ITEMS], const uint32_t (&lo_rel)[MJ_ITEMS],
                                              uint32_t* outR, uint32_t* outS) {
    const uint32_t e0 = threadIdx.x * MJ_ITEMS;
#pragma unroll
    for (int j = 0; j < MJ_ITEMS; j++) {
        uint32_t e = e0 + j;
        if (e < tn) {
            sh.off[e] = (uint32_t)run;
            sh.lo[e] = lo_rel[j];
            run += cnt[j];
        }
    }
    __syncthreads();
    for (uint64_t o = threadIdx.x; o < btotal; o += MJB) {
        uint32_t a = 0, b = tn;   // last element with off[e] <= o
        while (b - a > 1) {
            uint32_t m = (a + b) >> 1;
            if (sh.off[m] <= o) a = m;
            else b = m;
        }
        uint64_t sidx = wlo + sh.lo[a] + (o - sh.off[a]);
        outR[gofs + o] = rv ? rv[base + a] : (uint32_t)(base + a);
        outS[gofs + o] = sv ? sv[sidx] : (uint32_t)sidx;
    }
}

// Two-pass form.  WRITE = 0: per-tile counts + flags (+ match counts / driver annotation);
// WRITE = 1: pairs at the scanned tile offsets.
template <int WRITE>
__global__ void __launch_bounds__(MJB) mj_tile(const uint64_t* __restrict__ rk, const uint32_t* __restrict__ rv,
                                               uint64_t nR, const uint64_t* __restrict__ sk,
                                               const uint32_t* __restrict__ sv, uint64_t nS,
                                               const uint64_t* __restrict__ win, uint64_t* __restrict__ tile_counts,
                                               uint32_t* __restrict__ outR, uint32_t* __restrict__ outS,
                                               uint32_t* __restrict__ flags, uint32_t* __restrict__ annot,
                                               uint32_t* __restrict__ match) {
    __shared__ MJShared64 sh;
    const uint32_t tile = blockIdx.x;
    const uint64_t base = (uint64_t)tile * MJ_TILE;
    const uint32_t tn = (uint32_t)std::min<uint64_t>(MJ_TILE, nR - base);
    const uint64_t wlo = win[2 * tile], wn = win[2 * tile + 1] - wlo;
    mj_stage(sh, rk, base, tn, sk, wlo, wn, 0);
    uint32_t cnt[MJ_ITEMS], lo_rel[MJ_ITEMS];
    uint64_t tsum = mj_walk(sh, sk, wlo, wn, tn, 0, cnt, lo_rel);
    if (!WRITE) {
        uint32_t f = mj_annotate_rows(sh, rk, rv, nR, base, tn, 0, cnt, match, annot);
        uint64_t s = wave_sum_u64(tsum);
        if (lane_id() == 0) sh.red[wave_id()] = s;
        mj_publish_flags(sh, f, flags);   // contains the barrier
        if (threadIdx.x == 0) {
            uint64_t tc = 0;
            for (int w = 0; w < MJB / 64; w++) tc += sh.red[w];
            tile_counts[tile] = tc;
        }
        return;
    }
    uint64_t btotal;
    uint64_t run = mj_block_scan(sh, tsum, &btotal);   // barrier: the S window is dead
    const uint64_t gofs = tile_counts[tile];
    if (btotal > MJ_HEAVY_DEFER) return;               // mj_heavy_emit's
    if (mj_balanced<MJShared64>(btotal)) {
        mj_stage_out(sh, rv, base, tn, run, cnt, lo_rel);
        __syncthreads();
        mj_store_out(sh, sv, wlo, btotal, gofs, outR, outS);
    } else {
        mj_emit_heavy(sh, rv, sv, base, tn, wlo, run, btotal, gofs, cnt, lo_rel, outR, outS);
    }
}

// Single-pass form: count, decoupled lookback for the tile's output offset, write -- the keys
// are read once.  Outputs have room for `cap` pairs; a tile that would overflow writes nothing
// and the host re-runs the exact two-pass form (tile_counts is filled for it).
#ifdef QE_DIAG_STAMPS
__device__ uint64_t g_mj_stamps[STAMP_TILES * STAMP_SLOTS];
#endif

template <class SH>
__global__ void __launch_bounds__(MJB) mj_fused(const uint64_t* __restrict__ rk, const uint32_t* __restrict__ rv,
                                                uint64_t nR, const uint64_t* __restrict__ sk,
                                                const uint32_t* __restrict__ sv, uint64_t nS,
                                                const uint64_t* __restrict__ win, uint64_t* __restrict__ tile_counts,
                                                uint32_t* __restrict__ match, uint32_t* __restrict__ outR,
                                                uint32_t* __restrict__ outS, uint64_t cap, uint32_t* __restrict__ flags,
                                                uint64_t* status, uint32_t* ticket, uint32_t epoch, uint32_t ntiles,
                                                uint64_t* total_out, uint32_t* __restrict__ heavy,
                                                uint32_t* __restrict__ nheavy) {
    __shared__ SH sh;
#ifdef QE_DIAG_STAMPS
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
    const uint32_t tile = take_ticket(ticket, &sh.ticket);
#ifdef QE_DIAG_STAMPS
    if (threadIdx.x == 0 && tile < STAMP_TILES) g_mj_stamps[(uint64_t)tile * STAMP_SLOTS] = t_start;
#endif
    const uint64_t base = (uint64_t)tile * MJ_TILE;
    const uint32_t tn = (uint32_t)std::min<uint64_t>(MJ_TILE, nR - base);
    const uint64_t wlo = win[2 * tile], wn = win[2 * tile + 1] - wlo;
    const uint64_t kbase = sizeof(typename SH::Key) == 8 ? 0 : rk[base];   // the tile's first key
    QE_STAMP(g_mj_stamps, tile, 1);
    mj_stage(sh, rk, base, tn, sk, wlo, wn, kbase);
    QE_STAMP(g_mj_stamps, tile, 2);
    uint32_t cnt[MJ_ITEMS], lo_rel[MJ_ITEMS];
    uint64_t tsum = mj_walk(sh, sk, wlo, wn, tn, kbase, cnt, lo_rel);
    QE_STAMP(g_mj_stamps, tile, 6);
    uint32_t f = mj_annotate_rows(sh, rk, rv, nR, base, tn, kbase, cnt, match, nullptr);
    QE_STAMP(g_mj_stamps, tile, 7);
    uint64_t btotal;
    uint64_t run = mj_block_scan(sh, tsum, &btotal);   // barrier: the S window is dead
    QE_STAMP(g_mj_stamps, tile, 3);
    const bool balanced = mj_balanced<SH>(btotal);
#ifndef QE_DIAG_MJ_NOLB
    if (wave_id() == 0) lookback_publish(status, epoch, tile, btotal);
#endif
    if (balanced) mj_stage_out(sh, rv, base, tn, run, cnt, lo_rel);   // overlaps the predecessors
    if (wave_id() == 0) {
#ifdef QE_DIAG_MJ_NOLB   // ablation only: tile offset = its first R row (in range, wrong when fan-out != 1)
        uint64_t ex = base;
#else
        uint64_t ex = lookback_wait(status, epoch, tile, btotal);
#endif
        if (lane_id() == 0) {
            sh.excl = ex;
            tile_counts[tile] = btotal;
            if (tile == ntiles - 1) *total_out = ex + btotal;
            if (btotal > LB_VAL_MASK || ex + btotal > LB_VAL_MASK) atomicOr(flags, MJF_OVF);
        }
    }
    mj_publish_flags(sh, f, flags);   // contains the barrier that publishes sh.excl (and the staging)
    QE_STAMP(g_mj_stamps, tile, 4);
    const uint64_t gofs = sh.excl;
#ifdef QE_DIAG_MJ_NOEMIT
    if (gofs + btotal > cap + 1) outR[0] = (uint32_t)run;   // keep the walk alive, store nothing
#else
    if (btotal > MJ_HEAVY_DEFER) {
        if (heavy && threadIdx.x == 0) heavy[atomicAdd(nheavy, 1u)] = tile;
    } else if (gofs + btotal <= cap) {
        if (balanced) mj_store_out(sh, sv, wlo, btotal, gofs, outR, outS);
        else mj_emit_heavy(sh, rv, sv, base, tn, wlo, run, btotal, gofs, cnt, lo_rel, outR, outS);
    }
#endif
    QE_STAMP(g_mj_stamps, tile, 5);
}

// ---- deferred heavy tiles ------------------------------------------------------------------------
// prep: one workgroup per listed tile re-walks it and leaves, per R row, its absolute S start
// and its u64 output offset inside the tile (plus the tile's total)
__global__ void __launch_bounds__(MJB) mj_heavy_prep(const uint64_t* __restrict__ rk, uint64_t nR,
                                                     const uint64_t* __restrict__ sk, const uint64_t* __restrict__ win,
                                                     const uint32_t* __restrict__ heavy, uint32_t* __restrict__ hp_lo,
                                                     uint64_t* __restrict__ hp_off, uint64_t* __restrict__ hp_tot) {
    __shared__ MJShared64 sh;
    const uint32_t k = blockIdx.x;
    const uint32_t tile = heavy[k];
    const uint64_t base = (uint64_t)tile * MJ_TILE;
    const uint32_t tn = (uint32_t)std::min<uint64_t>(MJ_TILE, nR - base);
    const uint64_t wlo = win[2 * tile], wn = win[2 * tile + 1] - wlo;
    mj_stage(sh, rk, base, tn, sk, wlo, wn, 0);
    uint32_t cnt[MJ_ITEMS], lo_rel[MJ_ITEMS];
    const uint64_t tsum = mj_walk(sh, sk, wlo, wn, tn, 0, cnt, lo_rel);
    uint64_t btotal;
    uint64_t run = mj_block_scan(sh, tsum, &btotal);
    const uint32_t e0 = threadIdx.x * MJ_ITEMS;
#pragma unroll
    for (int j = 0; j < MJ_ITEMS; j++) {
        const uint32_t e = e0 + j;
        if (e < tn) {
            hp_lo[(uint64_t)k * MJ_TILE + e] = (uint32_t)(wlo + lo_rel[j]);
            hp_off[(uint64_t)k * MJ_TILE + e] = run;
            run += cnt[j];
        }
    }
    if (threadIdx.x == 0) hp_tot[k] = btotal;
}

// emit: one workgroup per MJ_HEAVY_CHUNK output slots of one listed tile; every slot finds its
// R row by binary search over the tile's offsets (staged in LDS); stores are coalesced
__global__ void __launch_bounds__(MJB) mj_heavy_emit(const uint32_t* __restrict__ rv, const uint32_t* __restrict__ sv,
                                                     uint64_t nR, const uint32_t* __restrict__ heavy,
                                                     const uint32_t* __restrict__ hp_lo,
                                                     const uint64_t* __restrict__ hp_off,
                                                     const uint64_t* __restrict__ hp_tot,
                                                     const uint32_t* __restrict__ chunk_k,
                                                     const uint64_t* __restrict__ chunk_start,
                                                     const uint64_t* __restrict__ tile_ofs, uint32_t* __restrict__ outR,
                                                     uint32_t* __restrict__ outS) {
    __shared__ uint64_t off[MJ_TILE];
    __shared__ uint32_t lo[MJ_TILE];
    const uint32_t k = chunk_k[blockIdx.x];
    const uint32_t tile = heavy[k];
    const uint64_t base = (uint64_t)tile * MJ_TILE;
    const uint32_t tn = (uint32_t)std::min<uint64_t>(MJ_TILE, nR - base);
    for (uint32_t e = threadIdx.x; e < tn; e += MJB) {
        off[e] = hp_off[(uint64_t)k * MJ_TILE + e];
        lo[e] = hp_lo[(uint64_t)k * MJ_TILE + e];
    }
    __syncthreads();
    const uint64_t c0 = chunk_start[blockIdx.x];
    const uint64_t c1 = std::min<uint64_t>(c0 + MJ_HEAVY_CHUNK, hp_tot[k]);
    const uint64_t gofs = tile_ofs[tile];
    for (uint64_t o = c0 + threadIdx.x; o < c1; o += MJB) {
        uint32_t a = 0, b = tn;   // last row with off <= o
        while (b - a > 1) {
            const uint32_t m = (a + b) >> 1;
            if (off[m] <= o) a = m;
            else b = m;
        }
        const uint64_t sidx = lo[a] + (o - off[a]);
        outR[gofs + o] = rv ? rv[base + a] : (uint32_t)(base + a);
        outS[gofs + o] = sv ? sv[sidx] : (uint32_t)sidx;
    }
}

// ---- the reference's two-pointer loop on UNSORTED inputs (src/join.c:342-377) ---------------------
// Only state-machine paths reach it (SORT_LHS / SORT_RHS on a list whose "sorted"
// mark is stale), never the measured configs.  Per R row the loop moves s_start to
//     f(s, k) = the first p >= s with S[p] >= k        (k = the row's key)
// and emits the p in [f, first p > f with S[p] > k) with S[p] == k.  Since f(f(s, k1), k2) =
// f(s, max(k1, k2)), the pointer after rows 0..pr is f(0, M) with M = max(R[0..pr]) -- so:
//   * a row can emit only if its key IS that running max M (else S[f] >= M > key: the inner
//     loop breaks at once), and M <= max(S) (else f = |S| and the outer loop has ended);
//   * it then emits exactly the positions where S equals its own running max and that max is
//     M ("record" positions of S with value M), in position order.
// So the loop is two prefix-max scans, two compactions and binary searches -- all parallel and
// exact (it was one lane walking up to 6e7 rows, ~1 s per call, in the C4 batch).
constexpr int PM_B = 256, PM_ITEMS = 16, PM_CHUNK = PM_B * PM_ITEMS;

__device__ __forceinline__ uint64_t wave_incl_max_u64(uint64_t v) {
    const int l = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v, d, 64);
        uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), d, 64);
        const uint64_t o = ((uint64_t)hi << 32) | lo;
        if (l >= d && o > v) v = o;
    }
    return v;
}

__global__ void __launch_bounds__(PM_B) pmax_reduce_kernel(const uint64_t* __restrict__ x, uint64_t n,
                                                           uint64_t* __restrict__ bmax) {
    __shared__ uint64_t red[PM_B / 64];
    const uint64_t base = (uint64_t)blockIdx.x * PM_CHUNK;
    uint64_t m = 0;
#pragma unroll
    for (int j = 0; j < PM_ITEMS; j++) {
        const uint64_t i = base + (uint64_t)j * PM_B + threadIdx.x;
        const uint64_t v = i < n ? x[i] : 0;
        m = v > m ? v : m;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t o = shfl_xor_u64(m, d);
        m = o > m ? o : m;
    }
    if (lane_id() == 0) red[wave_id()] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int w = 0; w < PM_B / 64; w++) t = red[w] > t ? red[w] : t;
        bmax[blockIdx.x] = t;
    }
}

// one block: exclusive prefix max of the block maxima, in place
__global__ void __launch_bounds__(1024) pmax_top_kernel(uint64_t* __restrict__ bmax, uint64_t nb) {
    __shared__ uint64_t wmax[16];
    __shared__ uint64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint64_t base = 0; base < nb; base += 1024) {
        const uint64_t i = base + threadIdx.x;
        const uint64_t x = i < nb ? bmax[i] : 0;
        const uint64_t inc = wave_incl_max_u64(x);
        if (lane_id() == 63) wmax[wave_id()] = inc;
        __syncthreads();
        uint64_t ex = carry;
        for (int w = 0; w < wave_id(); w++) ex = wmax[w] > ex ? wmax[w] : ex;
        const uint64_t prev = shfl_u64(inc, lane_id() == 0 ? 0 : lane_id() - 1);
        const uint64_t mine_ex = lane_id() == 0 ? ex : (prev > ex ? prev : ex);
        if (i < nb) bmax[i] = mine_ex;
        __syncthreads();
        if (threadIdx.x == 1023) carry = mine_ex > x ? mine_ex : x;
        __syncthreads();
    }
}

// out[i] = max(x[0..i]): each thread scans 16 consecutive values, then waves and the block combine
__global__ void __launch_bounds__(PM_B) pmax_apply_kernel(const uint64_t* __restrict__ x, uint64_t n,
                                                          const uint64_t* __restrict__ bex, uint64_t* __restrict__ out) {
    __shared__ uint64_t wmax[PM_B / 64];
    const uint64_t base = (uint64_t)blockIdx.x * PM_CHUNK + (uint64_t)threadIdx.x * PM_ITEMS;
    uint64_t v[PM_ITEMS], run = 0;
#pragma unroll
    for (int j = 0; j < PM_ITEMS; j++) {
        const uint64_t i = base + j;
        v[j] = i < n ? x[i] : 0;
        run = v[j] > run ? v[j] : run;
        v[j] = run;
    }
    const uint64_t inc = wave_incl_max_u64(run);
    if (lane_id() == 63) wmax[wave_id()] = inc;
    __syncthreads();
    uint64_t ex = bex[blockIdx.x];
    for (int w = 0; w < wave_id(); w++) ex = wmax[w] > ex ? wmax[w] : ex;
    const uint64_t prev = shfl_u64(inc, lane_id() == 0 ? 0 : lane_id() - 1);
    if (lane_id() != 0 && prev > ex) ex = prev;
#pragma unroll
    for (int j = 0; j < PM_ITEMS; j++) {
        const uint64_t i = base + j;
        if (i < n) out[i] = v[j] > ex ? v[j] : ex;
    }
}

// per candidate row: the record positions of S whose value equals its key -> [e0, e0 + cnt)
__global__ void __launch_bounds__(256) seqm_count_kernel(const uint64_t* __restrict__ rk, const uint32_t* __restrict__ cand,
                                                         uint64_t nc, const uint64_t* __restrict__ sk,
                                                         const uint32_t* __restrict__ rec, uint64_t nrec,
                                                         uint64_t* __restrict__ cnt, uint32_t* __restrict__ e0s) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nc) return;
    const uint64_t key = rk[cand[i]];
    auto at = [&](uint64_t e) { return sk[rec[e]]; };   // record values are non-decreasing
    const uint64_t e0 = lower_bound_f(0, nrec, key, at);
    const uint64_t e1 = (e0 < nrec && at(e0) == key) ? upper_bound_f(e0, nrec, key, at) : e0;
    cnt[i] = e1 - e0;
    e0s[i] = (uint32_t)e0;
}

__global__ void __launch_bounds__(256) seqm_write_kernel(const uint32_t* __restrict__ rv, const uint32_t* __restrict__ cand,
                                                         uint64_t nc, const uint32_t* __restrict__ sv,
                                                         const uint32_t* __restrict__ rec,
                                                         const uint64_t* __restrict__ off, const uint32_t* __restrict__ e0s,
                                                         uint64_t total, uint32_t* __restrict__ outR,
                                                         uint32_t* __restrict__ outS) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nc) return;
    const uint64_t o = off[i], end = i + 1 < nc ? off[i + 1] : total;
    const uint32_t pr = cand[i];
    const uint32_t r = rv ? rv[pr] : pr;
    for (uint64_t j = 0; o + j < end; j++) {
        const uint32_t p = rec[e0s[i] + j];
        outR[o + j] = r;
        outS[o + j] = sv ? sv[p] : p;
    }
}

__global__ void __launch_bounds__(256) is_sorted_kernel(const uint64_t* __restrict__ k, uint64_t n, uint32_t* bad) {
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    bool b = false;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i + 1 < n; i += stride)
        b |= k[i] > k[i + 1];
    if (__any(b) && lane_id() == 0) atomicOr(bad, 1u);
}

// keys = col[rows] in list order, plus the OR / AND of the gathered keys (the radix sort's
// pass plan) so the sort needs no reduction pass of its own
template <bool BITS>
__global__ void __launch_bounds__(256) gather_keys_kernel(const uint64_t* __restrict__ col,
                                                          const uint32_t* __restrict__ rows, uint64_t n,
                                                          uint64_t* __restrict__ out,
                                                          unsigned long long* __restrict__ bits) {
    uint64_t o = 0, a = ~0ull;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 4;   // bounded grid: few atomics
    for (uint64_t i4 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i4 < n; i4 += stride) {
        if (i4 + 3 < n) {
            uint4 r = *reinterpret_cast<const uint4*>(rows + i4);
            ulonglong2 x, y;
            x.x = col[r.x];
            x.y = col[r.y];
            y.x = col[r.z];
            y.y = col[r.w];
            *reinterpret_cast<ulonglong2*>(out + i4) = x;
            *reinterpret_cast<ulonglong2*>(out + i4 + 2) = y;
            o |= x.x | x.y | y.x | y.y;
            a &= x.x & x.y & y.x & y.y;
        } else {
            for (uint64_t i = i4; i < n; i++) {
                uint64_t k = col[rows[i]];
                out[i] = k;
                o |= k;
                a &= k;
            }
        }
    }
    if constexpr (!BITS) return;   // bounds known (column statistics): no reduction
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        o |= shfl_xor_u64(o, m);
        a &= shfl_xor_u64(a, m);
    }
    __shared__ uint64_t so[4], sa[4];
    if (lane_id() == 0) {
        so[wave_id()] = o;
        sa[wave_id()] = a;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        o = so[0] | so[1] | so[2] | so[3];
        a = sa[0] & sa[1] & sa[2] & sa[3];
        atomicOr(&bits[0], (unsigned long long)o);
        atomicAnd(&bits[1], (unsigned long long)a);
    }
}

// driver counts from the merge's per-row match counts: counts[rowid] = matches (every row of a
// rowid carries the same key, hence the same count: plain stores, no atomics)
__global__ void __launch_bounds__(256) scatter_match_kernel(const uint32_t* __restrict__ val,
                                                            const uint32_t* __restrict__ match, uint64_t n,
                                                            uint32_t* __restrict__ counts) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        uint32_t m = match[i];
        if (m) counts[val ? val[i] : (uint32_t)i] = m;
    }
}

// sum of col[rowid] mod 2^64 (print_sums, src/utilities.c:216-219); rows == null: whole column
__global__ void __launch_bounds__(256) checksum_kernel(const uint64_t* __restrict__ col,
                                                       const uint32_t* __restrict__ rows, uint64_t n,
                                                       unsigned long long* __restrict__ out) {
    uint64_t s = 0;
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 4;
    for (uint64_t i4 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i4 < n; i4 += stride) {
        if (i4 + 3 < n) {
            if (rows) {
                uint4 r = *reinterpret_cast<const uint4*>(rows + i4);
                s += col[r.x] + col[r.y] + col[r.z] + col[r.w];
            } else {
                ulonglong2 a = *reinterpret_cast<const ulonglong2*>(col + i4);
                ulonglong2 b = *reinterpret_cast<const ulonglong2*>(col + i4 + 2);
                s += a.x + a.y + b.x + b.y;
            }
        } else {
            for (uint64_t i = i4; i < n; i++) s += col[rows ? rows[i] : i];
        }
    }
    s = wave_sum_u64(s);
    __shared__ uint64_t red[4];
    if (lane_id() == 0) red[wave_id()] = s;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(out, (unsigned long long)(red[0] + red[1] + red[2] + red[3]));
}

// sum of col[val[i]] * match[i] mod 2^64 over one side of a sorted merge: the checksum of that
// side's output list (each row appears match[i] times) without materialising it -- aggregate
// push-down, SURVEY.md §0.7 / §8(e).  val == null: the rowid is the position.
__global__ void __launch_bounds__(256) checksum_weighted_kernel(const uint64_t* __restrict__ col,
                                                                const uint32_t* __restrict__ val,
                                                                const uint32_t* __restrict__ match, uint64_t n,
                                                                unsigned long long* __restrict__ out) {
    uint64_t s = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 4;
    for (uint64_t i4 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i4 < n; i4 += stride) {
        if (i4 + 3 < n) {
            const uint4 m = *reinterpret_cast<const uint4*>(match + i4);
            uint4 r;
            if (val) r = *reinterpret_cast<const uint4*>(val + i4);
            else r = make_uint4((uint32_t)i4, (uint32_t)i4 + 1, (uint32_t)i4 + 2, (uint32_t)i4 + 3);
            if (m.x) s += col[r.x] * m.x;
            if (m.y) s += col[r.y] * m.y;
            if (m.z) s += col[r.z] * m.z;
            if (m.w) s += col[r.w] * m.w;
        } else {
            for (uint64_t i = i4; i < n; i++)
                if (match[i]) s += col[val ? val[i] : (uint32_t)i] * match[i];
        }
    }
    s = wave_sum_u64(s);
    __shared__ uint64_t red[4];
    if (lane_id() == 0) red[wave_id()] = s;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(out, (unsigned long long)(red[0] + red[1] + red[2] + red[3]));
}

// nonzero bitmap of the driver counts: one sequential pass over the (rows x 4 B) counts array
// leaves rows/8 bytes that stay cache-resident for the pruning pass's random tests, which
// would otherwise fetch a 64-B line of the counts array per 4-B test
__global__ void __launch_bounds__(256) nonzero_bitmap_kernel(const uint32_t* __restrict__ counts, uint64_t rows,
                                                             uint32_t* __restrict__ bm) {
    const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;   // one 32-row word per thread
    const uint64_t r0 = w * 32;
    if (r0 >= rows) return;
    uint32_t bits = 0;
    if (r0 + 32 <= rows) {
        uint4 q[8];
        const uint4* p = reinterpret_cast<const uint4*>(counts + r0);
#pragma unroll
        for (int k = 0; k < 8; k++) q[k] = p[k];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            bits |= (q[k].x ? 1u : 0u) << (4 * k);
            bits |= (q[k].y ? 1u : 0u) << (4 * k + 1);
            bits |= (q[k].z ? 1u : 0u) << (4 * k + 2);
            bits |= (q[k].w ? 1u : 0u) << (4 * k + 3);
        }
    } else {
        for (uint64_t r = r0; r < rows; r++) bits |= (counts[r] ? 1u : 0u) << (r - r0);
    }
    bm[w] = bits;
}

// ---- join_payloads expansion (src/join.c:452-476 on sorted inputs) -------------------------------
// element i (sorted by last) is emitted counts[last[i]] times
constexpr int XB = 256, X_ITEMS = 8, X_TILE = XB * X_ITEMS;

constexpr int X_OUT = 2 * X_TILE;   // outputs a tile stages in LDS (mean multiplicity <= 2)

template <int WRITE>
union XShared {
    uint32_t out[X_OUT];
    struct {
        uint64_t off[X_TILE];   // run start per element (~0 past the tile end)
        uint32_t val[X_TILE];
    };
};
template <>
union XShared<0> {
    uint32_t out[1];
};

// WRITE = 1 emits vals[idx[i]] (idx != null) or vals[i]
template <int WRITE>
__global__ void __launch_bounds__(XB) expand_kernel(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                                                    uint64_t n, const uint32_t* __restrict__ counts,
                                                    uint64_t* __restrict__ tile_counts, uint32_t* __restrict__ out,
                                                    uint32_t* __restrict__ flags, const uint32_t* __restrict__ idx) {
    __shared__ XShared<WRITE> sx;
    __shared__ uint64_t s_red[XB / 64];
    const uint32_t tile = blockIdx.x;
    const uint64_t base = (uint64_t)tile * X_TILE;
    const uint32_t tn = (uint32_t)std::min<uint64_t>(X_TILE, n - base);
    uint32_t c[X_ITEMS];
    uint64_t tsum = 0;
    uint32_t mx = 0;
    const uint32_t e0 = threadIdx.x * X_ITEMS;
    uint32_t k[X_ITEMS];
    if (e0 + X_ITEMS <= tn) {   // 2 x 16-B loads of this thread's 8 keys
        uint4 a = *reinterpret_cast<const uint4*>(keys + base + e0);
        uint4 b = *reinterpret_cast<const uint4*>(keys + base + e0 + 4);
        k[0] = a.x; k[1] = a.y; k[2] = a.z; k[3] = a.w;
        k[4] = b.x; k[5] = b.y; k[6] = b.z; k[7] = b.w;
    } else {
#pragma unroll
        for (int j = 0; j < X_ITEMS; j++) k[j] = e0 + j < tn ? keys[base + e0 + j] : 0;
    }
#pragma unroll
    for (int j = 0; j < X_ITEMS; j++) {
        uint32_t e = e0 + j;
        c[j] = e < tn ? counts[k[j]] : 0;
        tsum += c[j];
        mx = c[j] > mx ? c[j] : mx;
    }
    if constexpr (!WRITE) {
        uint64_t s = wave_sum_u64(tsum);
        mx = wave_max_u32(mx);
        if (lane_id() == 0) {
            s_red[wave_id()] = s;
            // one flag word for the whole grid: skip the atomic once it is set (no hot-spot)
            if (mx > 1 && !(__hip_atomic_load(flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1u))
                atomicOr(flags, 1u);
        }
        __syncthreads();
        if (threadIdx.x == 0) tile_counts[tile] = s_red[0] + s_red[1] + s_red[2] + s_red[3];
        return;
    } else {   // (if constexpr: XShared<0> has no staging space)
    // this thread's 8 payloads, all loads in flight at once (idx is read in order, vals[idx] is
    // the random gather)
    uint32_t v[X_ITEMS];
    if (!idx && e0 + X_ITEMS <= tn) {   // payloads already in sorted order
        uint4 a = *reinterpret_cast<const uint4*>(vals + base + e0);
        uint4 b = *reinterpret_cast<const uint4*>(vals + base + e0 + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else if (idx && e0 + X_ITEMS <= tn) {
        uint4 a = *reinterpret_cast<const uint4*>(idx + base + e0);
        uint4 b = *reinterpret_cast<const uint4*>(idx + base + e0 + 4);
        uint32_t p[X_ITEMS] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int j = 0; j < X_ITEMS; j++) v[j] = c[j] ? vals[p[j]] : 0;
    } else {
#pragma unroll
        for (int j = 0; j < X_ITEMS; j++) {
            uint64_t e = base + e0 + j;
            v[j] = (e0 + j < tn && c[j]) ? vals[idx ? idx[e] : e] : 0;
        }
    }
    uint64_t inc = wave_incl_scan_u64(tsum);
    if (lane_id() == 63) s_red[wave_id()] = inc;
    __syncthreads();
    uint64_t add = 0;
    for (int w = 0; w < wave_id(); w++) add += s_red[w];
    uint64_t run = inc - tsum + add;
    const uint64_t btotal = s_red[0] + s_red[1] + s_red[2] + s_red[3];
    const uint64_t gofs = tile_counts[tile];
    if (btotal <= (uint64_t)X_OUT) {   // typical: the tile's output built in LDS, one coalesced run
#pragma unroll
        for (int j = 0; j < X_ITEMS; j++) {
            for (uint32_t q = 0; q < c[j]; q++) sx.out[sw32((uint32_t)run + q)] = v[j];
            run += c[j];
        }
        __syncthreads();
        for (uint32_t o = threadIdx.x; o < (uint32_t)btotal; o += XB) out[gofs + o] = sx.out[sw32(o)];
        return;
    }
    // heavy tile: run starts + payloads in LDS; output slot o finds its element by a fixed-step
    // binary search (last e with off[e] <= o), four slots interleaved per thread
#pragma unroll
    for (int j = 0; j < X_ITEMS; j++) {
        uint32_t e = e0 + j;
        sx.off[e] = e < tn ? run : ~0ull;
        sx.val[e] = v[j];
        run += c[j];
    }
    __syncthreads();
    for (uint64_t o0 = threadIdx.x; o0 < btotal; o0 += 4 * XB) {
        uint32_t a[4] = {0, 0, 0, 0};
#pragma unroll
        for (uint32_t step = X_TILE / 2; step; step >>= 1)
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (sx.off[a[q] + step] <= o0 + (uint64_t)q * XB) a[q] += step;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            uint64_t o = o0 + (uint64_t)q * XB;
            if (o < btotal) out[gofs + o] = sx.val[a[q]];
        }
    }
    }
}

// ---- general driver counts: exact distinct (pR, pS) pairs by sort + unique -------------------------
__global__ void __launch_bounds__(256) pack_pairs_kernel(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b,
                                                         uint64_t n, uint64_t* __restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = ((uint64_t)a[i] << 32) | b[i];
}

__global__ void __launch_bounds__(256) unique_count_kernel(const uint64_t* __restrict__ p, uint64_t n, int mode,
                                                           uint32_t* __restrict__ counts, uint64_t rows,
                                                           uint32_t* __restrict__ err) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (i > 0 && p[i] == p[i - 1]) return;
    uint32_t x = mode == 0 ? (uint32_t)(p[i] >> 32) : (uint32_t)p[i];
    if (x < rows) atomicAdd(&counts[x], 1u);
    else atomicOr(err, 1u);
}

}  // namespace qe

using namespace qe;

// =============================================================================================
// C ABI: device primitives
// =============================================================================================
namespace {

enum : uint32_t { PF_DISTINCT = 1u, PF_SORTED = 2u };

const char* op_ok(char op) { return (op == '=' || op == '<' || op == '>') ? nullptr : "Wrong operator"; }

// the listed heavy tiles' pairs at their exact offsets (tile_ofs: scanned tile counts)
void emit_deferred(qe_ctx* c, const qe_pairs* R, const qe_pairs* S, const uint64_t* win, const uint32_t* heavy,
                   uint32_t nheavy, const uint64_t* tile_ofs, uint32_t* outR, uint32_t* outS) {
    uint32_t* hp_lo = dalloc_t<uint32_t>(c, (uint64_t)nheavy * MJ_TILE);
    uint64_t* hp_off = dalloc_t<uint64_t>(c, (uint64_t)nheavy * MJ_TILE);
    uint64_t* hp_tot = dalloc_t<uint64_t>(c, nheavy);
    Timed t(c, "mj_heavy", 0);
    hipLaunchKernelGGL(mj_heavy_prep, dim3(nheavy), dim3(MJB), 0, c->stream, R->key, R->n, S->key, win, heavy, hp_lo,
                       hp_off, hp_tot);
    QE_HIP(hipGetLastError());
    std::vector<uint64_t> tot(nheavy);
    QE_HIP(hipMemcpyAsync(tot.data(), hp_tot, nheavy * 8ull, hipMemcpyDeviceToHost, c->stream));
    QE_HIP(hipStreamSynchronize(c->stream));
    std::vector<uint32_t> ck;
    std::vector<uint64_t> cs;
    double bytes = 0;
    for (uint32_t k = 0; k < nheavy; k++) {
        for (uint64_t o = 0; o < tot[k]; o += MJ_HEAVY_CHUNK) {
            ck.push_back(k);
            cs.push_back(o);
        }
        bytes += 12.0 * tot[k];
    }
    add_bytes(c, "mj_heavy", bytes);
    uint32_t* d_ck = dalloc_t<uint32_t>(c, ck.size());
    uint64_t* d_cs = dalloc_t<uint64_t>(c, cs.size());
    QE_HIP(hipMemcpyAsync(d_ck, ck.data(), ck.size() * 4, hipMemcpyHostToDevice, c->stream));
    QE_HIP(hipMemcpyAsync(d_cs, cs.data(), cs.size() * 8, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(mj_heavy_emit, dim3((unsigned)ck.size()), dim3(MJB), 0, c->stream, R->val, S->val, R->n, heavy,
                       hp_lo, hp_off, hp_tot, d_ck, d_cs, tile_ofs, outR, outS);
    QE_HIP(hipGetLastError());
    QE_HIP(hipStreamSynchronize(c->stream));   // the host vectors above are the copies' sources
    dfree(c, d_ck);
    dfree(c, d_cs);
    dfree(c, hp_lo);
    dfree(c, hp_off);
    dfree(c, hp_tot);
}

// merge join on sorted inputs; returns pair count and flags.  R->match receives each R row's
// number of S partners (the mode-0 driver counts come from it for free)
void merge_sorted(qe_ctx* c, qe_pairs* R, const qe_pairs* S, qe_list* outR, qe_list* outS, uint32_t* oflags) {
    const uint64_t nR = R->n, nS = S->n;
    outR->n = outS->n = 0;
    *oflags = 0;
    if (!R->match && nR) {
        R->match = dalloc_t<uint32_t>(c, nR);
        R->owns |= 4;
    }
    if (nR == 0 || nS == 0) {
        if (nR) QE_HIP(hipMemsetAsync(R->match, 0, nR * 4, c->stream));
        R->flags |= QE_PAIRS_MATCHED;
        outR->d = dalloc_t<uint32_t>(c, 1);
        outS->d = dalloc_t<uint32_t>(c, 1);
        outR->cap = outS->cap = 0;
        return;
    }
    const uint32_t nt = (uint32_t)((nR + MJ_TILE - 1) / MJ_TILE);
    uint64_t* win = dalloc_t<uint64_t>(c, 2 * (uint64_t)nt);
    uint64_t* tc = dalloc_t<uint64_t>(c, nt);
    uint32_t* d_flags = (uint32_t*)(c->d_scratch + 16);
    {
        Timed t(c, "mj_partition", 0);   // also clears the flags word and the heavy-tile count
        hipLaunchKernelGGL(mj_partition, dim3((nt + 3) / 4), dim3(256), 0, c->stream, R->key, nR, S->key, nS, nt,
                           win, c->d_scratch + 16, c->d_scratch + 19);
        QE_HIP(hipGetLastError());
    }
    // single pass with room for nR + nS pairs (every fan-out <= 1 + |S|/|R| case); the exact
    // two-pass form only when the join turns out larger
    const uint64_t cap = nR + nS;
    uint32_t* oR = dalloc_t<uint32_t>(c, cap);
    uint32_t* oS = dalloc_t<uint32_t>(c, cap);
    uint32_t* heavy = dalloc_t<uint32_t>(c, nt);
    {
        LBSlot s = lb_acquire(c, nt);
        Timed t(c, "mj_fused", 12.0 * nR + 12.0 * nS + 4.0 * nR);   // + 8 B per pair, added below
        // 32-bit tile offsets when R's keys vary only below bit 32 (known from the producer's
        // OR / AND): every key a tile compares then differs from its first R key by < 2^32
        const bool key32 = (R->flags & QE_PAIRS_BITS) && ((R->kor & ~R->kand) >> 32) == 0;
        if (key32 && nS <= nR)
            hipLaunchKernelGGL(mj_fused<MJShared32s>, dim3(nt), dim3(MJB), 0, c->stream, R->key, R->val, nR, S->key,
                               S->val, nS, win, tc, R->match, oR, oS, cap, d_flags, s.status, s.ticket, s.epoch, nt,
                               c->d_scratch + 17, heavy, (uint32_t*)(c->d_scratch + 19));
        else if (key32)
            hipLaunchKernelGGL(mj_fused<MJShared32>, dim3(nt), dim3(MJB), 0, c->stream, R->key, R->val, nR, S->key,
                               S->val, nS, win, tc, R->match, oR, oS, cap, d_flags, s.status, s.ticket, s.epoch, nt,
                               c->d_scratch + 17, heavy, (uint32_t*)(c->d_scratch + 19));
        else
            hipLaunchKernelGGL(mj_fused<MJShared64>, dim3(nt), dim3(MJB), 0, c->stream, R->key, R->val, nR, S->key,
                               S->val, nS, win, tc, R->match, oR, oS, cap, d_flags, s.status, s.ticket, s.epoch, nt,
                               c->d_scratch + 17, heavy, (uint32_t*)(c->d_scratch + 19));
        QE_HIP(hipGetLastError());
    }
    R->flags |= QE_PAIRS_MATCHED;
    uint64_t h[4];
    read_words(c, c->d_scratch + 16, h, 4);
    uint64_t P = h[1];
    *oflags = (uint32_t)h[0];
    const uint32_t nheavy = (uint32_t)h[3];
    const bool exact = P <= cap && !(h[0] & MJF_OVF);
    if (exact) add_bytes(c, "mj_fused", 8.0 * P);
    if (!exact || nheavy) {   // exact u64 offsets (and total) from the per-tile counts
        hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, c->stream, tc, (uint64_t)nt, c->d_scratch + 18);
        QE_HIP(hipGetLastError());
        P = read_u64(c, c->d_scratch + 18);
    }
    outR->n = outS->n = P;
    if (P > c->mat_limit) {   // R->match stays valid: the caller may take the aggregate form
        dfree(c, oR);
        dfree(c, oS);
        dfree(c, win);
        dfree(c, tc);
        dfree(c, heavy);
        outR->d = outS->d = nullptr;
        outR->cap = outS->cap = 0;
        char msg[160];
        snprintf(msg, sizeof msg, "merge join of %llu pairs exceeds the materialisation limit %llu",
                 (unsigned long long)P, (unsigned long long)c->mat_limit);
        throw Error(QE_ETOOBIG, msg);
    }
    if (exact) {
        outR->d = oR;
        outS->d = oS;
        outR->cap = outS->cap = cap;
    } else {
        dfree(c, oR);
        dfree(c, oS);
        outR->d = dalloc_t<uint32_t>(c, P);
        outS->d = dalloc_t<uint32_t>(c, P);
        outR->cap = outS->cap = P;
        Timed t(c, "mj_write", 12.0 * nR + 12.0 * nS + 8.0 * P);
        hipLaunchKernelGGL(mj_tile<1>, dim3(nt), dim3(MJB), 0, c->stream, R->key, R->val, nR, S->key, S->val, nS, win,
                           tc, outR->d, outS->d, nullptr, nullptr, nullptr);
        QE_HIP(hipGetLastError());
    }
    if (nheavy) emit_deferred(c, R, S, win, heavy, nheavy, tc, outR->d, outS->d);
    dfree(c, heavy);
    dfree(c, win);
    dfree(c, tc);
}

// count-only merge pass: A->match[i] = number of B rows with A's key (both sorted); returns
// the exact pair count.  The fused kernel runs with no output room, so it stores nothing.
uint64_t merge_count_side(qe_ctx* c, qe_pairs* A, const qe_pairs* B) {
    const uint64_t nA = A->n, nB = B->n;
    if (!A->match && nA) {
        A->match = dalloc_t<uint32_t>(c, nA);
        A->owns |= 4;
    }
    if (nA == 0) return 0;
    if (nB == 0) {
        QE_HIP(hipMemsetAsync(A->match, 0, nA * 4, c->stream));
        return 0;
    }
    const uint32_t nt = (uint32_t)((nA + MJ_TILE - 1) / MJ_TILE);
    uint64_t* win = dalloc_t<uint64_t>(c, 2 * (uint64_t)nt);
    uint64_t* tc = dalloc_t<uint64_t>(c, nt);
    uint32_t* sink = dalloc_t<uint32_t>(c, 1);
    uint32_t* d_flags = (uint32_t*)(c->d_scratch + 16);
    QE_HIP(hipMemsetAsync(d_flags, 0, 4, c->stream));
    {
        Timed t(c, "mj_count", 12.0 * nA + 12.0 * nB + 4.0 * nA);
        hipLaunchKernelGGL(mj_partition, dim3((nt + 3) / 4), dim3(256), 0, c->stream, A->key, nA, B->key, nB, nt,
                           win, nullptr, nullptr);
        QE_HIP(hipGetLastError());
        LBSlot s = lb_acquire(c, nt);
        const bool key32 = (A->flags & QE_PAIRS_BITS) && ((A->kor & ~A->kand) >> 32) == 0;
        if (key32)
            hipLaunchKernelGGL(mj_fused<MJShared32>, dim3(nt), dim3(MJB), 0, c->stream, A->key, A->val, nA, B->key,
                               B->val, nB, win, tc, A->match, sink, sink, 0ull, d_flags, s.status, s.ticket, s.epoch,
                               nt, c->d_scratch + 17, nullptr, nullptr);
        else
            hipLaunchKernelGGL(mj_fused<MJShared64>, dim3(nt), dim3(MJB), 0, c->stream, A->key, A->val, nA, B->key,
                               B->val, nB, win, tc, A->match, sink, sink, 0ull, d_flags, s.status, s.ticket, s.epoch,
                               nt, c->d_scratch + 17, nullptr, nullptr);
        QE_HIP(hipGetLastError());
        hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, c->stream, tc, (uint64_t)nt, c->d_scratch + 18);
        QE_HIP(hipGetLastError());
    }
    const uint64_t P = read_u64(c, c->d_scratch + 18);
    dfree(c, win);
    dfree(c, tc);
    dfree(c, sink);
    return P;
}

static void prefix_max(qe_ctx* c, const uint64_t* x, uint64_t n, uint64_t* out) {
    const uint64_t nb = (n + PM_CHUNK - 1) / PM_CHUNK;
    uint64_t* bmax = dalloc_t<uint64_t>(c, std::max<uint64_t>(nb, 1));
    hipLaunchKernelGGL(pmax_reduce_kernel, dim3((unsigned)nb), dim3(PM_B), 0, c->stream, x, n, bmax);
    QE_HIP(hipGetLastError());
    hipLaunchKernelGGL(pmax_top_kernel, dim3(1), dim3(1024), 0, c->stream, bmax, nb);
    QE_HIP(hipGetLastError());
    hipLaunchKernelGGL(pmax_apply_kernel, dim3((unsigned)nb), dim3(PM_B), 0, c->stream, x, n, bmax, out);
    QE_HIP(hipGetLastError());
    dfree(c, bmax);
}

void merge_sequential(qe_ctx* c, const qe_pairs* R, const qe_pairs* S, qe_list* outR, qe_list* outS) {
    const uint64_t nR = R->n, nS = S->n;
    outR->n = outS->n = outR->cap = outS->cap = 0;
    if (nR == 0 || nS == 0) {
        outR->d = dalloc_t<uint32_t>(c, 1);
        outS->d = dalloc_t<uint32_t>(c, 1);
        return;
    }
    uint64_t* pmR = dalloc_t<uint64_t>(c, nR);
    uint64_t* pmS = dalloc_t<uint64_t>(c, nS);
    uint32_t* rec = dalloc_t<uint32_t>(c, nS);
    uint32_t* cand = dalloc_t<uint32_t>(c, nR);
    uint64_t maxS, nrec, nc;
    {
        Timed t(c, "seq_merge", 16.0 * (nR + nS));
        prefix_max(c, R->key, nR, pmR);
        prefix_max(c, S->key, nS, pmS);
    }
    maxS = read_u64(c, pmS + nS - 1);
    nrec = compact_prefix_max_hits(c, S->key, pmS, nS, ~0ull, rec);     // S's record positions
    nc = compact_prefix_max_hits(c, R->key, pmR, nR, maxS, cand);       // rows that can emit
    uint64_t P = 0;
    uint64_t* cnt = nullptr;
    uint32_t* e0s = nullptr;
    if (nc) {
        cnt = dalloc_t<uint64_t>(c, nc);
        e0s = dalloc_t<uint32_t>(c, nc);
        Timed t(c, "seq_merge", 0);
        hipLaunchKernelGGL(seqm_count_kernel, dim3(grid_for(nc, 256)), dim3(256), 0, c->stream, R->key, cand, nc,
                           S->key, rec, nrec, cnt, e0s);
        QE_HIP(hipGetLastError());
        scan_u64(c, cnt, nc, c->d_scratch + 20);
        P = read_u64(c, c->d_scratch + 20);
    }
    if (getenv("QE_SEQ_DEBUG"))
        fprintf(stderr, "[seq_merge] nR %lu nS %lu records %lu candidates %lu pairs %lu\n", (unsigned long)nR,
                (unsigned long)nS, (unsigned long)nrec, (unsigned long)nc, (unsigned long)P);
    outR->d = dalloc_t<uint32_t>(c, std::max<uint64_t>(P, 1));
    outS->d = dalloc_t<uint32_t>(c, std::max<uint64_t>(P, 1));
    outR->n = outS->n = outR->cap = outS->cap = P;
    if (P) {
        Timed t(c, "seq_merge", 8.0 * P);
        hipLaunchKernelGGL(seqm_write_kernel, dim3(grid_for(nc, 256)), dim3(256), 0, c->stream, R->val, cand, nc,
                           S->val, rec, cnt, e0s, P, outR->d, outS->d);
        QE_HIP(hipGetLastError());
    }
    if (cnt) dfree(c, cnt);
    if (e0s) dfree(c, e0s);
    dfree(c, pmR);
    dfree(c, pmS);
    dfree(c, rec);
    dfree(c, cand);
}

bool pairs_sorted(qe_ctx* c, const qe_pairs* p) {
    if (p->flags & PF_SORTED) return true;
    if (p->n < 2) return true;
    uint32_t* bad = (uint32_t*)(c->d_scratch + 24);
    QE_HIP(hipMemsetAsync(bad, 0, 4, c->stream));
    {
        Timed t(c, "is_sorted", 8.0 * p->n);
        hipLaunchKernelGGL(is_sorted_kernel, dim3(grid_for(p->n, 256 * 8, 4096)), dim3(256), 0, c->stream, p->key,
                           p->n, bad);
        QE_HIP(hipGetLastError());
    }
    return (read_u64(c, c->d_scratch + 24) & 0xFFFFFFFFull) == 0;
}

// dense driver counts by exact sort + unique of the packed pairs (any input order)
uint32_t* driver_counts_general(qe_ctx* c, const qe_list* outR, const qe_list* outS, int mode, uint64_t rows) {
    uint32_t* cnt = dalloc_t<uint32_t>(c, std::max<uint64_t>(rows, 1));
    QE_HIP(hipMemsetAsync(cnt, 0, std::max<uint64_t>(rows, 1) * 4, c->stream));
    const uint64_t n = outR->n;
    if (n == 0) return cnt;
    uint64_t* packed = dalloc_t<uint64_t>(c, n);
    {
        Timed t(c, "dedup_pack", 16.0 * n);
        hipLaunchKernelGGL(pack_pairs_kernel, dim3(grid_for(n, 256)), dim3(256), 0, c->stream, outR->d, outS->d, n,
                           packed);
        QE_HIP(hipGetLastError());
    }
    SortOut so = radix_sort_u64(c, packed, nullptr, n, false);
    const uint64_t* sp = (const uint64_t*)so.keys;
    uint32_t* err = (uint32_t*)(c->d_scratch + 26);
    QE_HIP(hipMemsetAsync(err, 0, 4, c->stream));
    {
        Timed t(c, "dedup_count", 8.0 * n);
        hipLaunchKernelGGL(unique_count_kernel, dim3(grid_for(n, 256)), dim3(256), 0, c->stream, sp, n, mode, cnt, rows,
                           err);
        QE_HIP(hipGetLastError());
    }
    if (so.keys_new) dfree(c, so.keys);
    dfree(c, packed);
    if (read_u64(c, c->d_scratch + 26) & 0xFFFFFFFFull) throw Error(QE_EINVAL, "driver rowid out of range");
    return cnt;
}

// fast path: sorted merge inputs whose partner side is distinct -> the count of a rowid is the
// length of its partner's equal-key run (every pair of that run is distinct)
uint32_t* driver_counts_sorted(qe_ctx* c, const qe_pairs* A, const qe_pairs* B, uint64_t rows) {
    uint32_t* cnt = dalloc_t<uint32_t>(c, std::max<uint64_t>(rows, 1));
    QE_HIP(hipMemsetAsync(cnt, 0, std::max<uint64_t>(rows, 1) * 4, c->stream));
    if (A->n == 0 || B->n == 0) return cnt;
    if (A->match) {   // A was the merge's R side: its per-row match counts are the answer
        Timed t(c, "driver_scatter", 12.0 * A->n);
        hipLaunchKernelGGL(scatter_match_kernel, dim3(grid_for(A->n, 256)), dim3(256), 0, c->stream, A->val, A->match,
                           A->n, cnt);
        QE_HIP(hipGetLastError());
        return cnt;
    }
    const uint32_t nt = (uint32_t)((A->n + MJ_TILE - 1) / MJ_TILE);
    uint64_t* win = dalloc_t<uint64_t>(c, 2 * (uint64_t)nt);
    uint64_t* tc = dalloc_t<uint64_t>(c, nt);
    uint32_t* d_flags = (uint32_t*)(c->d_scratch + 28);
    {
        Timed t(c, "mj_annotate", 12.0 * A->n + 8.0 * B->n);
        hipLaunchKernelGGL(mj_partition, dim3((nt + 3) / 4), dim3(256), 0, c->stream, A->key, A->n, B->key, B->n,
                           nt, win, nullptr, nullptr);
        QE_HIP(hipGetLastError());
        hipLaunchKernelGGL(mj_tile<0>, dim3(nt), dim3(MJB), 0, c->stream, A->key, A->val, A->n, B->key, B->val, B->n,
                           win, tc, nullptr, nullptr, d_flags, cnt, nullptr);
        QE_HIP(hipGetLastError());
    }
    dfree(c, win);
    dfree(c, tc);
    return cnt;
}

}  // namespace

extern "C" {

int qe_filter_scan(qe_ctx* c, qe_col col, char op, uint64_t v, qe_list* out) {
    QE_API_BEGIN(c)
    if (op_ok(op)) throw Error(QE_EINVAL, op_ok(op));
    out->d = dalloc_t<uint32_t>(c, std::max<uint64_t>(col.n, 1));
    out->cap = col.n;
    out->n = filter_scan(c, col.d, col.n, op, v, out->d);
    out->flags = QE_LIST_DISTINCT;
    return 0;
    QE_API_END(c)
}

int qe_filter_refine(qe_ctx* c, qe_col col, char op, uint64_t v, qe_list* inout) {
    QE_API_BEGIN(c)
    if (op_ok(op)) throw Error(QE_EINVAL, op_ok(op));
    if (inout->n == 0) return 0;
    uint32_t* o = dalloc_t<uint32_t>(c, inout->n);
    uint64_t m = filter_refine(c, col.d, inout->d, inout->n, op, v, o);
    dfree(c, inout->d);
    inout->d = o;
    inout->cap = inout->n;
    inout->n = m;
    return 0;
    QE_API_END(c)
}

int qe_gather_pairs(qe_ctx* c, qe_col col, const qe_list* rows, qe_pairs* out) {
    QE_API_BEGIN(c)
    out->match = nullptr;
    if (!rows) {
        out->key = const_cast<uint64_t*>(col.d);
        out->val = nullptr;
        out->n = col.n;
        out->flags = PF_DISTINCT;
        out->owns = 0;
        // a base column: its OR / AND were computed when the relation was loaded
        for (auto& r : c->rels)
            for (size_t j = 0; j < r.cols.size(); j++)
                if (r.cols[j] == col.d && r.rows == col.n && j < r.kor.size()) {
                    out->kor = r.kor[j];
                    out->kand = r.kand[j];
                    out->flags |= QE_PAIRS_BITS;
                }
        return 0;
    }
    const uint64_t n = rows->n;
    out->key = dalloc_t<uint64_t>(c, std::max<uint64_t>(n, 1));
    out->val = rows->d;   // borrowed: the caller keeps the list alive while the pairs live
    out->n = n;
    out->flags = (rows->flags & QE_LIST_DISTINCT) ? PF_DISTINCT : 0;
    out->owns = 1;
    // a loaded relation's column: its load-time OR / AND bound the gathered keys too, so the
    // gather needs no reduction and no host round trip (the sort plans on the column's bits)
    for (auto& r : c->rels)
        for (size_t j = 0; j < r.cols.size(); j++)
            if (r.cols[j] == col.d && r.rows == col.n && j < r.kor.size() && !getenv("QE_GATHER_EXACT_BITS")) {
                if (n && !(getenv("QE_GATHER_HIST") && getenv("QE_GATHER_HIST")[0] == '0') &&
                    gather_with_hist(c, col.d, rows->d, n, r.kor[j], r.kand[j], out->key, col.n)) {
                    // gathered together with the histogram its sort will read
                } else if (n) {
                    Timed t(c, "gather_keys", 12.0 * n + 8.0 * n);
                    hipLaunchKernelGGL(gather_keys_kernel<false>, dim3(grid_for((n + 3) / 4, 256, 4096)), dim3(256), 0,
                                       c->stream, col.d, rows->d, n, out->key, (unsigned long long*)nullptr);
                    QE_HIP(hipGetLastError());
                }
                out->kor = r.kor[j];
                out->kand = r.kand[j];
                out->flags |= QE_PAIRS_BITS;
                return 0;
            }
    uint64_t* d_bits = c->d_scratch + 44;
    hipLaunchKernelGGL(set2_kernel, dim3(1), dim3(64), 0, c->stream, d_bits, 0ull, ~0ull);
    QE_HIP(hipGetLastError());
    if (n) {
        Timed t(c, "gather_keys", 12.0 * n + 8.0 * n);
        hipLaunchKernelGGL(gather_keys_kernel<true>, dim3(grid_for((n + 3) / 4, 256, 4096)), dim3(256), 0, c->stream,
                           col.d, rows->d, n, out->key, (unsigned long long*)d_bits);
        QE_HIP(hipGetLastError());
    }
    uint64_t kb[2];
    read_words(c, d_bits, kb, 2);
    out->kor = kb[0];
    out->kand = kb[1];
    out->flags |= QE_PAIRS_BITS;
    return 0;
    QE_API_END(c)
}

// qe_sort_pairs' body; defer: a large two-level sort may stop before its per-bucket step
// (qe_join_pairs hands such sides to bucket_join)
static void sort_pairs_raw(qe_ctx* c, qe_pairs* p, bool defer) {
    if (p->flags & PF_SORTED) return;
    p->flags &= ~QE_PAIRS_MATCHED;
    uint64_t bits[2] = {p->kor, p->kand};
    SortOut so = radix_sort_u64(c, p->key, p->val, p->n, true, (p->flags & QE_PAIRS_BITS) ? bits : nullptr, defer);
    if (so.keys_new) {
        pairs_drop_deferred(c, p, !(p->owns & 1));   // a gathered histogram the sort did not take dies with the keys
        if (p->owns & 1) dfree(c, p->key);
        p->key = (uint64_t*)so.keys;
        p->owns |= 1;
    }
    if (so.vals_new) {
        if (p->owns & 2) dfree(c, p->val);
        p->val = so.vals;
        p->owns |= 2;
    }
    p->flags |= PF_SORTED;
}

// ---- a batch's shared sorts of whole base columns (qe_sort_cache) -----------------------------
// Within one batch many queries join the same base relation on the same column (the C4 batch:
// 1292 base join sides over 46 distinct columns).  The sort of a whole column -- (key, row) pairs,
// rows implicit -- depends on the column alone, so the first lane that needs it sorts it on its
// own stream and publishes the result with an event; every later join of the batch on that column
// waits on the event and reads the same buffers.  A deferred two-level sort is shared as its
// bucket-partitioned words (each reader gets its own, unfilled, key / row buffers for a possible
// completion: the words are only read); a complete sort as its key and row arrays, lent to the
// pairs (not owned).  Sorts that carry payloads or pack values are query-specific and never cached.
// Scope: one qe_sort_cache(ctx, 1) .. qe_sort_cache(ctx, 0) bracket (a batch): nothing outlives it.
namespace qe {
struct SortCacheEntry {
    bool ready = false, deferred = false;
    DeferredSort d{};                       // deferred: the shared words / bstart / d_max
    uint64_t* keys = nullptr;               // complete: the sorted keys and rows
    uint32_t* vals = nullptr;
    bool own_keys = false, own_vals = false;
    hipEvent_t ev = nullptr;                // recorded on the builder's stream after the sort
    qe_ctx* owner = nullptr;                // the builder (its allocator frees the buffers)
};
struct SortCache {
    std::mutex mu;
    std::condition_variable cv;
    std::map<std::tuple<const void*, uint64_t, int, uint64_t, uint64_t>, SortCacheEntry> m;   // + the bounds
    uint64_t hits = 0, builds = 0;
};
}  // namespace qe

static bool is_base_column(const qe_ctx* c, const void* key, uint64_t n) {
    for (const auto& r : c->rels)
        if (r.rows == n)
            for (const uint64_t* col : r.cols)
                if (col == key) return true;
    return false;
}

// true: p is sorted from (or into) the batch's cache
static bool sort_cached(qe_ctx* c, qe_pairs* p, bool defer) {
    SortCache* sc = c->scache;
    if (!sc || p->val || (p->owns & 3) || !p->key || p->n < 2) return false;
    if (c->carry_xa || c->carry_xb || c->carry_x32 || c->carry_c64 || c->sort_v64) return false;
    if (!is_base_column(c, p->key, p->n)) return false;
    const int mode = defer ? (c->sort_keys_only ? 2 : 1) : 0;
    const auto key = std::make_tuple((const void*)p->key, p->n, mode, p->kor, p->kand);
    std::unique_lock<std::mutex> lk(sc->mu);
    auto it = sc->m.find(key);
    if (it == sc->m.end()) {   // this lane builds it
        SortCacheEntry& slot = sc->m[key];
        slot.owner = c;
        lk.unlock();
        // everything that can throw before the entry is published sits in this try: a slot left
        // unready would block every other lane that needs the column forever
        hipEvent_t ev = nullptr;
        try {
            QE_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            sort_pairs_raw(c, p, defer);
            QE_HIP(hipEventRecord(ev, c->stream));
        } catch (...) {
            if (ev) (void)hipEventDestroy(ev);
            lk.lock();
            sc->m.erase(key);
            sc->cv.notify_all();
            throw;
        }
        SortCacheEntry e;
        e.owner = c;
        e.ev = ev;
        auto dit = c->deferred.find(p->key);
        if (dit != c->deferred.end()) {
            dit->second.shared = true;   // this pairs' own key / row buffers stay its own
            e.deferred = true;
            e.d = dit->second;
            c->pinned.insert({e.d.words, e.d.bstart, e.d.d_max});   // freed only when the batch ends
        } else {
            e.keys = p->key;
            e.vals = p->val;
            e.own_keys = (p->owns & 1) != 0;
            e.own_vals = (p->owns & 2) != 0;
            p->owns &= ~3u;                  // lent by the cache from now on
            c->pinned.insert({(const void*)e.keys, (const void*)e.vals});
        }
        e.ready = true;
        lk.lock();
        sc->m[key] = e;
        sc->builds++;
        sc->cv.notify_all();
        return true;
    }
    sc->cv.wait(lk, [&] {
        auto j = sc->m.find(key);
        return j == sc->m.end() || j->second.ready;
    });
    it = sc->m.find(key);
    if (it == sc->m.end()) return false;   // its build failed: sort privately
    const SortCacheEntry e = it->second;
    sc->hits++;
    lk.unlock();
    if (e.owner != c) QE_HIP(hipStreamWaitEvent(c->stream, e.ev, 0));
    c->sort_keys_only = false;   // (what the sort would have consumed)
    p->flags &= ~QE_PAIRS_MATCHED;
    if (e.deferred) {
        DeferredSort d = e.d;
        d.kout = dalloc_t<uint64_t>(c, p->n);   // filled only if a reader completes the sort
        d.vout = dalloc_t<uint32_t>(c, p->n);
        d.shared = true;
        c->deferred[d.kout] = d;
        p->key = d.kout;
        p->val = d.vout;
        p->owns |= 3u;
    } else {
        p->key = e.keys;
        p->val = e.vals;
        p->owns &= ~3u;
    }
    p->flags |= PF_SORTED;
    return true;
}

// the two sides of a join sorted concurrently (SideFork): both large enough for the lookback-free
// two-level sort, outside a batch's shared sorts (the lanes are the concurrency there)
static bool fork_sides(const qe_ctx* c, const qe_pairs* R, const qe_pairs* S) {
    return !c->scache && R->n >= (1u << 22) && S->n >= (1u << 22) && !(R->flags & PF_SORTED) &&
           !(S->flags & PF_SORTED);
}

static void sort_pairs(qe_ctx* c, qe_pairs* p, bool defer) {
    if (p->flags & PF_SORTED) return;
    if (sort_cached(c, p, defer)) return;
    sort_pairs_raw(c, p, defer);
}

int qe_sort_cache(qe_ctx* c, int on) {
    if (!c) return QE_EINVAL;
    QE_API_BEGIN(c)
    if (on) {
        const char* env = getenv("QE_SORT_CACHE");   // (read per batch: the bench A/Bs it)
        if (c->scache || (env && env[0] == '0')) return 0;
        c->scache = new SortCache;
        for (qe_ctx* w : c->workers) w->scache = c->scache;
        return 0;
    }
    SortCache* sc = c->scache;
    if (!sc) return 0;
    c->scache = nullptr;
    for (qe_ctx* w : c->workers)
        if (w->scache == sc) w->scache = nullptr;
    sync(c);   // every reader of the shared buffers has finished
    for (qe_ctx* w : c->workers) sync(w);
    for (auto& kv : sc->m) {
        SortCacheEntry& e = kv.second;
        qe_ctx* o = e.owner;
        o->pinned.clear();
        if (e.deferred) {
            dfree(o, e.d.words);
            dfree(o, e.d.bstart);
            dfree(o, e.d.d_max);
        } else {
            if (e.own_keys) dfree(o, e.keys);
            if (e.own_vals) dfree(o, e.vals);
        }
        if (e.ev) QE_HIP(hipEventDestroy(e.ev));
    }
    c->scache_hits += sc->hits;
    c->scache_builds += sc->builds;
    delete sc;
    // a lane that tried to return a shared sort's buffer to its allocator (dfree records it, it
    // cannot throw from the destructors it runs in): the batch fails loudly here
    for (qe_ctx* x : c->workers)
        if (!x->late_err.empty()) {
            const std::string m = x->late_err;
            x->late_err.clear();
            throw Error(QE_EINVAL, m);
        }
    if (!c->late_err.empty()) {
        const std::string m = c->late_err;
        c->late_err.clear();
        throw Error(QE_EINVAL, m);
    }
    return 0;
    QE_API_END(c)
}

int qe_sort_cache_stats(qe_ctx* c, uint64_t* hits, uint64_t* builds) {
    if (!c) return QE_EINVAL;
    if (hits) *hits = c->scache_hits;
    if (builds) *builds = c->scache_builds;
    return 0;
}

int qe_join_pairs(qe_ctx* c, qe_pairs* R, qe_pairs* S, qe_list* outR, qe_list* outS) {
    QE_API_BEGIN(c)
    // one bucket geometry for both sides (QE_JOIN_UNIFY=0 keeps each side's own bounds): C4 2504 ->
    // 2529-2533 queries/s same box, 155 bucket joins per batch instead of 104 (profiles/r03_c4_knobs_ab.log)
    static const bool unify = !(getenv("QE_JOIN_UNIFY") && getenv("QE_JOIN_UNIFY")[0] == '0');
    if (unify) unify_geometry(R, S);
    {
        SideFork fk(c, fork_sides(c, R, S));
        fk.enter();
        sort_pairs(c, R, true);
        fk.leave();
        sort_pairs(c, S, true);
    }
    if (bucket_join(c, R, S, outR, outS)) return 0;
    pairs_need_keys(c, R);
    pairs_need_keys(c, S);
    uint32_t fl = MJF_R_FANOUT | MJF_S_DUP;
    merge_sorted(c, R, S, outR, outS, &fl);
    outR->flags = outS->flags = 0;
    return 0;
    QE_API_END(c)
}

}  // extern "C"

namespace qe {
bool join_pairs_carry(qe_ctx* c, qe_pairs* R, qe_pairs* S, const uint32_t* xa, const uint32_t* xb, qe_list* outR,
                      qe_list* outS, qe_list* outX0, qe_list* outX1, const uint32_t* rx32, const uint64_t* rc64,
                      qe_list* outRX, const uint64_t* rv64) {
    const bool rpay = rx32 || rc64;
    if ((!xa && !rpay) || !carry_eligible(R, S, rpay || rv64)) return false;
    if (rv64 && R->val) return false;
    const qe_pairs R0 = *R, S0 = *S;   // views of the caller's arrays (nothing owned)
    if ((R0.owns | S0.owns) & 7) return false;
    c->carry_x32 = rx32;
    c->carry_c64 = rc64;
    c->sort_v64 = rv64;
    SideFork fk(c, fork_sides(c, R, S));   // R's sort on the side stream, S's beside it
    fk.enter();
    sort_pairs(c, R, true);
    fk.leave();
    c->carry_x32 = nullptr;   // (consumed by R's sort; cleared in any case)
    c->carry_c64 = nullptr;
    c->sort_v64 = nullptr;
    if (rv64) {   // the values must have gone into R's words (its sort's deferred lookback-free form)
        auto it = c->deferred.find(R->key);
        if (it == c->deferred.end() || it->second.v64 != rv64) {
            qe_pairs_free(c, R);
            *R = R0;
            return false;
        }
    }
    c->carry_xa = xb ? xa : nullptr;   // two columns: one 64-bit payload; one: 32-bit
    c->carry_xb = xb;
    c->carry_x32 = xb ? nullptr : xa;
    sort_pairs(c, S, true);
    c->carry_xa = c->carry_xb = c->carry_x32 = nullptr;   // (consumed by S's sort; cleared in any case)
    fk.join();
    if (bucket_join(c, R, S, outR, outS, xa ? outX0 : nullptr, xa && xb ? outX1 : nullptr, rpay ? outRX : nullptr))
        return true;
    // a bucket beyond LDS: drop both deferred sorts, give the caller its inputs back
    qe_pairs_free(c, R);
    qe_pairs_free(c, S);
    *R = R0;
    *S = S0;
    return false;
}

bool join_pairs_sums(qe_ctx* c, qe_pairs* R, qe_pairs* S, const uint32_t* xa, const uint32_t* xb, const HjSums& sc,
                     uint64_t* pairs, uint64_t* sums) {
    if (!carry_eligible(R, S)) return false;
    const qe_pairs R0 = *R, S0 = *S;
    if ((R0.owns | S0.owns) & 7) return false;
    {
        SideFork fk(c, fork_sides(c, R, S));   // R's sort on the side stream, S's beside it
        c->sort_keys_only = !R->val;   // R's keys are only counted: its rows never travel
        fk.enter();
        sort_pairs(c, R, true);
        fk.leave();
        c->sort_keys_only = false;
        c->carry_xa = xb ? xa : nullptr;   // (null: no payload; one column: 32-bit)
        c->carry_xb = xb;
        c->carry_x32 = xb ? nullptr : xa;
        sort_pairs(c, S, true);
        c->carry_xa = c->carry_xb = c->carry_x32 = nullptr;
    }
    if (bucket_join_sums(c, R, S, sc, pairs, sums)) return true;
    qe_pairs_free(c, R);
    qe_pairs_free(c, S);
    *R = R0;
    *S = S0;
    return false;
}
}  // namespace qe

extern "C" {

int qe_sort_pairs(qe_ctx* c, qe_pairs* p) {
    QE_API_BEGIN(c)
    if (p->flags & PF_SORTED) return 0;
    p->flags &= ~QE_PAIRS_MATCHED;
    uint64_t bits[2] = {p->kor, p->kand};
    SortOut so = radix_sort_u64(c, p->key, p->val, p->n, true, (p->flags & QE_PAIRS_BITS) ? bits : nullptr, false);
    if (so.keys_new) {
        pairs_drop_deferred(c, p, !(p->owns & 1));   // a gathered histogram the sort did not take dies with the keys
        if (p->owns & 1) dfree(c, p->key);
        p->key = (uint64_t*)so.keys;
        p->owns |= 1;
    }
    if (so.vals_new) {
        if (p->owns & 2) dfree(c, p->val);
        p->val = so.vals;
        p->owns |= 2;
    }
    p->flags |= PF_SORTED;
    return 0;
    QE_API_END(c)
}

int qe_is_sorted(qe_ctx* c, const qe_pairs* p, int* sorted) {
    QE_API_BEGIN(c)
    pairs_need_keys(c, p);
    *sorted = pairs_sorted(c, p) ? 1 : 0;
    return 0;
    QE_API_END(c)
}

int qe_merge_join(qe_ctx* c, qe_pairs* R, const qe_pairs* S, qe_list* outR, qe_list* outS) {
    QE_API_BEGIN(c)
    const bool sorted = pairs_sorted(c, R) && pairs_sorted(c, S);
    uint32_t fl = MJF_R_FANOUT | MJF_S_DUP;
    pairs_need_keys(c, R);
    pairs_need_keys(c, S);
    if (sorted) merge_sorted(c, R, S, outR, outS, &fl);
    else merge_sequential(c, R, S, outR, outS);
    outR->flags = ((R->flags & PF_DISTINCT) && sorted && !(fl & MJF_R_FANOUT)) ? QE_LIST_DISTINCT : 0;
    outS->flags = ((S->flags & PF_DISTINCT) && sorted && !(fl & MJF_S_DUP)) ? QE_LIST_DISTINCT : 0;
    return 0;
    QE_API_END(c)
}

int qe_merge_join_counts(qe_ctx* c, qe_pairs* R, qe_pairs* S, uint64_t* pairs) {
    QE_API_BEGIN(c)
    if (!pairs_sorted(c, R) || !pairs_sorted(c, S)) throw Error(QE_EINVAL, "qe_merge_join_counts needs sorted inputs");
    pairs_need_keys(c, R);
    pairs_need_keys(c, S);
    const bool r_done = (R->flags & QE_PAIRS_MATCHED) && (R->match || R->n == 0);
    const uint64_t Q = merge_count_side(c, S, R);
    if (!r_done) {
        const uint64_t P = merge_count_side(c, R, S);
        if (P != Q) throw Error(QE_EINVAL, "internal: the two count passes disagree");
    }
    R->flags |= QE_PAIRS_MATCHED;
    S->flags |= QE_PAIRS_MATCHED;
    *pairs = Q;
    return 0;
    QE_API_END(c)
}

int qe_checksum_weighted(qe_ctx* c, qe_col col, const qe_pairs* p, uint64_t* sum) {
    QE_API_BEGIN(c)
    if (p->n && !p->match) throw Error(QE_EINVAL, "qe_checksum_weighted needs match counts");
    pairs_need_vals(c, p);
    unsigned long long* d = (unsigned long long*)(c->d_scratch + 40);
    hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(64), 0, c->stream, (uint64_t*)d, 1);
    QE_HIP(hipGetLastError());
    if (p->n) {
        Timed t(c, "checksum_weighted", (p->val ? 8.0 : 4.0) * p->n);
        hipLaunchKernelGGL(checksum_weighted_kernel, dim3(grid_for(p->n, 256 * 16, 8192)), dim3(256), 0, c->stream,
                           col.d, p->val, p->match, p->n, d);
        QE_HIP(hipGetLastError());
    }
    *sum = read_u64(c, (const uint64_t*)d);
    return 0;
    QE_API_END(c)
}

int qe_set_materialize_limit(qe_ctx* c, uint64_t pairs) {
    QE_API_BEGIN(c)
    c->mat_limit = pairs;
    return 0;
    QE_API_END(c)
}

int qe_scan_join(qe_ctx* c, const qe_pairs* R, const qe_pairs* S, qe_list* outR, qe_list* outS) {
    QE_API_BEGIN(c)
    pairs_need_keys(c, R);
    pairs_need_keys(c, S);
    uint64_t n = std::min(R->n, S->n);
    outR->d = dalloc_t<uint32_t>(c, std::max<uint64_t>(n, 1));
    outS->d = dalloc_t<uint32_t>(c, std::max<uint64_t>(n, 1));
    outR->cap = outS->cap = n;
    uint64_t m = scan_join_k(c, R->key, R->val, S->key, S->val, n, outR->d, outS->d);
    outR->n = outS->n = m;
    outR->flags = (R->flags & PF_DISTINCT) ? QE_LIST_DISTINCT : 0;
    outS->flags = (S->flags & PF_DISTINCT) ? QE_LIST_DISTINCT : 0;
    return 0;
    QE_API_END(c)
}

int qe_driver_counts(qe_ctx* c, const qe_pairs* R, const qe_pairs* S, const qe_list* outR, const qe_list* outS,
                     int mode, uint64_t rows, uint32_t** d_counts) {
    QE_API_BEGIN(c)
    if (mode != 0 && mode != 1) throw Error(QE_EINVAL, "mode");
    const bool sorted_inputs = R && S && (R->flags & PF_SORTED) && (S->flags & PF_SORTED);
    // the fast path reads the driving side's rowids + match counts (a fused join writes both) or,
    // without match counts, both sides' sorted keys; the general path reads the lists only
    const qe_pairs* A = mode == 0 ? R : S;
    const qe_pairs* B = mode == 0 ? S : R;
    if (sorted_inputs && (B->flags & PF_DISTINCT)) {
        if (A->match) {
            pairs_need_vals(c, A);
        } else {
            pairs_need_keys(c, A);
            pairs_need_keys(c, B);
        }
    }
    if (sorted_inputs && mode == 0 && (S->flags & PF_DISTINCT)) *d_counts = driver_counts_sorted(c, R, S, rows);
    else if (sorted_inputs && mode == 1 && (R->flags & PF_DISTINCT)) *d_counts = driver_counts_sorted(c, S, R, rows);
    else *d_counts = driver_counts_general(c, outR, outS, mode, rows);
    return 0;
    QE_API_END(c)
}

int qe_join_payloads_multi(qe_ctx* c, const uint32_t* d_counts, uint64_t rows, const qe_list* last,
                           const qe_list* const* edits, int nedits, qe_list* outs) {
    QE_API_BEGIN(c)
    for (int k = 0; k < nedits; k++)
        if (edits[k]->n < last->n) throw Error(QE_EINVAL, "join_payloads: |edit| < |last| (reference-undefined)");
    const uint64_t n = last->n;
    for (int k = 0; k < nedits; k++) {
        outs[k].n = outs[k].cap = 0;
        outs[k].flags = 0;
        outs[k].d = nullptr;
    }
    // 1. positions whose driver count is 0 emit nothing: keep (last[i], i) for the others -- or,
    //    with one edit list, (last[i], edit[i]): the stable sort below then leaves the payloads in
    //    the order edit[perm] would have, and the expansion reads them in order instead of
    //    gathering one 128-B line per 4-B payload
    const bool direct = nedits == 1;
    uint32_t* pl = dalloc_t<uint32_t>(c, std::max<uint64_t>(n, 1));
    uint32_t* pi = dalloc_t<uint32_t>(c, std::max<uint64_t>(n, 1));
    uint64_t m = 0;
    if (n) {
        const uint64_t nw = (rows + 31) / 32;
        uint32_t* nz = dalloc_t<uint32_t>(c, std::max<uint64_t>(nw, 1));
        {
            Timed t(c, "payload_bitmap", 4.0 * rows + nw * 4.0);
            hipLaunchKernelGGL(nonzero_bitmap_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, c->stream,
                               d_counts, rows, nz);
            QE_HIP(hipGetLastError());
        }
        m = compact_nonzero_pairs(c, nz, nw, last->d, direct ? edits[0]->d : nullptr, n, pl, pi);
        dfree(c, nz);
    }
    // 2. one stable sort by `last` for every edit list (the reference sorts R = (last, edit)
    //    by key per entry, src/join.c:444; the permutation is the same for all of them).
    //    Rowids are < rows, which bounds the bits the sort has to look at.
    uint64_t hb = 0;
    while (hb < 64 && (rows - 1) >> hb) hb++;
    uint64_t bits[2] = {hb >= 64 ? ~0ull : ((1ull << hb) - 1), 0};
    SortOut so = radix_sort_u32(c, pl, pi, m, rows > 1 ? bits : nullptr);
    const uint32_t* sk = (const uint32_t*)so.keys;
    const uint32_t* sidx = so.vals;
    // 3. per sorted position: driver multiplicity -> output offsets (shared)
    uint64_t P = 0;
    uint32_t mflag = 0;
    uint64_t* tc = nullptr;
    uint32_t nt = 0;
    if (m) {
        nt = (uint32_t)((m + X_TILE - 1) / X_TILE);
        tc = dalloc_t<uint64_t>(c, nt);
        uint32_t* d_flags = (uint32_t*)(c->d_scratch + 30);
        QE_HIP(hipMemsetAsync(d_flags, 0, 4, c->stream));
        {
            Timed t(c, "payload_count", 8.0 * m);
            hipLaunchKernelGGL(expand_kernel<0>, dim3(nt), dim3(XB), 0, c->stream, sk, sidx, m, d_counts, tc, nullptr,
                               d_flags, nullptr);
            QE_HIP(hipGetLastError());
            hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, c->stream, tc, (uint64_t)nt,
                               c->d_scratch + 31);
            QE_HIP(hipGetLastError());
        }
        uint64_t h[2];
        read_words(c, c->d_scratch + 30, h, 2);
        mflag = (uint32_t)h[0];
        P = h[1];
    }
    if (P > c->mat_limit) {   // the reference's DArray cannot hold it either (src/DArray.h:14-15)
        if (tc) dfree(c, tc);
        if (so.keys_new) dfree(c, so.keys);
        if (so.vals_new) dfree(c, so.vals);
        dfree(c, pl);
        dfree(c, pi);
        char msg[160];
        snprintf(msg, sizeof msg, "join_payloads of %llu rowids exceeds the materialisation limit %llu",
                 (unsigned long long)P, (unsigned long long)c->mat_limit);
        throw Error(QE_ETOOBIG, msg);
    }
    // 4. per edit list: edit[perm[i]] x multiplicity, in sorted order
    for (int k = 0; k < nedits; k++) {
        outs[k].d = dalloc_t<uint32_t>(c, std::max<uint64_t>(P, 1));
        outs[k].n = outs[k].cap = P;
        outs[k].flags = ((edits[k]->flags & QE_LIST_DISTINCT) && !(mflag & 1u)) ? QE_LIST_DISTINCT : 0;
        if (P) {
            Timed t(c, "payload_expand", 12.0 * m + 4.0 * P);
            hipLaunchKernelGGL(expand_kernel<1>, dim3(nt), dim3(XB), 0, c->stream, sk, direct ? sidx : edits[k]->d, m,
                               d_counts, tc, outs[k].d, nullptr, direct ? nullptr : sidx);
            QE_HIP(hipGetLastError());
        }
    }
    if (tc) dfree(c, tc);
    if (so.keys_new) dfree(c, so.keys);
    if (so.vals_new) dfree(c, so.vals);
    dfree(c, pl);
    dfree(c, pi);
    return 0;
    QE_API_END(c)
}

int qe_join_payloads(qe_ctx* c, const uint32_t* d_counts, uint64_t rows, const qe_list* last, const qe_list* edit,
                     qe_list* out) {
    const qe_list* e[1] = {edit};
    return qe_join_payloads_multi(c, d_counts, rows, last, e, 1, out);
}

int qe_checksum(qe_ctx* c, qe_col col, const qe_list* rows, uint64_t* sum) {
    QE_API_BEGIN(c)
    uint64_t n = rows ? rows->n : col.n;
    unsigned long long* d = (unsigned long long*)(c->d_scratch + 40);
    hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(64), 0, c->stream, (uint64_t*)d, 1);
    QE_HIP(hipGetLastError());
    if (n) {
        Timed t(c, "checksum", rows ? 12.0 * n : 8.0 * n);
        hipLaunchKernelGGL(checksum_kernel, dim3(grid_for(n, 256 * 16, 8192)), dim3(256), 0, c->stream, col.d,
                           rows ? rows->d : nullptr, n, d);
        QE_HIP(hipGetLastError());
    }
    *sum = read_u64(c, (const uint64_t*)d);
    return 0;
    QE_API_END(c)
}

int qe_checksums(qe_ctx* c, int n, const qe_col* cols, const qe_list* const* rows, uint64_t* sums) {
    QE_API_BEGIN(c)
    if (n < 0) throw Error(QE_EINVAL, "n");
    for (int k0 = 0; k0 < n; k0 += 32) {   // 32 sums per round trip (the pinned scratch holds 64 words)
        const int m = std::min(32, n - k0);
        unsigned long long* d = (unsigned long long*)dalloc_t<uint64_t>(c, 32);
        hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(64), 0, c->stream, (uint64_t*)d, 32);
        QE_HIP(hipGetLastError());
        for (int k = 0; k < m; k++) {
            const qe_list* r = rows[k0 + k];
            const uint64_t len = r ? r->n : cols[k0 + k].n;
            if (!len) continue;
            Timed t(c, "checksum", r ? 12.0 * len : 8.0 * len);
            hipLaunchKernelGGL(checksum_kernel, dim3(grid_for(len, 256 * 16, 8192)), dim3(256), 0, c->stream,
                               cols[k0 + k].d, r ? r->d : nullptr, len, d + k);
            QE_HIP(hipGetLastError());
        }
        read_words(c, (const uint64_t*)d, sums + k0, m);
        dfree(c, d);
    }
    return 0;
    QE_API_END(c)
}

}  // extern "C"

#ifdef QE_DIAG_STAMPS
extern "C" int qe_diag_stamps_sort(const char* which, uint64_t* out, uint64_t n);
extern "C" int qe_diag_stamps_cp(uint64_t* out, uint64_t n);
extern "C" int qe_diag_stamps_ag(uint64_t* out, uint64_t n);
// tuning builds only (not part of qe.h): copy the last launch's phase stamps out
extern "C" int qe_diag_stamps(const char* which, uint64_t* out, uint64_t n) {
    (void)hipDeviceSynchronize();
    if (!strcmp(which, "mj")) return hipMemcpyFromSymbol(out, HIP_SYMBOL(qe::g_mj_stamps), n * 8) == hipSuccess ? 0 : -2;
    if (!strcmp(which, "cp")) return qe_diag_stamps_cp(out, n);
    if (!strcmp(which, "ag")) return qe_diag_stamps_ag(out, n);
    return qe_diag_stamps_sort(which, out, n);
}
#endif
