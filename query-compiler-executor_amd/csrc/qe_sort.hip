// qe_sort.hip -- stable LSD radix sort of (key, rowid) pairs on gfx950.
//
// Replaces the reference's iterative_sort (MSD radix with a FIFO of buckets, src/join.c:5-94)
// and its randomised quicksort for small buckets (src/quicksort.c:7-64).  The reference's tie
// order depends on rand(); ours is stable (input order), which is one of the orders the
// reference can produce and unobservable on the rand-invariant domain.
//
// Pipeline for n pairs:
//   1. key bits     -- OR / AND of the keys (known from the producer: column statistics at load
//                      time, or fused into the gather): only the bit range [lo, hi) that varies is
//                      sorted -- 27 bits at 100 M rows, i.e. 3 passes of 9 bits, not 8 of 8.
//   2. packing      -- when hi - lo <= 32 the pair travels as ONE u64 word (field << 32 | rowid):
//                      the first pass reads key + rowid and writes words, middle passes move 8 B
//                      in + 8 B out per pair, the last pass writes key + rowid back (the key's
//                      constant bits are restored from the AND).  Otherwise key and rowid travel
//                      separately (64-bit keys with > 32 varying bits; the dedup sort of packed
//                      pairs has no rowid at all).
//   3. digit_hist   -- one read of the keys builds the histograms of every pass in LDS.
//   4. digit_scan   -- exclusive scan per pass -> global base offset of each digit.
//   5. radix_pass   -- per pass: a tile of 512 x 16 words is ranked in registers (RBITS
//                      ballots per element = wave match-any, per-wave LDS counters), staged in
//                      LDS in digit order, THEN the per-digit decoupled lookback (thread-serial,
//                      one chain per digit) -- its latency overlaps the staging -- and the tile
//                      is written as runs of equal digits.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "qe_device.h"
#include "qe_internal.h"

namespace qe {

// pass outputs: plain or non-temporal stores (tuning knob, A/B: QE_NT_STORE=1)
#ifdef QE_NT_STORE
#define QE_ST(ptr, v) __builtin_nontemporal_store((v), (ptr))
#else
#define QE_ST(ptr, v) (*(ptr) = (v))
#endif

// Where a write-out lane with nothing to write may send its store (QE_STORE_SINK=1 builds): every
// store of a write-out loop is then issued unconditionally, so the compiler waits for the payload
// loads with a counted vmcnt(N) instead of vmcnt(0) (a guarded store is a branch; gfx9 counts loads
// and stores together).  Measured: the sink form 3.08 vs 3.02-3.05 ms of sort_pass_carry per C3
// query for guarded stores, same box (profiles/r04h_store_sink_ab.log) -- pass 2's sub-tiles leave
// ~10 % of the lanes without a word, and their sink stores cost more than the waits saved.  The
// default keeps guarded stores.
__device__ uint64_t g_store_sink[64];
#ifndef QE_STORE_SINK
#define QE_STORE_SINK 0
#endif
// QE_STS(ok, ptr, sinkptr, v): the store of a write-out lane -- to ptr when ok, else (sink form)
// to the sink, or (QE_STORE_SINK=0, A/B build) not at all
#if QE_STORE_SINK
#define QE_STS(ok, ptr, sinkp, v) QE_ST((ok) ? (ptr) : (sinkp), (v))
#define QE_STP(ok, ptr, sinkp, v) (*((ok) ? (ptr) : (sinkp)) = (v))
#else
#define QE_STP(ok, ptr, sinkp, v) \
    do {                          \
        if (ok) *(ptr) = (v);     \
    } while (0)
#define QE_STS(ok, ptr, sinkp, v) \
    do {                          \
        if (ok) QE_ST((ptr), (v)); \
    } while (0)
#endif
// the two-level second pass's stores (QE_NT_STORE2=1, A/B build: non-temporal there only).  Round 6,
// same box: sort_pass_carry 3.04 -> 3.67 ms per C3 query, while the kernels reading its output got
// faster (bucket_join_sums 0.262 -> 0.204) -- a net loss (profiles/r06zc_c3_bench.log)
#ifdef QE_NT_STORE2
#define QE_STS2(ok, ptr, sinkp, v)                               \
    do {                                                         \
        if (ok) __builtin_nontemporal_store((v), (ptr));         \
    } while (0)
#else
#define QE_STS2(ok, ptr, sinkp, v) QE_STS(ok, ptr, sinkp, v)
#endif


constexpr int RB = 256;          // block
constexpr int RNW = RB / 64;     // waves per block
#ifndef QE_R_ITEMS
#define QE_R_ITEMS 16
#endif
#ifndef QE_R_THREADS
#define QE_R_THREADS 512
#endif
constexpr int R_NT = QE_R_THREADS;    // threads per onesweep tile
constexpr int R_ITEMS = QE_R_ITEMS;   // words per thread per tile
constexpr int RTILE = R_NT * R_ITEMS;
constexpr int KV_TILE = RB * R_ITEMS;   // radix_pass_kv_kernel: always RB threads
constexpr int MAX_PASS = 8;

template <typename K>
__global__ void __launch_bounds__(256) key_bits_kernel(const K* __restrict__ keys, uint64_t n, uint64_t* out) {
    uint64_t o = 0, a = ~0ull;
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint64_t k = (uint64_t)keys[i];
        o |= k;
        a &= k;
    }
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
        for (int w = 1; w < 4; w++) {
            o |= so[w];
            a &= sa[w];
        }
        atomicOr((unsigned long long*)&out[0], (unsigned long long)o);
        atomicAnd((unsigned long long*)&out[1], (unsigned long long)a);
    }
}

struct PassDesc {
    int npass;
    int shift[MAX_PASS];        // absolute key bit of each digit
    uint32_t mask[MAX_PASS];
};

// Visits keys[0, n): a block takes chunks of blockDim * U consecutive keys (grid-stride), thread t
// keys t, t + blockDim, ... of its chunk, all U loads of a chunk in flight together -- unconditional
// in a full chunk, index-clamped and masked in the last one.  (A guarded load per element, `i < n ?
// keys[i] : 0`, left one load in flight per thread: the histogram kernels below were latency-bound.)
template <int U, typename K, typename F>
__device__ __forceinline__ void for_each_key(const K* __restrict__ keys, uint64_t n, F&& f) {
    const uint64_t per = (uint64_t)blockDim.x * U;
    for (uint64_t c0 = (uint64_t)blockIdx.x * per; c0 < n; c0 += (uint64_t)gridDim.x * per) {
        K k[U];
        if (c0 + per <= n) {   // block-uniform
#pragma unroll
            for (int q = 0; q < U; q++) k[q] = keys[c0 + (uint64_t)q * blockDim.x + threadIdx.x];
#pragma unroll
            for (int q = 0; q < U; q++) f(k[q]);
        } else {
#pragma unroll
            for (int q = 0; q < U; q++) {
                const uint64_t i = c0 + (uint64_t)q * blockDim.x + threadIdx.x;
                k[q] = keys[i < n ? i : n - 1];
            }
#pragma unroll
            for (int q = 0; q < U; q++)
                if (c0 + (uint64_t)q * blockDim.x + threadIdx.x < n) f(k[q]);
        }
    }
}

template <typename K, int RBITS>
__global__ void __launch_bounds__(256) digit_hist_kernel(const K* __restrict__ keys, uint64_t n, PassDesc pd,
                                                         uint32_t* __restrict__ hist) {
    constexpr int BINS = 1 << RBITS;
    constexpr int HP = RBITS <= 8 ? 8 : (64 + RBITS - 1) / RBITS;   // passes that fit
    __shared__ uint32_t h[HP * BINS];
    for (int i = threadIdx.x; i < HP * BINS; i += blockDim.x) h[i] = 0;
    __syncthreads();
    for_each_key<8>(keys, n, [&](K kk) {
        const uint64_t k = (uint64_t)kk;
        for (int p = 0; p < pd.npass; p++) atomicAdd(&h[p * BINS + ((uint32_t)(k >> pd.shift[p]) & pd.mask[p])], 1u);
    });
    __syncthreads();
    for (int i = threadIdx.x; i < pd.npass * BINS; i += blockDim.x) {
        uint32_t v = h[i];
        if (v) atomicAdd(&hist[i], v);
    }
}

// block of 256 threads per pass: exclusive scan of BINS counts (thread owns BINS/256 digits)
template <int RBITS>
__global__ void __launch_bounds__(256) digit_scan_kernel(uint32_t* hist) {
    constexpr int BINS = 1 << RBITS, DPT = BINS / RB;
    __shared__ uint32_t wsum[RNW];
    uint32_t* h = hist + blockIdx.x * BINS;
    uint32_t v[DPT], s = 0;
#pragma unroll
    for (int q = 0; q < DPT; q++) {
        v[q] = h[threadIdx.x * DPT + q];
        s += v[q];
    }
    uint32_t inc = wave_incl_scan_u32(s);
    if (lane_id() == 63) wsum[wave_id()] = inc;
    __syncthreads();
    uint32_t run = inc - s;
    for (int w = 0; w < wave_id(); w++) run += wsum[w];
#pragma unroll
    for (int q = 0; q < DPT; q++) {
        h[threadIdx.x * DPT + q] = run;
        run += v[q];
    }
}

// input / output formats of a pass
enum { IN_WORD = 0, IN_KV = 1, IN_KIOTA = 2, IN_KV64 = 3 };   // IN_KV64: `vin` is a u64 column, low 32 bits packed
enum { OUT_WORD = 0, OUT_KV = 1, OUT_W32 = 2 };   // OUT_W32: the word's field only, as u32 (no rowid)

// word <-> (key, rowid).  PACK: word = ((key >> lo) & fmask) << 32 | rowid, key restored as
// kconst | (field << lo).  !PACK: word = key (no rowid; key-only sorts of 64-bit words).
struct Field {
    int lo;
    uint64_t fmask;
    uint64_t kconst;
};

#ifdef QE_DIAG_STAMPS
__device__ uint64_t g_sort_stamps[STAMP_TILES * STAMP_SLOTS];
__device__ uint64_t g_hj_stamps[STAMP_TILES * STAMP_SLOTS];
__device__ uint32_t g_sort_stamp_on = 1;   // the sort kernels stamp only while this is set
// QE_STAMP_SEL=p1:K or p2:K (tuning builds only): stamp only the K-th lookback-free first pass /
// the K-th second pass of the process (1-based; their order is logged to stderr), so one
// launch of a whole query's sorts can be looked at (tools/stamps.py --what c3p1 / c3p2)
static void stamp_select(qe_ctx* c, const char* kind, uint64_t n) {
    static uint32_t cnt[2] = {0, 0};
    const int k = kind[1] == '1' ? 0 : 1;
    const uint32_t idx = ++cnt[k];
    const char* sel = getenv("QE_STAMP_SEL");
    uint32_t on = 1;
    if (sel && sel[0] == 'p') on = (sel[1] == kind[1] && (uint32_t)atoi(sel + 3) == idx) ? 1u : 0u;
    if (sel) fprintf(stderr, "[stamps] %s launch %u: n = %llu%s\n", kind, idx, (unsigned long long)n, on ? " (stamped)" : "");
    QE_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_sort_stamp_on), &on, sizeof on, 0, hipMemcpyHostToDevice, c->stream));
}
#define QE_SORT_STAMP(tile, k) \
    do {                       \
        if (g_sort_stamp_on) QE_STAMP(g_sort_stamps, tile, k); \
    } while (0)
#else
#define QE_SORT_STAMP(tile, k) ((void)0)
#endif

// XCD-contiguous work items for the lookback-free passes: a grid of 8 * per blocks, block b takes
// item (b % 8) * per + b / 8, so the blocks that share an XCD (b % 8 equal under the observed
// round-robin placement -- speed only) walk one contiguous range of tiles in dispatch order, and
// the digit runs that neighbouring tiles write side by side mostly meet in the same L2, which
// merges their shared boundary lines.  QE_XCD_TILES=0 (build knob) keeps item = b.
#ifndef QE_XCD_TILES
#define QE_XCD_TILES 1
#endif
__device__ __forceinline__ uint32_t xcd_item(uint32_t b) {
    return QE_XCD_TILES ? (b & 7u) * (gridDim.x >> 3) + (b >> 3) : b;
}
static inline uint32_t xcd_grid(uint64_t items) {
    return QE_XCD_TILES ? (uint32_t)(8 * ((items + 7) / 8)) : (uint32_t)items;
}

// One pass over a tile of NT x ITEMS words: rank in registers (RBITS ballots per element = wave
// match-any, per-wave LDS counters), stage the tile in LDS in digit order, then write it as runs
// of equal digits.  The tile's global digit offsets come from a per-digit decoupled lookback
// (thread-serial, one chain per digit; the tile aggregate is published before staging so the
// chain overlaps it).  `offs` = the pass's digit bases.
// Measured on MI355X (1e8 pairs, 4 passes): tile size sets the length of each digit's output run
// (tile / bins words) -- 8192-word tiles beat 4096 by 15 %; 512 threads x 16 beat 256 x 32 by
// 10 % (twice the waves per CU at the same LDS); a reduce-then-scan variant without lookback
// (per-tile count pass + scan + scatter) measured equal: its extra read cancels the saving.
// PRE = true: the tile's global digit offsets were computed before the launch (the two-level
// sort's first pass, whose per-tile counts come out of the histogram read it does anyway,
// tl_hist_tiles_kernel) -- `offs` is a table of BINS offsets per tile; no ticket, no lookback.
// CARRY (PRE, OUT_WORD only): a payload per element rides along, written to xout at the element's
// output position -- X64: 64 bits, xa[i] | xb[i] << 32 in input order (xb nullable; the partitioned
// plan's carried bindings, qe_join_carry); X32: 32 bits, xa[i] (u32 input); XCOL: 32 bits, the low
// word of the u64 column xa points to (a base relation's next join key riding with its rows).  The
// words are written first; the same LDS stage then takes the payloads in the words' slots, so
// they leave in the same runs.
// TM (PRE only): one workgroup takes TM consecutive counted tiles -- its run of digit d starts at
// the first one's offset and is the TM tiles' runs back to back (the column scan orders a group's
// tiles consecutively), so nothing else changes (see P1_TM).
// UNSTABLE: ranks from per-wave LDS counters (one ds_add_rtn per element) instead of the 8-ballot
// match-any -- equal digits keep no order.  For the partitioned plan's deferred sorts (their
// consumer, bucket_join, needs the buckets, not an order inside them) and the first LSD pass of
// the aggregate join's sorts (no earlier order to keep, none needed among equal keys).
#ifndef QE_P1_EARLY
#define QE_P1_EARLY 1
#endif
#ifndef QE_STAGE_FLAT   // (build knob: 1 = branch-free staging in pass 1, measured ~1 % slower)
#define QE_STAGE_FLAT 0
#endif
enum { X_NONE = 0, X64 = 1, X32 = 2, XCOL = 3 };
template <typename K, int IN, int OUT, bool PACK, int RBITS, int ITEMS, int NT, bool PRE = false, int CARRY = X_NONE,
          bool UNSTABLE = false, int TM = 1>
__global__ void __launch_bounds__(NT) radix_pass_kernel(const K* __restrict__ kin, const uint64_t* __restrict__ win,
                                                        const uint32_t* __restrict__ vin, K* __restrict__ kout,
                                                        uint64_t* __restrict__ wout, uint32_t* __restrict__ vout,
                                                        uint64_t n, int dsh, uint32_t mask, Field f,
                                                        const uint32_t* __restrict__ offs, uint64_t* status,
                                                        uint32_t* ticket, uint32_t epoch,
                                                        const uint32_t* __restrict__ xa = nullptr,
                                                        const uint32_t* __restrict__ xb = nullptr,
                                                        uint64_t* __restrict__ xout = nullptr) {
    static_assert(CARRY == X_NONE || (PRE && OUT == OUT_WORD), "payload carry: the lookback-free first pass only");
    static_assert(TM == 1 || PRE, "a tile of TM counted tiles: the lookback-free first pass only");
    constexpr int BINS = 1 << RBITS, DPT = BINS >= NT ? BINS / NT : 1;   // digits per thread
    constexpr int NW = NT / 64;
    constexpr int TILE = NT * ITEMS, WT = 64 * ITEMS;
    const bool owner = DPT > 1 || (int)threadIdx.x < BINS;   // this thread owns digits
    // per-wave digit counts -> exclusive over waves; UNSTABLE ranks on ONE block-wide row (no order
    // to keep between waves), which leaves a 1024-thread tile in 2 workgroups' LDS per CU
    constexpr int NWH = UNSTABLE ? 1 : NW;
    __shared__ uint64_t stage[TILE + 1];     // (+1: the flat staging's spare slot)
    __shared__ uint32_t whist[NWH][BINS];
    __shared__ uint32_t bexcl[BINS];        // tile-local exclusive offset of each digit
    __shared__ uint32_t gofs[BINS];         // global position of the digit's run - bexcl
    __shared__ uint32_t wsum[NW];
    __shared__ uint32_t s_ticket;

#ifdef QE_DIAG_STAMPS
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
    const uint32_t tile = PRE ? xcd_item(blockIdx.x) : take_ticket(ticket, &s_ticket);
    if (PRE && (uint64_t)tile * TILE >= n) return;   // the XCD grid's padding blocks (block-uniform)
#ifdef QE_DIAG_STAMPS
    if (g_sort_stamp_on && threadIdx.x == 0 && tile < STAMP_TILES) g_sort_stamps[(uint64_t)tile * STAMP_SLOTS] = t_start;
#endif
    const int w = wave_id(), l = lane_id();
    const uint64_t lt = lanemask_lt();
    // PRE: this tile's digit offsets, loaded first -- issued after the payload loads, their wait
    // also waited for those
    uint32_t pre_off[PRE ? DPT : 1];
    if constexpr (PRE) {
#pragma unroll
        for (int q = 0; q < DPT; q++) pre_off[q] = owner ? offs[(uint64_t)tile * TM * BINS + threadIdx.x * DPT + q] : 0u;
    }
    // the rank counters are zeroed AFTER the element loads are issued (below, for PRE tiles): a
    // barrier first would hold every wave's loads until the block's last wave has launched
    // (QE_P1_EARLY=0: build knob, round 4's zero -> barrier -> loads)
    if constexpr (!PRE || !QE_P1_EARLY) {
        for (int i = threadIdx.x; i < NWH * BINS; i += NT) (&whist[0][0])[i] = 0;
        __syncthreads();
    }
    QE_SORT_STAMP(tile, 1);

    uint64_t word[ITEMS];
    uint32_t pos[ITEMS];
    // every load unconditional, through buffer descriptors over this tile's elements (those past
    // n read as 0): a guarded load became a branch whose value the compiler waited for inside it
    const uint64_t tb = (uint64_t)tile * TILE;
    const uint32_t tcount = (uint32_t)((n - tb) < (uint64_t)TILE ? (n - tb) : (uint64_t)TILE);
    const uint32_t loc0 = (uint32_t)w * WT + (uint32_t)l;   // this lane's first tile-local element
    // V4 (unstable ranks, u32 keys and u32 side arrays): a lane loads 16 B = 4 consecutive elements
    // of each array (1 KiB per wave instruction instead of 256 B) -- element j of lane l is then
    // tile-local w * WT + (j / 4) * 256 + 4 l + j % 4.  A partial tile loads them one by one.
    constexpr bool V4 = UNSTABLE && sizeof(K) == 4 && (IN == IN_KIOTA || IN == IN_KV) && CARRY != XCOL && ITEMS % 4 == 0;
    auto loc_of = [&](int j) -> uint32_t {
        return V4 ? (uint32_t)w * WT + (uint32_t)(j >> 2) * 256u + (uint32_t)l * 4u + (uint32_t)(j & 3)
                  : loc0 + (uint32_t)j * 64u;
    };
    // u32 elements j of one array at the V4 mapping, every tile alike (no branch: the compiler's
    // waits stay counted).  The descriptors of V4 arrays cover the tile rounded up to whole 16-B
    // units (v4_bytes): the last unit of a partial tile reads up to 3 elements past n -- inside the
    // allocation, whose size granule is a multiple of 16 B (the V4 arrays are hipMalloc'd u32 column
    // copies or dalloc'd lists, 256-B aligned) -- and they are masked by `ok` like the rest.
    auto load_v4 = [&](const __amdgpu_buffer_rsrc_t& r, uint32_t (&x)[ITEMS]) {
#pragma unroll
        for (int g = 0; g < ITEMS / 4; g++) {
            const uint4 a = buf_load_u4(r, ((uint32_t)w * WT + (uint32_t)l * 4u) * 4u, (uint32_t)g * 1024u);
            x[4 * g] = a.x;
            x[4 * g + 1] = a.y;
            x[4 * g + 2] = a.z;
            x[4 * g + 3] = a.w;
        }
    };
    const uint32_t v4_bytes = (tcount * 4u + 15u) & ~15u;
    if constexpr (IN == IN_WORD) {
        const auto rw = buf_rsrc(win + tb, tcount * 8u);
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint2 v = buf_load_u2(rw, loc0 * 8u, (uint32_t)j * 512u);
            word[j] = (uint64_t)v.y << 32 | v.x;
        }
    } else if constexpr (V4) {
        uint32_t kk[ITEMS], vv[ITEMS];
        load_v4(buf_rsrc(kin + tb, v4_bytes), kk);
        if constexpr (IN == IN_KV) load_v4(buf_rsrc(vin + tb, v4_bytes), vv);
#pragma unroll
        for (int j = 0; j < ITEMS; j++)
            word[j] = ((((uint64_t)kk[j] >> f.lo) & f.fmask) << 32) |
                      (IN == IN_KV ? vv[j] : (uint32_t)(tb + loc_of(j)));
    } else {
        const auto rk = buf_rsrc(kin + tb, tcount * (uint32_t)sizeof(K));
        const auto rv = IN == IN_KV64 ? buf_rsrc(reinterpret_cast<const uint64_t*>(vin) + tb, tcount * 8u)
                                      : buf_rsrc(IN == IN_KV ? vin + tb : vin, IN == IN_KV ? tcount * 4u : 0u);
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            uint64_t k;
            if constexpr (sizeof(K) == 8) {
                const uint2 v = buf_load_u2(rk, loc0 * 8u, (uint32_t)j * 512u);
                k = (uint64_t)v.y << 32 | v.x;
            } else {
                k = buf_load_u32(rk, loc0 * 4u, (uint32_t)j * 256u);
            }
            if (PACK) {
                uint32_t v;
                if constexpr (IN == IN_KV) v = buf_load_u32(rv, loc0 * 4u, (uint32_t)j * 256u);
                else if constexpr (IN == IN_KV64) v = buf_load_u2(rv, loc0 * 8u, (uint32_t)j * 512u).x;
                else v = (uint32_t)(tb + loc0 + (uint32_t)j * 64);
                word[j] = (((k >> f.lo) & f.fmask) << 32) | v;
            } else {
                word[j] = k;
            }
        }
    }
    constexpr bool P32 = CARRY == X32 || CARRY == XCOL;
    uint32_t xw[P32 ? ITEMS : 1];
    auto load_payloads = [&]() {
        if constexpr (CARRY != X_NONE) {
            const auto ra = CARRY == XCOL ? buf_rsrc(reinterpret_cast<const uint64_t*>(xa) + tb, tcount * 8u)
                                          : buf_rsrc(xa + tb, V4 ? v4_bytes : tcount * 4u);
            const auto rb = buf_rsrc(xb ? xb + tb : xa, xb ? (V4 ? v4_bytes : tcount * 4u) : 0u);   // (no xb: reads 0)
            if constexpr (V4 && CARRY == X64) {
                uint32_t xa4[ITEMS], xb4[ITEMS];
                load_v4(ra, xa4);
                load_v4(rb, xb4);
#pragma unroll
                for (int j = 0; j < ITEMS; j++) word[j] = (uint64_t)xa4[j] | (uint64_t)xb4[j] << 32;
            } else if constexpr (V4) {
                load_v4(ra, xw);
            } else {
#pragma unroll
                for (int j = 0; j < ITEMS; j++) {
                    if constexpr (CARRY == X64)
                        word[j] = (uint64_t)buf_load_u32(ra, loc0 * 4u, (uint32_t)j * 256u) |
                                  (uint64_t)buf_load_u32(rb, loc0 * 4u, (uint32_t)j * 256u) << 32;
                    else if constexpr (CARRY == X32) xw[j] = buf_load_u32(ra, loc0 * 4u, (uint32_t)j * 256u);
                    else xw[j] = buf_load_u2(ra, loc0 * 8u, (uint32_t)j * 512u).x;
                }
            }
        }
    };
    if constexpr (PRE && QE_P1_EARLY) {   // (the loads above are in flight across this barrier)
        for (int i = threadIdx.x; i < NWH * BINS; i += NT) (&whist[0][0])[i] = 0;
        __syncthreads();
    }
    // stable rank inside the wave: element order is (j, lane)
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        const bool ok = loc_of(j) < tcount;
        uint32_t d = (uint32_t)(word[j] >> dsh) & mask;
        if constexpr (UNSTABLE) {
            pos[j] = ok ? atomicAdd(&whist[0][d], 1u) : 0u;
            continue;
        }
#ifdef QE_DIAG_SORT_NORANK   // ablation only: LDS-atomic ranks instead of match-any (unstable, in range)
        (void)lt;
        pos[j] = ok ? atomicAdd(&whist[w][d], 1u) : 0u;
#else
        uint64_t peers = __ballot(ok);
#pragma unroll
        for (int b = 0; b < RBITS; b++) {
            bool bit = (d >> b) & 1u;
            uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        int leader = peers ? (__ffsll((unsigned long long)peers) - 1) : 0;
        uint32_t old = 0;
        if (ok && l == leader) {
            old = whist[w][d];
            whist[w][d] = old + (uint32_t)__popcll(peers);
        }
        old = (uint32_t)__shfl((int)old, leader, 64);
        pos[j] = old + (uint32_t)__popcll(peers & lt);
#endif
    }
    uint32_t tot[DPT], tsum = 0;
    __syncthreads();
    QE_SORT_STAMP(tile, 2);
    // thread t owns digits t*DPT .. t*DPT+DPT-1: totals, exclusive over waves, publish aggregate
#pragma unroll
    for (int q = 0; q < DPT; q++) {
        const uint32_t d = threadIdx.x * DPT + q;
        tot[q] = 0;
        if (!owner) continue;
        uint32_t t = 0;
#pragma unroll
        for (int ww = 0; ww < NWH; ww++) {
            uint32_t c = whist[ww][d];
            whist[ww][d] = t;
            t += c;
        }
        tot[q] = t;
        tsum += t;
        if (!PRE) st_agent(&status[(uint64_t)tile * BINS + d], lb_word(epoch, tile == 0 ? LB_FLAG_INC : LB_FLAG_AGG, t));
    }
    uint32_t inc = wave_incl_scan_u32(tsum);
    if (l == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t run = inc - tsum;
    for (int ww = 0; ww < w; ww++) run += wsum[ww];
#pragma unroll
    for (int q = 0; q < DPT; q++) {
        if (owner) bexcl[threadIdx.x * DPT + q] = run;
        run += tot[q];
    }
    __syncthreads();
    QE_SORT_STAMP(tile, 3);
    // stage the tile in digit order (tile-local offsets only).  QE_STAGE_FLAT (round 5): every
    // slot's offset read issued before the first store, no branch per element (an element past
    // the tile goes to the spare slot), and unstable ranks read one table, not two (their wave
    // row is all zeros after the scan); else the round-4 form, one guarded round trip per element
    if constexpr (QE_STAGE_FLAT) {
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint32_t dd = (uint32_t)(word[j] >> dsh) & mask;
            const uint32_t b = bexcl[dd] + (UNSTABLE ? 0u : whist[w][dd]);
            pos[j] = loc_of(j) < tcount ? b + pos[j] : (uint32_t)TILE;
        }
#pragma unroll
        for (int j = 0; j < ITEMS; j++) stage[pos[j]] = word[j];   // (pos: the slot from here on)
    } else {
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        if (loc_of(j) < tcount) {
            uint32_t dd = (uint32_t)(word[j] >> dsh) & mask;
            const uint32_t slot = bexcl[dd] + whist[UNSTABLE ? 0 : w][dd] + pos[j];
            stage[slot] = word[j];
            if constexpr (CARRY != X_NONE) pos[j] = slot;   // the payload takes the same slot later
        }
    }
    }
    // the payloads load into the words' registers (a 32-bit one into registers of its own), in
    // flight during the write-out
    load_payloads();
#pragma unroll
    for (int q = 0; q < DPT; q++) {
        const uint32_t d = threadIdx.x * DPT + q;
        if (!owner) continue;
        if constexpr (PRE) {
            gofs[d] = pre_off[q] - bexcl[d];
            continue;
        }
        // the predecessors' counts: by this time most have published their inclusive prefix
        uint64_t ex = 0;
#ifndef QE_DIAG_SORT_NOLB   // ablation only: skip the lookback (output positions are wrong)
        if (tile > 0) {
            ex = lookback_serial(status, epoch, tile, BINS, d);
            st_agent(&status[(uint64_t)tile * BINS + d], lb_word(epoch, LB_FLAG_INC, ex + tot[q]));
        }
#endif
        gofs[d] = offs[d] + (uint32_t)ex - bexcl[d];
    }
    QE_SORT_STAMP(tile, 4);
    __syncthreads();
    QE_SORT_STAMP(tile, 5);
    const uint64_t tbase = (uint64_t)tile * TILE;
    const uint32_t tn = (uint32_t)((n - tbase) < (uint64_t)TILE ? (n - tbase) : (uint64_t)TILE);
    uint32_t pk[CARRY != X_NONE ? ITEMS : 1];
    // written in chunks of RW_CH slots: a chunk's stage and offset reads are all issued before its
    // first store (no branch between them: a slot past the tile reads a stale word and is not
    // stored), the next chunk held back (sched_barrier) so the registers stay within budget
    constexpr int RW_CH = ITEMS % 8 == 0 ? 8 : 1;
#pragma unroll
    for (int k0 = 0; k0 < ITEMS; k0 += RW_CH) {
        uint64_t wd[RW_CH];
        uint32_t pp[RW_CH];
#pragma unroll
        for (int q = 0; q < RW_CH; q++) wd[q] = stage[(uint32_t)(k0 + q) * NT + threadIdx.x];
#pragma unroll
        for (int q = 0; q < RW_CH; q++) {
            const uint32_t i = (uint32_t)(k0 + q) * NT + threadIdx.x;
#ifdef QE_DIAG_SORT_LINEAR   // ablation only: contiguous output instead of the digit scatter
            pp[q] = (uint32_t)(tbase + i);
#else
            pp[q] = gofs[(uint32_t)(wd[q] >> dsh) & mask] + i;
#endif
        }
#pragma unroll
        for (int q = 0; q < RW_CH; q++) {
            const int k = k0 + q;
            const uint32_t i = (uint32_t)k * NT + threadIdx.x, p = pp[q];
            // (p >= n: never with consistent offsets; keeps stores in bounds)
            const bool ok = i < tn && (uint64_t)p < n;
            if constexpr (CARRY != X_NONE) pk[k] = ok ? p : 0xFFFFFFFFu;
            const uint64_t x = wd[q];
            // every store issued (a lane with nothing to write stores to g_store_sink): no branch
            if (OUT == OUT_WORD) {
                QE_STS(ok, &wout[p], &g_store_sink[l], x);
            } else if (OUT == OUT_W32) {
                QE_STS(ok, &reinterpret_cast<uint32_t*>(wout)[p], reinterpret_cast<uint32_t*>(&g_store_sink[l]), (uint32_t)(x >> 32));
            } else if (PACK) {
                QE_STP(ok, &kout[p], reinterpret_cast<K*>(&g_store_sink[l]), (K)(f.kconst | ((x >> 32) << f.lo)));
                QE_STP(ok, &vout[p], reinterpret_cast<uint32_t*>(&g_store_sink[l]), (uint32_t)x);
            } else {
                QE_STP(ok, &kout[p], reinterpret_cast<K*>(&g_store_sink[l]), (K)x);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (CARRY != X_NONE) {
        __syncthreads();   // every word is out of the stage
        uint32_t* st32 = reinterpret_cast<uint32_t*>(stage);   // (32-bit payloads: 4-B slots)
#pragma unroll
        for (int j = 0; j < ITEMS; j++)
            if (QE_STAGE_FLAT || loc_of(j) < tcount) {   // (flat: past the tile, the spare slot)
                if constexpr (P32) st32[pos[j]] = xw[j];
                else stage[pos[j]] = word[j];
            }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < ITEMS; k++) {
            const uint32_t i = (uint32_t)k * NT + threadIdx.x;
            const bool ok = pk[k] != 0xFFFFFFFFu;   // (set only for i < tn)
            if constexpr (CARRY == X64) QE_STS(ok, &xout[pk[k]], &g_store_sink[l], stage[i]);
            else QE_STS(ok, &reinterpret_cast<uint32_t*>(xout)[pk[k]], reinterpret_cast<uint32_t*>(&g_store_sink[l]), st32[i]);
        }
    }
    QE_SORT_STAMP(tile, 6);
}

// ---- two-level sort: 14 high bits by two global passes, the rest inside LDS per bucket ---------
// For 20..31 varying bits: the top H = 15 bits split the array into 32768 buckets (~4 K words
// each at 10^8 keys below 10^8 -- keys rarely fill their top bit's range, so H leaves room);
// two onesweep passes (8 + 7 bits, LSD order) leave it bucket-partitioned and stable; then one
// workgroup per bucket sorts the bucket's remaining L = bits - 15 bits in LDS (two stable ranking
// rounds, no lookback: the bucket boundaries come from the histogram) and writes key + rowid
// coalesced.  64 B per element instead of 80, two lookback passes instead of 4.  A bucket larger
// than LDS (skew) sends the whole sort back to the plain LSD passes.
constexpr int TL_H = 15;
constexpr int TL_BUCKETS = 1 << TL_H;
#ifndef QE_TL_NT
#define QE_TL_NT 512
#endif
#ifndef QE_TL_ITEMS
#define QE_TL_ITEMS 10
#endif
constexpr int TL_NT = QE_TL_NT, TL_ITEMS = QE_TL_ITEMS, TL_CAP = TL_NT * TL_ITEMS;   // words per bucket in LDS

// histogram of the top TL_H varying bits (bucket id = field >> L)
template <typename K>
__global__ void __launch_bounds__(1024) tl_hist_kernel(const K* __restrict__ keys, uint64_t n, Field f, int L,
                                                       uint32_t* __restrict__ hist) {
    __shared__ alignas(16) uint32_t h[TL_BUCKETS];   // 128 KiB: one block per CU, 16 waves
    for (int i = threadIdx.x; i < TL_BUCKETS; i += 1024) h[i] = 0;
    __syncthreads();
    for_each_key<8>(keys, n, [&](K k) {
        atomicAdd(&h[(uint32_t)(((((uint64_t)k >> f.lo) & f.fmask) >> L) & (TL_BUCKETS - 1))], 1u);
    });
    __syncthreads();
    for (int i = threadIdx.x; i < TL_BUCKETS; i += 1024)
        if (h[i]) atomicAdd(&hist[i], h[i]);
}

// A 32 K-bucket table held by one 1024-thread block, 32 consecutive buckets per thread (the scans'
// layout), moved between global memory and registers through LDS padded by one word per 32:
// lane-contiguous global accesses and conflict-free row reads (stride 33 words).  Each thread
// reading its own 32 words from global memory was 32 instructions of 64 cache lines each -- the
// single-block scans took 9.7-14.7 us per sort that way (profiles/r05qc4_kernel_stats.csv).
constexpr int TP_WORDS = TL_BUCKETS + TL_BUCKETS / 32;
__device__ __forceinline__ uint32_t tp_at(uint32_t i) { return i + (i >> 5); }
// v <- the thread's row of g (zero: g is cleared behind the read); ends with sp readable again
__device__ __forceinline__ void rows_in(uint32_t* g, uint32_t* sp, uint32_t (&v)[32], bool zero) {
#pragma unroll 8
    for (int j = 0; j < 32; j++) {
        const uint32_t i = (uint32_t)j * 1024u + threadIdx.x;
        sp[tp_at(i)] = g[i];
        if (zero) g[i] = 0;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 32; k++) v[k] = sp[threadIdx.x * 33u + k];
}
// g <- the threads' rows v (every read of sp done before the call: it is overwritten)
__device__ __forceinline__ void rows_out(uint32_t* g, uint32_t* sp, const uint32_t (&v)[32]) {
#pragma unroll
    for (int k = 0; k < 32; k++) sp[threadIdx.x * 33u + k] = v[k];
    __syncthreads();
#pragma unroll 8
    for (int j = 0; j < 32; j++) {
        const uint32_t i = (uint32_t)j * 1024u + threadIdx.x;
        g[i] = sp[tp_at(i)];
    }
}

// one block: bucket starts (+ the end) and the largest bucket only -- the lookback-free form
// computes its digit bases in the count scans, so it needs none of tl_scan_kernel's marginals
// (whose serial loops made that kernel ~22 us per sort)
// cbase (nullable): the two count scans' column bases, 256 + 128 words -- cbase[d1] = the keys with
// a smaller first-pass digit (d1 = bucket bits 0-7; from d1part, tl_gfold_kernel's four partial
// sums per d1), cbase[256 + d2] = bstart[d2 << 8]
__global__ void __launch_bounds__(1024) tl_bstart_kernel(const uint32_t* __restrict__ hist, uint32_t* __restrict__ bstart,
                                                         uint64_t* __restrict__ maxb, uint32_t* __restrict__ cbase = nullptr,
                                                         const uint32_t* __restrict__ d1part = nullptr) {
    constexpr int PER = TL_BUCKETS / 1024;
    static_assert(PER == 32 && TL_BUCKETS == 128 * 256, "thread t holds buckets t * 32 .. t * 32 + 31");
    __shared__ uint32_t sp[TP_WORDS];
    __shared__ uint32_t wsum[16], wmax[16];
    const int t = threadIdx.x;
    uint4 dp = make_uint4(0, 0, 0, 0);
    if (cbase && t < 256) dp = reinterpret_cast<const uint4*>(d1part)[t];
    uint32_t v[PER], mine = 0, mx = 0;
    rows_in(const_cast<uint32_t*>(hist), sp, v, false);
#pragma unroll
    for (int k = 0; k < PER; k++) {
        mine += v[k];
        mx = v[k] > mx ? v[k] : mx;
    }
    const uint32_t inc = wave_incl_scan_u32(mine);
    mx = wave_max_u32(mx);
    if (lane_id() == 63) wsum[wave_id()] = inc;
    if (lane_id() == 0) wmax[wave_id()] = mx;
    __syncthreads();
    uint32_t run = inc - mine;
    for (int w = 0; w < wave_id(); w++) run += wsum[w];
    const uint32_t bstart_first = run;
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const uint32_t x = v[k];
        v[k] = run;
        run += x;
    }
    rows_out(bstart, sp, v);
    if (t == 1023) bstart[TL_BUCKETS] = run;
    if (t == 0) {
        uint32_t m = 0;
        for (int w = 0; w < 16; w++) m = wmax[w] > m ? wmax[w] : m;
        *maxb = m;
    }
    if (!cbase) return;   // (grid-uniform)
    if ((t & 7) == 0) cbase[256 + (t >> 3)] = bstart_first;   // (bucket t * PER = d2 << 8)
    __syncthreads();   // (wmax read)
    const uint32_t x = dp.x + dp.y + dp.z + dp.w, i1 = wave_incl_scan_u32(x);
    if (t < 256 && lane_id() == 63) wmax[wave_id()] = i1;   // (wmax reused: the first 4 waves' totals)
    __syncthreads();
    if (t < 256) {
        uint32_t r = i1 - x;
        for (int w = 0; w < wave_id(); w++) r += wmax[w];
        cbase[t] = r;
    }
}

// one block: bucket starts (exclusive scan, plus the end), the two global passes' digit bases (the
// histogram's marginals over the low 8 / high 7 bucket bits) and the largest bucket
// (hist is left zeroed for the next sort on this stream: no memset launch per sort)
__global__ void __launch_bounds__(1024) tl_scan_kernel(uint32_t* __restrict__ hist, uint32_t* __restrict__ bstart,
                                                       uint32_t* __restrict__ base1, uint32_t* __restrict__ base2,
                                                       uint64_t* __restrict__ maxb) {
    constexpr int PER = TL_BUCKETS / 1024;
    __shared__ uint32_t h[TP_WORDS];   // the histogram, padded (tp_at)
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t c1[256], c2[128];
    __shared__ uint32_t wmax[16];
    const int t = threadIdx.x;
    uint32_t v[PER], bs[PER], mine = 0, mx = 0;
    rows_in(hist, h, v, true);
#pragma unroll
    for (int k = 0; k < PER; k++) {
        mine += v[k];
        mx = v[k] > mx ? v[k] : mx;
    }
    uint32_t inc = wave_incl_scan_u32(mine);
    mx = wave_max_u32(mx);
    if (lane_id() == 63) wsum[wave_id()] = inc;
    if (lane_id() == 0) wmax[wave_id()] = mx;
    __syncthreads();
    uint32_t run = inc - mine;
    for (int w = 0; w < wave_id(); w++) run += wsum[w];
#pragma unroll
    for (int k = 0; k < PER; k++) {
        bs[k] = run;
        run += v[k];
    }
    if (t == 1023) bstart[TL_BUCKETS] = run;
    if (t == 0) {
        uint32_t m = 0;
        for (int w = 0; w < 16; w++) m = wmax[w] > m ? wmax[w] : m;
        *maxb = m;
    }
    // marginals: pass 1 sorts by the bucket's low 8 bits, pass 2 by its high 7.  All in parallel
    // (the serial form -- a 64-way bank conflict down each row, one thread scanning 512 values --
    // took ~30 us per sort: 212 ms per C4 batch profile, profiles/r04f_c4_kernel_stats.csv)
    __shared__ uint32_t part[4][256];
    {   // c1[d1]: four partial column sums of 32 rows each (consecutive threads, consecutive banks)
        const int d1 = t & 255, q = t >> 8;
        uint32_t a = 0;
#pragma unroll 8
        for (int d2 = q * 32; d2 < q * 32 + 32; d2++) a += h[tp_at(d2 * 256 + d1)];
        part[q][d1] = a;
    }
    // c2[d2]: row d2 = the 256 buckets of threads 8*d2 .. 8*d2 + 7 (their `mine`), one shuffle tree
    uint32_t r8 = mine;
#pragma unroll
    for (int m = 1; m < 8; m <<= 1) r8 += (uint32_t)__shfl_xor((int)r8, m, 64);
    if ((t & 7) == 0) c2[t >> 3] = r8;
    __syncthreads();
    if (t < 256) c1[t] = part[0][t] + part[1][t] + part[2][t] + part[3][t];
    rows_out(bstart, h, bs);   // (every read of h passed the barrier above)
    __syncthreads();
    if (t < 64) {   // one wave scans both: 4 digits of base1 and 2 of base2 per lane
        uint32_t a[4], sa = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            a[k] = c1[t * 4 + k];
            sa += a[k];
        }
        uint32_t run1 = wave_incl_scan_u32(sa) - sa;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            base1[t * 4 + k] = run1;
            run1 += a[k];
        }
        const uint32_t b0 = c2[t * 2], b1 = c2[t * 2 + 1];
        uint32_t run2 = wave_incl_scan_u32(b0 + b1) - b0 - b1;
        base2[t * 2] = run2;
        base2[t * 2 + 1] = run2 + b0;
        const uint32_t tot2 = (uint32_t)__builtin_amdgcn_readlane((int)(run2 + b0 + b1), 63);
        base2[128 + t * 2] = tot2;   // (digits 128..255 of the second pass are empty)
        base2[128 + t * 2 + 1] = tot2;
    }
}

// H = 8 (a small sort's single global pass): 256 buckets, so a 1 KiB histogram instead of the
// 128 KiB one -- for the C4 batch's many small sorts the fixed cost of zeroing, flushing and
// scanning 32768 bins was most of the histogram time
template <typename K>
__global__ void __launch_bounds__(256) tl_hist8_kernel(const K* __restrict__ keys, uint64_t n, Field f, int L,
                                                       uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    for_each_key<8>(keys, n, [&](K k) { atomicAdd(&h[(uint32_t)((((uint64_t)k >> f.lo) & f.fmask) >> L) & 255u], 1u); });
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}

// one block: the 256 bucket starts (+ the end), which are also the pass's digit bases, and the
// largest bucket
// (hist is left zeroed for the next sort on this stream: no memset launch per sort)
__global__ void __launch_bounds__(256) tl_scan8_kernel(uint32_t* __restrict__ hist, uint32_t* __restrict__ bstart,
                                                       uint64_t* __restrict__ maxb) {
    __shared__ uint32_t wsum[4], wmax[4];
    const uint32_t v = hist[threadIdx.x];
    hist[threadIdx.x] = 0;
    const uint32_t inc = wave_incl_scan_u32(v);
    const uint32_t mx = wave_max_u32(v);
    if (lane_id() == 63) wsum[wave_id()] = inc;
    if (lane_id() == 0) wmax[wave_id()] = mx;
    __syncthreads();
    uint32_t ex = inc - v;
    for (int w = 0; w < wave_id(); w++) ex += wsum[w];
    bstart[threadIdx.x] = ex;
    if (threadIdx.x == 255) bstart[256] = ex + v;
    if (threadIdx.x == 0) {
        uint32_t m = 0;
        for (int w = 0; w < 4; w++) m = wmax[w] > m ? wmax[w] : m;
        *maxb = m;
    }
}

// one workgroup per bucket: up to TL_CAP packed words, sorted by the low L bits in LDS.  Each wave
// owns a contiguous slice of jm x 64 words, jm = ceil(m / (waves x 64)): every wave works and the
// work is proportional to the bucket, not to TL_CAP.
// LDS rounds of a local sort: round r sorts field bits [32 + sum(bits[<r]), ... + bits[r])
struct LocalRounds {
    int n;
    int bits[4];
};

// IN == IN_WORD: packed words of a bucket-partitioned array (bstart); IN_KV / IN_KIOTA: ONE
// bucket of single_n (key, rowid) pairs packed on load (a small sort: a single launch)
// NT: threads per bucket -- TL_NT, or 64 (one wave, TL_ITEMS x 64 words) for the many small buckets
// of a two-level sort over a few million keys (32 K buckets of tens to hundreds of words: 512 threads
// and their barriers per bucket were most of the C4 batch's local-sort time)
// UN0: the first round ranks unstably (one LDS atomic per element instead of up to 8 ballots) -- a
// deferred sort's completion, whose consumer (the plan's merge) needs no order among equal keys;
// later rounds stay stable (they must keep the earlier rounds' order)
template <typename K, int IN, int NT = TL_NT, bool UN0 = false>
__global__ void __launch_bounds__(NT) tl_local_kernel(const uint64_t* __restrict__ win, const K* __restrict__ kin,
                                                         const uint32_t* __restrict__ vin, K* __restrict__ kout,
                                                         uint32_t* __restrict__ vout,
                                                         const uint32_t* __restrict__ bstart, uint32_t single_n,
                                                         Field f, LocalRounds lr) {
    constexpr int NW = NT / 64, BINS = 256;
    __shared__ uint64_t stage[NT * TL_ITEMS];
    __shared__ uint32_t whist[NW][BINS];
    __shared__ uint32_t bexcl[BINS];
    __shared__ uint32_t wsum[NW];
    const uint32_t s0 = IN == IN_WORD ? bstart[blockIdx.x] : 0u;
    const uint32_t m = IN == IN_WORD ? bstart[blockIdx.x + 1] - s0 : single_n;
    if (m == 0) return;   // block-uniform
    const int w = wave_id(), l = lane_id();
    const uint64_t lt = lanemask_lt();
    const uint32_t jm = (m + NW * 64 - 1) / (NW * 64);   // <= TL_ITEMS since m <= NT * TL_ITEMS
    const uint32_t wbase = (uint32_t)w * jm * 64;
    uint64_t word[TL_ITEMS];
#pragma unroll
    for (int j = 0; j < TL_ITEMS; j++) {
        const uint32_t i = wbase + (uint32_t)j * 64 + l;
        const bool ok = (uint32_t)j < jm && i < m;
        if (IN == IN_WORD) {
            word[j] = ok ? win[s0 + i] : 0;
        } else {
            const uint64_t k = ok ? (uint64_t)kin[i] : 0;
            const uint32_t v = IN == IN_KV ? (ok ? vin[i] : 0u) : i;
            word[j] = (((k >> f.lo) & f.fmask) << 32) | v;
        }
    }
    int dsh = 32;
    for (int r = 0; r < lr.n; r++) {
        const int bits = lr.bits[r];
        if (r > 0) dsh += lr.bits[r - 1];
        const uint32_t mask = (1u << bits) - 1u;
        for (int i = threadIdx.x; i < NW * BINS; i += NT) (&whist[0][0])[i] = 0;
        __syncthreads();
        uint32_t pos[TL_ITEMS];
#pragma unroll
        for (int j = 0; j < TL_ITEMS; j++) {   // stable rank inside the wave: (j, lane) order
            pos[j] = 0;
            if ((uint32_t)j >= jm) continue;     // wave-uniform
            const uint32_t i = wbase + (uint32_t)j * 64 + l;
            const bool ok = i < m;
            const uint32_t d = (uint32_t)(word[j] >> dsh) & mask;
            if (UN0 && r == 0) {   // (block-uniform)
                pos[j] = ok ? atomicAdd(&whist[w][d], 1u) : 0u;
                continue;
            }
            uint64_t peers = __ballot(ok);
#pragma unroll
            for (int b = 0; b < 8; b++) {
                if (b >= bits) break;
                const bool bit = (d >> b) & 1u;
                const uint64_t mm = __ballot(bit);
                peers &= bit ? mm : ~mm;
            }
            const int leader = peers ? (__ffsll((unsigned long long)peers) - 1) : 0;
            uint32_t old = 0;
            if (ok && l == leader) {
                old = whist[w][d];
                whist[w][d] = old + (uint32_t)__popcll(peers);
            }
            old = (uint32_t)__shfl((int)old, leader, 64);
            pos[j] = old + (uint32_t)__popcll(peers & lt);
        }
        __syncthreads();
        // thread t owns digits t * DPT .. + DPT - 1: totals over the waves, then one exclusive scan
        constexpr int DPT = BINS >= NT ? BINS / NT : 1;
        const bool owner = DPT > 1 || (int)threadIdx.x < BINS;
        uint32_t tq[DPT], tot = 0;
#pragma unroll
        for (int q = 0; q < DPT; q++) {
            const uint32_t d = threadIdx.x * DPT + q;
            uint32_t t = 0;
            if (owner) {
#pragma unroll
                for (int ww = 0; ww < NW; ww++) {
                    const uint32_t c = whist[ww][d];
                    whist[ww][d] = t;
                    t += c;
                }
            }
            tq[q] = t;
            tot += t;
        }
        const uint32_t inc = wave_incl_scan_u32(tot);
        if (l == 63) wsum[w] = inc;
        __syncthreads();
        if (owner) {
            uint32_t ex = inc - tot;
            for (int ww = 0; ww < w; ww++) ex += wsum[ww];
#pragma unroll
            for (int q = 0; q < DPT; q++) {
                bexcl[threadIdx.x * DPT + q] = ex;
                ex += tq[q];
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < TL_ITEMS; j++) {
            const uint32_t i = wbase + (uint32_t)j * 64 + l;
            if ((uint32_t)j < jm && i < m) {
                const uint32_t d = (uint32_t)(word[j] >> dsh) & mask;
                stage[bexcl[d] + whist[w][d] + pos[j]] = word[j];
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < TL_ITEMS; j++) {
            const uint32_t i = wbase + (uint32_t)j * 64 + l;
            word[j] = ((uint32_t)j < jm && i < m) ? stage[i] : 0;
        }
        __syncthreads();   // every read of stage before the next round writes it
    }
#pragma unroll
    for (int j = 0; j < TL_ITEMS; j++) {
        const uint32_t i = wbase + (uint32_t)j * 64 + l;
        if ((uint32_t)j < jm && i < m) {
            kout[s0 + i] = (K)(f.kconst | ((word[j] >> 32) << f.lo));
            vout[s0 + i] = (uint32_t)word[j];
        }
    }
}

// ---- lookback-free global passes of the two-level sort ---------------------------------------
// The histogram pass reads every key anyway, so it also leaves
//   * tcnt[t][d1]   -- per first-pass tile t (RTILE keys) the count of each first-pass digit d1
//                      (the bucket's low 8 bits), and
//   * gcnt[s][d2]   -- per segment s = d1 * G + g (group g = TL_TPG consecutive tiles) the count
//                      of each second-pass digit d2 (the bucket's high 7 bits) among group g's
//                      keys with digit d1.
// Column-wise exclusive scans (column_scan) turn both into global output offsets.  Pass 1 places
// tile t's keys of digit d1 from tcnt[t][d1] on -- no ticket, no status words, no lookback.
// After pass 1 (stable) group g's keys with digit d1 form ONE contiguous run, segment s, which
// starts at tcnt[g * TL_TPG][d1]; pass 2 gives every segment a workgroup that places its keys of
// digit d2 from gcnt[s][d2] on -- again without a lookback.  Segments average RTILE keys
// (TL_TPG tiles x RTILE keys / 256 digits), and a larger one is walked in sub-tiles.
#ifndef QE_TL_TPG
#define QE_TL_TPG 256
#endif
constexpr uint32_t TL_TPG = QE_TL_TPG;   // first-pass tiles per group
static_assert(RTILE == 8192, "tl_hist_tiles_kernel counts 8192-key first-pass tiles (1024 threads x 8)");

// The end of a histogram block: its group's 32 K bucket counts stored PLAINLY, each of a group's Q
// blocks into its own slice gout + q * nseg * 128 (gcnt's layout), folded by tl_gfold_kernel.  Round
// 3 added them into gcnt with device-scope atomics: those execute at the memory side, one 256-B wave
// instruction per ~50 ns per CU (MI355X_MICROARCH "Global float atomics") = ~25 us for a block's
// 128 KiB, every block at once at the end of the pass, and gcnt needed a memset first.
__device__ inline void tl_store_counts(const uint32_t* h, uint32_t g, uint32_t q, uint32_t G, uint32_t* gout) {
    uint32_t* o = gout + (uint64_t)q * 256u * G * 128u;
    for (uint32_t i = threadIdx.x * 4u; i < TL_BUCKETS; i += blockDim.x * 4u)   // 16-B stores, 512-B runs
        *reinterpret_cast<uint4*>(o + ((uint64_t)(i >> 7) * G + g) * 128u + (i & 127u)) =
            *reinterpret_cast<const uint4*>(h + i);
}

template <typename K>
__global__ void __launch_bounds__(1024) tl_hist_tiles_kernel(const K* __restrict__ keys, uint64_t n, Field f, int L,
                                                             uint32_t nt, uint32_t G, uint32_t Q,
                                                             uint32_t* __restrict__ tcnt, uint32_t* __restrict__ gout) {
    __shared__ alignas(16) uint32_t h[TL_BUCKETS];   // index d1 * 128 + d2: 128 KiB, one block per CU
    __shared__ uint32_t th[2][256];      // the tile's d1 counts, double-buffered: one barrier per tile
    for (int i = threadIdx.x; i < TL_BUCKETS; i += 1024) h[i] = 0;
    if (threadIdx.x < 512) (&th[0][0])[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t g = blockIdx.x / Q, q = blockIdx.x % Q;   // Q blocks share group g's tiles
    const uint32_t t_end = (g + 1) * TL_TPG < nt ? (g + 1) * TL_TPG : nt;
    // (a tile's counts do not depend on which thread counts which key: u32 keys are loaded two per
    // 8-B load, so a wave instruction still moves 512 contiguous bytes)
    // Every load unconditional, all of a tile's in flight at once: guarded loads (`i < n ? ...`)
    // compiled to a branch and a vmcnt(0) wait per load -- 12 of the 16 loads of a tile served one
    // after another (round 3: 0.20 ms per 1e8 u32 keys).  A full tile takes 8-B loads of two u32
    // keys; the last, partial tile clamps its indices and masks the surplus.
    // The next tile's keys are loaded before this tile's atomics (two register buffers, the loop
    // unrolled by two so neither is copied): one block per CU has no other block to hide the load
    // round trip behind its atomics and barrier (round 4: load -> wait -> atomics -> barrier).
    // Every load is a buffer load over the tile's keys (those past n read 0 and are masked): no
    // branch between a full and a partial tile, whose register merge made the compiler wait for
    // the loads right where they were issued.  A u32 tile takes 8-B loads of two keys.
    // (live = false: a tile past the group -- no keys, the loads return 0 -- so the next tile's
    // load is unconditional too; a guarded one merged registers and waited the same way)
    auto load = [&](uint32_t t, uint64_t (&k)[8], bool live) -> uint32_t {   // -> the valid-key mask
        const uint64_t base = live ? (uint64_t)t * RTILE : 0u;
        const uint32_t tc = !live ? 0u : (uint32_t)((n - base) < (uint64_t)RTILE ? (n - base) : (uint64_t)RTILE);
        uint32_t vm = 0;
        if constexpr (sizeof(K) == 4) {
            const auto r = buf_rsrc(keys + base, (tc * 4u + 7u) & ~7u);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t e = 2u * ((uint32_t)j * 1024u + threadIdx.x);
                const uint2 v = buf_load_u2(r, e * 4u, 0u);
                k[2 * j] = v.x;
                k[2 * j + 1] = v.y;
                vm |= (e < tc ? 1u : 0u) << (2 * j) | (e + 1u < tc ? 1u : 0u) << (2 * j + 1);
            }
        } else {
            const auto r = buf_rsrc(keys + base, tc * 8u);
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t e = (uint32_t)j * 1024u + threadIdx.x;
                const uint2 v = buf_load_u2(r, e * 8u, 0u);
                k[j] = (uint64_t)v.y << 32 | v.x;
                vm |= (e < tc ? 1u : 0u) << j;
            }
        }
        return vm;
    };
    const uint32_t t0 = g * TL_TPG + q;
    uint32_t prev = 0, par = 0;
    // count tile t (keys k, mask vm): flush the previous tile's d1 counts first (its barrier passed)
    auto count = [&](uint32_t t, const uint64_t (&k)[8], uint32_t vm) {
        if (t != t0 && threadIdx.x < 256) {
            tcnt[(uint64_t)prev * 256 + threadIdx.x] = th[par ^ 1u][threadIdx.x];
            th[par ^ 1u][threadIdx.x] = 0;
        }
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if ((vm >> j) & 1u) {
                const uint32_t b = (uint32_t)((((k[j] >> f.lo) & f.fmask) >> L) & (TL_BUCKETS - 1));
                atomicAdd(&h[((b & 255u) << 7) | (b >> 8)], 1u);
                atomicAdd(&th[par][b & 255u], 1u);
            }
        }
        __syncthreads();
        prev = t;
        par ^= 1u;
    };
    uint64_t ka[8], kb[8];
    uint32_t va = load(t0, ka, t0 < t_end), vb;
    for (uint32_t t = t0; t < t_end; t += 2 * Q) {   // (block-uniform trip count)
        vb = load(t + Q, kb, t + Q < t_end);
        count(t, ka, va);
        if (t + Q >= t_end) break;
        va = load(t + 2 * Q, ka, t + 2 * Q < t_end);
        count(t + Q, kb, vb);
    }
    if (g * TL_TPG + q < t_end && threadIdx.x < 256) tcnt[(uint64_t)prev * 256 + threadIdx.x] = th[par ^ 1u][threadIdx.x];
    __syncthreads();
    tl_store_counts(h, g, q, G, gout);
}

// tl_hist_tiles_kernel fused into the gather that produces the keys: keys = col[rows] in list
// order, and the same per-tile / per-segment counts (one pass instead of a gather + a re-read).
// DIRECT: keys = rows[i] widened -- a list of carried key values (no gather).  col32: the column's
// u32 copy (Relation::cols32), read instead when given
template <bool DIRECT = false>
__global__ void __launch_bounds__(1024) tl_gather_hist_kernel(const uint64_t* __restrict__ col,
                                                              const uint32_t* __restrict__ rows, uint64_t n,
                                                              uint64_t* __restrict__ keys, Field f, int L, uint32_t nt,
                                                              uint32_t G, uint32_t Q, uint32_t* __restrict__ tcnt,
                                                              uint32_t* __restrict__ gout,
                                                              const uint32_t* __restrict__ col32 = nullptr,
                                                              uint32_t* __restrict__ k32out = nullptr) {
    __shared__ alignas(16) uint32_t h[TL_BUCKETS];
    __shared__ uint32_t th[2][256];
    for (int i = threadIdx.x; i < TL_BUCKETS; i += 1024) h[i] = 0;
    if (threadIdx.x < 512) (&th[0][0])[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t g = blockIdx.x / Q, q = blockIdx.x % Q;
    const uint32_t t_end = (g + 1) * TL_TPG < nt ? (g + 1) * TL_TPG : nt;
    uint32_t prev = 0, par = 0;
    // the next tile's rowids are loaded while this tile's gathers are in flight: one sequential
    // round trip less per tile on the critical path (one block per CU: nothing else hides it)
    uint32_t rn[8];
    auto load_rows = [&](uint32_t t) {
        const uint64_t base = (uint64_t)t * RTILE;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint64_t i = base + (uint64_t)j * 1024 + threadIdx.x;
            rn[j] = i < n ? rows[i] : 0u;
        }
    };
    if (g * TL_TPG + q < t_end) load_rows(g * TL_TPG + q);
    for (uint32_t t = g * TL_TPG + q; t < t_end; t += Q, par ^= 1u) {
        const uint64_t base = (uint64_t)t * RTILE;
        uint32_t r[8];
        uint64_t k[8];
#pragma unroll
        for (int j = 0; j < 8; j++) r[j] = rn[j];
#pragma unroll
        for (int j = 0; j < 8; j++) {   // 8 random gathers in flight per thread
            const uint64_t i = base + (uint64_t)j * 1024 + threadIdx.x;
            k[j] = i < n ? (DIRECT ? (uint64_t)r[j] : col32 ? (uint64_t)col32[r[j]] : col[r[j]]) : 0;
        }
        if (t + Q < t_end) load_rows(t + Q);
        if (t != g * TL_TPG + q && threadIdx.x < 256) {
            tcnt[(uint64_t)prev * 256 + threadIdx.x] = th[par ^ 1u][threadIdx.x];
            th[par ^ 1u][threadIdx.x] = 0;
        }
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint64_t i = base + (uint64_t)j * 1024 + threadIdx.x;
            if (i < n) {
                if (k32out) {   // (grid-uniform: keys below 2^32, PreHist::k32)
                    if (k32out != rows) k32out[i] = (uint32_t)k[j];   // (== rows: DIRECT adopts its input)
                }
                else keys[i] = k[j];
                const uint32_t b = (uint32_t)((((k[j] >> f.lo) & f.fmask) >> L) & (TL_BUCKETS - 1));
                atomicAdd(&h[((b & 255u) << 7) | (b >> 8)], 1u);
                atomicAdd(&th[par][b & 255u], 1u);
            }
        }
        __syncthreads();
        prev = t;
    }
    if (g * TL_TPG + q < t_end && threadIdx.x < 256) tcnt[(uint64_t)prev * 256 + threadIdx.x] = th[par ^ 1u][threadIdx.x];
    __syncthreads();
    tl_store_counts(h, g, q, G, gout);
}

// gcnt = the sum of a histogram's Q slices (src != dst), and with `hist` the bucket histogram in
// natural order (bucket = d2 << 8 | d1) from the segment counts.  Block = (d1, 32 d2's) x 8 group
// lanes, G x Q / 8 (~32) independent loads per thread; the lanes' sums meet in LDS.
__global__ void __launch_bounds__(256) tl_gfold_kernel(const uint32_t* __restrict__ src, uint32_t Q, uint32_t G,
                                                       uint32_t* __restrict__ dst, uint32_t* __restrict__ hist,
                                                       uint32_t* __restrict__ d1part = nullptr) {
    __shared__ uint32_t part[8][32];
    const uint32_t d1 = blockIdx.x >> 2, d2 = (blockIdx.x & 3u) * 32u + (threadIdx.x & 31u), gl = threadIdx.x >> 5;
    const uint64_t S = (uint64_t)256u * G * 128u;
    uint32_t acc = 0;
#pragma unroll 2
    for (uint32_t g = gl; g < G; g += 8) {
        const uint64_t o = ((uint64_t)d1 * G + g) * 128u + d2;
        uint32_t s = 0;
#pragma unroll 4
        for (uint32_t q = 0; q < Q; q++) s += src[q * S + o];
        if (dst != src) dst[o] = s;
        acc += s;
    }
    if (!hist) return;   // (grid-uniform)
    part[gl][threadIdx.x & 31u] = acc;
    __syncthreads();
    if (threadIdx.x < 32) {
        uint32_t t = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) t += part[j][threadIdx.x];
        hist[(d2 << 8) | d1] = t;
        if (d1part) {   // (grid-uniform) this block's 32 d2's summed: d1part[d1 * 4 + quarter]
#pragma unroll
            for (int m = 16; m >= 1; m >>= 1) t += (uint32_t)__shfl_xor((int)t, m, 32);
            if (threadIdx.x == 0) d1part[blockIdx.x] = t;
        }
    }
}

// Column-wise exclusive scan of a rows x C matrix of u32 counts, in place: m[r][c] <- base[c] +
// sum of m[<r][c], with base[c] = sum of all counts of the columns before c (the digit's global
// start).  Three launches for BOTH matrices of a sort (tile counts, C = 256; segment counts,
// C = 128): chunk sums, a one-block-per-matrix scan of the chunk sums, apply.
#ifndef QE_CS_TOP_REG
#define QE_CS_TOP_REG 1   // (build knob, 0 = round 3's two walks) the chunk-sum scan holds its sums in registers
#endif
constexpr uint32_t CS_CH = 64;
struct CSJob {
    uint32_t* m;
    uint32_t* part;
    uint32_t rows, C, nb;   // nb = chunks of CS_CH rows
    // (the tile-count job of a two-level sort, nullable) the second pass's segment starts:
    // seg[d1 * G + g] = the scanned count of group g's first tile, seg[256 * G] = ntot
    uint32_t* seg;
    uint32_t G, ntot;
};
struct CSJobs {
    CSJob j[2];
};

__device__ __forceinline__ const CSJob& cs_job(const CSJobs& js, uint32_t& blk) {
    if (blk < js.j[0].nb) return js.j[0];
    blk -= js.j[0].nb;
    return js.j[1];
}

__global__ void __launch_bounds__(256) cs_reduce_kernel(CSJobs js) {
    uint32_t blk = blockIdx.x;
    const CSJob& J = cs_job(js, blk);
    const uint32_t c = threadIdx.x, r0 = blk * CS_CH;
    if (c >= J.C) return;
    uint32_t v[CS_CH];
#pragma unroll
    for (uint32_t r = 0; r < CS_CH; r++) v[r] = r0 + r < J.rows ? J.m[(uint64_t)(r0 + r) * J.C + c] : 0u;
    uint32_t s = 0;
#pragma unroll
    for (uint32_t r = 0; r < CS_CH; r++) s += v[r];
    J.part[(uint64_t)blk * J.C + c] = s;
}

__global__ void __launch_bounds__(1024) cs_top_kernel(CSJobs js) {
    const CSJob& J = js.j[blockIdx.x];
    const uint32_t C = J.C, QN = 1024 / C, nb = J.nb;   // thread (c, q) walks chunk sums q*per .. +per
    __shared__ uint32_t tot[1024];
    __shared__ uint32_t colbase[256];
    __shared__ uint32_t wsum[16];
    const uint32_t c = threadIdx.x % C, q = threadIdx.x / C;
    const uint32_t per = (nb + QN - 1) / QN, b0 = q * per < nb ? q * per : nb, b1 = b0 + per < nb ? b0 + per : nb;
    // up to CS_TOP_REG chunk sums per thread are read ONCE, all in flight together (buffer loads,
    // past the matrix read 0), and kept in registers for the rewrite: one global round trip each
    // way instead of a chain of them (~10 us of this one-block kernel per sort)
    constexpr uint32_t CS_TOP_REG = 48;   // (C3: 191 chunks of the tile matrix over 4 row groups)
    const bool reg = QE_CS_TOP_REG && per <= CS_TOP_REG;   // (block-uniform)
    uint32_t v[CS_TOP_REG];
    uint32_t s = 0;
    if (reg) {
        const auto rp = buf_rsrc(J.part, nb * C * 4u);
#pragma unroll
        for (uint32_t i = 0; i < CS_TOP_REG; i++) v[i] = buf_load_u32(rp, ((b0 + i) * C + c) * 4u, 0u);
#pragma unroll
        for (uint32_t i = 0; i < CS_TOP_REG; i++) s += b0 + i < b1 ? v[i] : 0u;
    } else {
#pragma unroll 8
        for (uint32_t b = b0; b < b1; b++) s += J.part[(uint64_t)b * C + c];
    }
    tot[q * C + c] = s;
    __syncthreads();
    uint32_t T = 0;
    if (threadIdx.x < C)
        for (uint32_t k = 0; k < QN; k++) T += tot[k * C + threadIdx.x];
    const uint32_t inc = wave_incl_scan_u32(T);
    if (lane_id() == 63) wsum[wave_id()] = inc;
    __syncthreads();
    if (threadIdx.x < C) {
        uint32_t ex = inc - T;
        for (int w = 0; w < wave_id(); w++) ex += wsum[w];
        colbase[threadIdx.x] = ex;
    }
    __syncthreads();
    uint32_t run = colbase[c];
    for (uint32_t k = 0; k < q; k++) run += tot[k * C + c];
    if (reg) {
#pragma unroll
        for (uint32_t i = 0; i < CS_TOP_REG; i++) {
            if (b0 + i < b1) J.part[(uint64_t)(b0 + i) * C + c] = run;
            run += b0 + i < b1 ? v[i] : 0u;
        }
        return;
    }
#pragma unroll 8
    for (uint32_t b = b0; b < b1; b++) {
        const uint32_t x = J.part[(uint64_t)b * C + c];
        J.part[(uint64_t)b * C + c] = run;
        run += x;
    }
}

__global__ void __launch_bounds__(256) cs_apply_kernel(CSJobs js) {
    uint32_t blk = blockIdx.x;
    const CSJob& J = cs_job(js, blk);
    const uint32_t c = threadIdx.x, r0 = blk * CS_CH;
    if (c >= J.C) return;
    uint32_t run = J.part[(uint64_t)blk * J.C + c];
    uint32_t v[CS_CH];
#pragma unroll
    for (uint32_t r = 0; r < CS_CH; r++) v[r] = r0 + r < J.rows ? J.m[(uint64_t)(r0 + r) * J.C + c] : 0u;
#pragma unroll
    for (uint32_t r = 0; r < CS_CH; r++) {
        if (r0 + r < J.rows) {
            J.m[(uint64_t)(r0 + r) * J.C + c] = run;
            if (J.seg && (r0 + r) % TL_TPG == 0) J.seg[c * J.G + (r0 + r) / TL_TPG] = run;
        }
        run += v[r];
    }
    if (J.seg && blk == 0 && c == 0) J.seg[J.C * J.G] = J.ntot;
}

// The same scans in ONE pass (round 5): the column bases come from the bucket histogram
// (tl_bstart_kernel's cbase), so a chunk needs only the sums of the chunks above it -- a decoupled
// lookback per column (thread c walks column c's status words), as the sort passes do per digit.
// Every count is read once and written once (the three-launch form read them twice: 1.54x the
// algorithmic bytes in PMC, round 4), and the one-block middle launch is gone.
// 1024 threads per block: thread (q, c) owns CS_CH rows of column c (q < 1024 / C row groups), so a
// block covers 256 (C = 256) or 512 (C = 128) rows and the lookback chain is that much shorter
// (~48 links at 1e8 keys instead of ~190: with 64-row blocks the walks, 8 status words a round,
// cost more than the reads -- 17.6 us per sort, and 21 us with 32-word rounds).
__global__ void __launch_bounds__(1024) cs_single_kernel(CSJobs js, const uint32_t* __restrict__ cbase,
                                                         uint64_t* status, uint32_t* ticket, uint32_t epoch) {
    __shared__ uint32_t s_ticket;
    __shared__ uint32_t gsum[1024];   // per (row group, column): the group's sum
    __shared__ uint32_t spre[256];    // per column: the rows above this block
    const uint32_t gb = take_ticket(ticket, &s_ticket);   // predecessors in ticket order are resident
    uint32_t blk = gb;
    const CSJob& J = cs_job(js, blk);
    const uint32_t C = J.C, QN = 1024u / C, c = threadIdx.x % C, q = threadIdx.x / C;
    const uint32_t r0 = (blk * QN + q) * CS_CH;
    const uint32_t nrow = r0 >= J.rows ? 0u : (J.rows - r0 < CS_CH ? J.rows - r0 : CS_CH);
    const auto rm = buf_rsrc(J.m + (uint64_t)(nrow ? r0 : 0u) * C, nrow * C * 4u);
    uint32_t v[CS_CH];
#pragma unroll
    for (uint32_t r = 0; r < CS_CH; r++) v[r] = buf_load_u32(rm, (r * C + c) * 4u, 0u);   // (past the matrix: 0)
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t r = 0; r < CS_CH; r++) sum += v[r];
    gsum[threadIdx.x] = sum;   // (= gsum[q * C + c])
    __syncthreads();
    if (q == 0) {
        uint32_t tot = 0;
        for (uint32_t k = 0; k < QN; k++) tot += gsum[k * C + c];
        // a job's first block publishes its inclusive sum at once and ends every walk of that job
        st_agent(&status[(uint64_t)gb * 256u + c], lb_word(epoch, blk == 0 ? LB_FLAG_INC : LB_FLAG_AGG, tot));
        uint32_t ex = 0;
        if (blk > 0) {
            ex = (uint32_t)lookback_serial(status, epoch, gb, 256u, c);
            st_agent(&status[(uint64_t)gb * 256u + c], lb_word(epoch, LB_FLAG_INC, (uint64_t)ex + tot));
        }
        spre[c] = ex;
    }
    __syncthreads();
    uint32_t run = cbase[(C == 256u ? 0u : 256u) + c] + spre[c];
    for (uint32_t k = 0; k < q; k++) run += gsum[k * C + c];
#pragma unroll
    for (uint32_t r = 0; r < CS_CH; r++) {
        if (r < nrow) {
            J.m[(uint64_t)(r0 + r) * C + c] = run;
            if (J.seg && (r0 + r) % TL_TPG == 0) J.seg[c * J.G + (r0 + r) / TL_TPG] = run;
        }
        run += v[r];
    }
    if (J.seg && gb == 0 && threadIdx.x == 0) J.seg[C * J.G] = J.ntot;
}

// pass 2: one workgroup per segment s = d1 * G + g (the run of group g's keys with first-pass
// digit d1), stable by the second-pass digit d2 = word bits [dsh, dsh + 7); segment bounds from
// the scanned tile counts (off1), digit offsets from the scanned segment counts (off2).  A
// sub-tile of up to TL2_TILE words is ranked in registers, staged in LDS in digit order and
// written as runs; a segment longer than that is walked in sub-tiles with running offsets.
// (K only names the instance after the sort it serves; the kernel moves packed words.)
#ifndef QE_TL2_ITEMS
#define QE_TL2_ITEMS 18
#endif
#ifndef QE_TL2_NT
#define QE_TL2_NT 512
#endif
// (A/B build: QE_P2_LOAD_NT=1 reads the first pass's words and payloads -- their last read --
// with non-temporal loads)
#ifndef QE_P2_LOAD_NT
#define QE_P2_LOAD_NT 0
#endif
constexpr int QE_P2_AUX = QE_P2_LOAD_NT ? 2 : QE_LOAD_AUX;
constexpr int TL2_NT = QE_TL2_NT, TL2_ITEMS = QE_TL2_ITEMS, TL2_TILE = TL2_NT * TL2_ITEMS;   // 9216: mean 8192 + 11 sd
#ifndef QE_TL2_WCH
#define QE_TL2_WCH 6
#endif
constexpr int TL2_WCH = QE_TL2_WCH;   // write-out chunk (slots whose LDS reads are in flight together)
// waves per SIMD the kernel is compiled for: 4 (128 VGPRs) at 18 words per thread, whose 75 KB of
// LDS leave two workgroups per CU anyway; 8 (64 VGPRs) for sub-tiles small enough for four
#ifndef QE_TL2_WPE
#define QE_TL2_WPE (QE_TL2_ITEMS <= 9 ? 8 : 2048 / QE_TL2_NT)
#endif
constexpr int TL2_WPE = QE_TL2_WPE;
static_assert(TL2_ITEMS % TL2_WCH == 0, "whole chunks");
// the strided buffer loads' soffset is not range-checked (qe_device.h): the largest stride a lane
// adds past its buffer -- pass 2's TL2_ITEMS x 512 B, pass 1's R_ITEMS x 512 B (u64 words) or
// R_ITEMS / 4 x 1 KiB (V4) -- must stay inside the allocation's slack
static_assert((size_t)TL2_ITEMS * 512u < DALLOC_SLACK && (size_t)R_ITEMS * 512u < DALLOC_SLACK &&
                  (size_t)(R_ITEMS / 4) * 1024u < DALLOC_SLACK,
              "a strided load's soffset can pass DALLOC_SLACK");

// CARRY: the payloads of pass 1 (xin, in pass-1 order; X64: 64-bit, X32: 32-bit) follow the words
// to xout, staged in the words' LDS slots after the words have left (as in radix_pass_kernel).
// W32: the words are u32 fields (a key-only first pass, OUT_W32): loaded into the high half, stored back as u32
// XS (X64 only): the 64-bit payloads are staged too -- each slot's second-pass digit is kept in a
// byte of a register while its word leaves, the payloads then take the words' slots and leave as
// the same runs (coalesced), instead of every lane storing its payload at its slot's destination.
template <typename K, int CARRY = X_NONE, bool UNSTABLE = false, bool W32 = false, bool XS = false>
__global__ void __launch_bounds__(TL2_NT, TL2_WPE) tl_pass2_kernel(const uint64_t* __restrict__ win, uint64_t* __restrict__ wout,
                                                         uint64_t n, int dsh, const uint32_t* __restrict__ seg,
                                                         const uint32_t* __restrict__ off2, uint32_t G,
                                                         const uint64_t* __restrict__ xin = nullptr,
                                                         uint64_t* __restrict__ xout = nullptr) {
    constexpr int BINS = 128, NW = TL2_NT / 64, WT = 64 * TL2_ITEMS;
    constexpr int NWH = UNSTABLE ? 1 : NW;   // unstable ranks: one block-wide counter row
    __shared__ uint64_t stage[TL2_TILE];
    __shared__ uint32_t whist[NWH][BINS];
    __shared__ uint32_t bexcl[BINS];
    __shared__ uint32_t gofs[BINS];
    __shared__ uint32_t wsum[NW];
    const uint32_t s = xcd_item(blockIdx.x);
    if (s >= 256u * G) return;   // the XCD grid's padding blocks (block-uniform)
    // the segment's bounds from the compact table column_scans wrote (48 KB at 1e8 keys, L2-hot):
    // reading them from the 12.5 MB tile-count matrix put a far dependent load before every word load
#ifdef QE_DIAG_STAMPS
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    if (g_sort_stamp_on && threadIdx.x == 0 && s < STAMP_TILES) g_sort_stamps[(uint64_t)s * STAMP_SLOTS] = t_start;
#endif
    const uint32_t start = seg[s], end = seg[s + 1];
    const int w = wave_id(), l = lane_id();
    const uint64_t lt = lanemask_lt();
    const uint32_t d = threadIdx.x;   // threads 0..127 own one digit each
    uint32_t run = 0;
    const uint32_t* runp = off2 + (uint64_t)s * BINS + (d < BINS ? d : BINS - 1);
    for (uint32_t base = start; base < end; base += TL2_TILE) {   // block-uniform
        const uint32_t m = end - base < (uint32_t)TL2_TILE ? end - base : (uint32_t)TL2_TILE;
        for (int i = threadIdx.x; i < NWH * BINS; i += TL2_NT) (&whist[0][0])[i] = 0;
        uint64_t word[TL2_ITEMS];
        uint32_t pos2[(TL2_ITEMS + 1) / 2];   // ranks < TL2_TILE: two u16 per register
        const int lim = (int)m - (int)((uint32_t)w * WT + l);   // element j valid iff j * 64 < lim
        // every load unconditional, all 18 in flight at once, through a buffer descriptor over the
        // sub-tile: one 32-bit lane offset + a constant per element (18 64-bit clamped addresses
        // held 36 VGPRs and made the kernel spill; the stride in soffset: no VGPR per element).
        // Elements past the segment are masked by `lim`; the strided reads stay inside the
        // dalloc block's slack (win and xin are always dalloc'd: DALLOC_SLACK > 18 x 512 B)
        const uint32_t o0 = (uint32_t)w * WT + l;
        {
            const auto rw = W32 ? buf_rsrc(reinterpret_cast<const uint32_t*>(win) + base, m * 4u) : buf_rsrc(win + base, m * 8u);
#pragma unroll
            for (int j = 0; j < TL2_ITEMS; j++) {
                if constexpr (W32) word[j] = (uint64_t)buf_load_u32<QE_P2_AUX>(rw, o0 * 4u, (uint32_t)j * 256u) << 32;
                else {
                    const uint2 v = buf_load_u2<QE_P2_AUX>(rw, o0 * 8u, (uint32_t)j * 512u);
                    word[j] = (uint64_t)v.y << 32 | v.x;
                }
            }
        }
        if (base == start) run = *runp;   // the digit offsets, behind the words (clamped: no branch)
        __syncthreads();   // whist zeroed
        if (base == start) QE_SORT_STAMP(s, 1);
#pragma unroll
        for (int j = 0; j < TL2_ITEMS; j++) {   // stable rank inside the wave: (j, lane) order
            const bool ok = j * 64 < lim;
            const uint32_t dd = (uint32_t)(word[j] >> dsh) & (BINS - 1);
            uint32_t r;
            if constexpr (UNSTABLE) {
                r = ok ? atomicAdd(&whist[0][dd], 1u) : 0u;
            } else {
                uint64_t peers = __ballot(ok);
#pragma unroll
                for (int b = 0; b < 7; b++) {
                    const bool bit = (dd >> b) & 1u;
                    const uint64_t mm = __ballot(bit);
                    peers &= bit ? mm : ~mm;
                }
                const int leader = peers ? (__ffsll((unsigned long long)peers) - 1) : 0;
                uint32_t old = 0;
                if (ok && l == leader) {
                    old = whist[w][dd];
                    whist[w][dd] = old + (uint32_t)__popcll(peers);
                }
                old = (uint32_t)__shfl((int)old, leader, 64);
                r = old + (uint32_t)__popcll(peers & lt);
            }
            if (j & 1) pos2[j >> 1] |= r << 16;
            else pos2[j >> 1] = r;
            if (j % TL2_WCH == TL2_WCH - 1) __builtin_amdgcn_sched_barrier(0);   // a chunk's atomics in flight, not 18
        }
        __syncthreads();
        if (base == start) QE_SORT_STAMP(s, 2);
        uint32_t tot = 0;
        if (d < BINS) {
#pragma unroll
            for (int ww = 0; ww < NWH; ww++) {
                const uint32_t cc = whist[ww][d];
                whist[ww][d] = tot;
                tot += cc;
            }
        }
        const uint32_t inc = wave_incl_scan_u32<UNSTABLE>(tot);
        if (l == 63) wsum[w] = inc;
        __syncthreads();
        if (d < BINS) {
            uint32_t ex = inc - tot;
            for (int ww = 0; ww < w; ww++) ex += wsum[ww];
            bexcl[d] = ex;
            gofs[d] = run - ex;
            run += tot;
        }
        __syncthreads();
        if (base == start) QE_SORT_STAMP(s, 3);
        // staged in chunks: a chunk's offset reads all issued before its stores (branch-free up to
        // the store), the next chunk's held back (sched_barrier) so registers stay within budget
#pragma unroll
        for (int j0 = 0; j0 < TL2_ITEMS; j0 += TL2_WCH) {
            uint32_t sl[TL2_WCH];
#pragma unroll
            for (int q = 0; q < TL2_WCH; q++) {
                const int j = j0 + q;
                const uint32_t dd = (uint32_t)(word[j] >> dsh) & (BINS - 1);
                // (unstable ranks: the wave row is all zeros after the scan -- one table read)
                sl[q] = bexcl[dd] + (UNSTABLE ? 0u : whist[w][dd]) + ((pos2[j >> 1] >> (16 * (j & 1))) & 0xFFFFu);
            }
#pragma unroll
            for (int q = 0; q < TL2_WCH; q++) {
                const int j = j0 + q;
                if (j * 64 < lim) {
                    stage[sl[q]] = word[j];
                    if constexpr (CARRY != X_NONE)   // pos2 becomes the slot (< TL2_TILE: still 16 bits)
                        pos2[j >> 1] = (j & 1) ? ((pos2[j >> 1] & 0xFFFFu) | (sl[q] << 16)) : ((pos2[j >> 1] & 0xFFFF0000u) | sl[q]);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        // the payloads load into the words' registers (a 32-bit one into registers of its own),
        // in flight during the write-out
        uint32_t xw[CARRY == X32 ? TL2_ITEMS : 1];
        if constexpr (CARRY != X_NONE) {
            const auto rx = CARRY == X64 ? buf_rsrc(xin + base, m * 8u)
                                         : buf_rsrc(reinterpret_cast<const uint32_t*>(xin) + base, m * 4u);
#pragma unroll
            for (int j = 0; j < TL2_ITEMS; j++) {
                if constexpr (CARRY == X64) {
                    const uint2 v = buf_load_u2<QE_P2_AUX>(rx, o0 * 8u, (uint32_t)j * 512u);
                    word[j] = (uint64_t)v.y << 32 | v.x;
                } else {
                    xw[j] = buf_load_u32<QE_P2_AUX>(rx, o0 * 4u, (uint32_t)j * 256u);
                }
            }
        }
        __syncthreads();
        if (base == start) QE_SORT_STAMP(s, 4);
        if constexpr (CARRY == X64 && XS) {
            uint32_t dg[(TL2_ITEMS + 3) / 4];   // slot k's digit in byte k % 4 of dg[k / 4]
#pragma unroll
            for (int k = 0; k < TL2_ITEMS; k++) {
                const uint32_t i = (uint32_t)k * TL2_NT + threadIdx.x;
                const uint64_t wd = stage[i];   // (a slot past m: a stale word, not stored)
                const uint32_t dd = i < m ? (uint32_t)(wd >> dsh) & (BINS - 1) : 0u;
#ifdef QE_DIAG_SORT_LINEAR
                const uint32_t p = base + i;
#else
                const uint32_t p = gofs[dd] + i;
#endif
                QE_STS2(i < m && (uint64_t)p < n, &wout[p], &g_store_sink[l], wd);
                if (k & 3) dg[k >> 2] |= dd << (8 * (k & 3));
                else dg[k >> 2] = dd;
                if (k % 6 == 5) __builtin_amdgcn_sched_barrier(0);   // six slots' LDS reads in flight, not 18
            }
            __syncthreads();   // every word is out of the stage
#pragma unroll
            for (int j = 0; j < TL2_ITEMS; j++)
                if (j * 64 < lim) stage[(pos2[j >> 1] >> (16 * (j & 1))) & 0xFFFFu] = word[j];
            __syncthreads();
#pragma unroll
            for (int k = 0; k < TL2_ITEMS; k++) {
                const uint32_t i = (uint32_t)k * TL2_NT + threadIdx.x;
                const uint32_t p = gofs[(dg[k >> 2] >> (8 * (k & 3))) & 0xFFu] + i;
                QE_STS2(i < m && (uint64_t)p < n, &xout[p], &g_store_sink[l], stage[i]);
                if (k % 6 == 5) __builtin_amdgcn_sched_barrier(0);
            }
        } else if constexpr (CARRY != X_NONE) {
            // the payloads: each slot's destination is read back from its word before the slot
            // is reused (one u32 per slot in the LDS word itself: high half = destination).
            // Write-outs go in chunks of TL2_WCH slots whose LDS reads are all issued before the
            // first store (branch-free up to the store: one LDS round trip per chunk, not per slot)
#pragma unroll
            for (int k0 = 0; k0 < TL2_ITEMS; k0 += TL2_WCH) {
                uint64_t wd[TL2_WCH];
                uint32_t p[TL2_WCH];
#pragma unroll
                for (int q = 0; q < TL2_WCH; q++) wd[q] = stage[(uint32_t)(k0 + q) * TL2_NT + threadIdx.x];
#pragma unroll
                for (int q = 0; q < TL2_WCH; q++)
#ifdef QE_DIAG_SORT_LINEAR   // ablation only: contiguous output instead of the digit scatter
                    p[q] = base + (uint32_t)(k0 + q) * TL2_NT + threadIdx.x;
#else
                    p[q] = gofs[(uint32_t)(wd[q] >> dsh) & (BINS - 1)] + (uint32_t)(k0 + q) * TL2_NT + threadIdx.x;
#endif
#pragma unroll
                for (int q = 0; q < TL2_WCH; q++) {
                    const uint32_t i = (uint32_t)(k0 + q) * TL2_NT + threadIdx.x;
                    const bool ok = i < m && (uint64_t)p[q] < n;
                    QE_STS2(ok, &wout[p[q]], &g_store_sink[l], wd[q]);   // (every store issued: counted waits)
                    if (i < m) reinterpret_cast<uint32_t*>(stage)[2 * i] = p[q];   // slot i now holds its destination
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            __syncthreads();
            if (base == start) QE_SORT_STAMP(s, 5);
            if constexpr (CARRY == X64) {
#pragma unroll
                for (int j = 0; j < TL2_ITEMS; j++) {   // payload j goes straight to its slot's destination
                    const uint32_t sl = (pos2[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
                    const uint32_t dst = reinterpret_cast<const uint32_t*>(stage)[2 * sl];
                    QE_STS2(j * 64 < lim && (uint64_t)dst < n, &xout[dst], &g_store_sink[l], word[j]);
                }
            } else {
                // a 32-bit payload joins its destination in the slot's other half, and the slots
                // then leave in order: the payloads are written as runs, like the words
                uint32_t* st32 = reinterpret_cast<uint32_t*>(stage);
#pragma unroll
                for (int j = 0; j < TL2_ITEMS; j++)
                    if (j * 64 < lim) st32[2 * ((pos2[j >> 1] >> (16 * (j & 1))) & 0xFFFFu) + 1] = xw[j];
                __syncthreads();
                uint32_t* xo = reinterpret_cast<uint32_t*>(xout);
#pragma unroll
                for (int k0 = 0; k0 < TL2_ITEMS; k0 += TL2_WCH) {
                    uint2 dv[TL2_WCH];
#pragma unroll
                    for (int q = 0; q < TL2_WCH; q++)
                        dv[q] = reinterpret_cast<const uint2*>(stage)[(uint32_t)(k0 + q) * TL2_NT + threadIdx.x];
#pragma unroll
                    for (int q = 0; q < TL2_WCH; q++)
                        QE_STS2((uint32_t)(k0 + q) * TL2_NT + threadIdx.x < m && (uint64_t)dv[q].x < n, &xo[dv[q].x], reinterpret_cast<uint32_t*>(&g_store_sink[l]), dv[q].y);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        } else {
#pragma unroll
            for (int k0 = 0; k0 < TL2_ITEMS; k0 += TL2_WCH) {
                uint64_t wd[TL2_WCH];
                uint32_t p[TL2_WCH];
#pragma unroll
                for (int q = 0; q < TL2_WCH; q++) wd[q] = stage[(uint32_t)(k0 + q) * TL2_NT + threadIdx.x];
#pragma unroll
                for (int q = 0; q < TL2_WCH; q++)
#ifdef QE_DIAG_SORT_LINEAR   // ablation only: contiguous output instead of the digit scatter
                    p[q] = base + (uint32_t)(k0 + q) * TL2_NT + threadIdx.x;
#else
                    p[q] = gofs[(uint32_t)(wd[q] >> dsh) & (BINS - 1)] + (uint32_t)(k0 + q) * TL2_NT + threadIdx.x;
#endif
#pragma unroll
                for (int q = 0; q < TL2_WCH; q++) {
                    const uint32_t i = (uint32_t)(k0 + q) * TL2_NT + threadIdx.x;
                    const bool ok = i < m && (uint64_t)p[q] < n;   // (p < n: never false with consistent offsets)
                    if constexpr (W32)
                        QE_STS2(ok, &reinterpret_cast<uint32_t*>(wout)[p[q]], reinterpret_cast<uint32_t*>(&g_store_sink[l]), (uint32_t)(wd[q] >> 32));
                    else QE_STS2(ok, &wout[p[q]], &g_store_sink[l], wd[q]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        __syncthreads();   // stage / whist / gofs are rewritten by the next sub-tile
        if (base == start) QE_SORT_STAMP(s, 6);
    }
}

// the staged 64-bit payload form of pass 2 (XS); QE_X64_STAGE=0 (A/B knob) keeps the per-lane stores
static bool x64_staged() {
    static const bool on = !(getenv("QE_X64_STAGE") && getenv("QE_X64_STAGE")[0] == '0');
    return on;
}

// ---- bucket join (the partitioned plan's join: pairs in no particular order) ----------------
// Both join sides went through the two global passes of the two-level sort with the same bucket
// geometry, so equal keys share a bucket and bucket b of R joins bucket b of S only -- and inside
// a bucket a key is its L low field bits (L <= HJ_DBITS): a dense domain.  One workgroup per
// bucket (in order, by ticket): R's rowids are grouped by key value with an LDS counting sort
// (histogram, scan, scatter -- the runs need no order inside), every S row finds its R run by
// one LDS read of the run bounds, a (row-group, wave) scan gives the offsets inside the bucket and
// ONE atomic reserves the bucket's output slice (no order between buckets is needed: no lookback
// chain through 32 K buckets), and consecutive lanes write consecutive pairs.  This replaces, for a join whose
// pairs need no order, the per-bucket LDS sorts of both sides (12 B/row written and read back)
// and the merge's searches: words in (8 B/row), pairs out (8 B/pair).  LDS: run bounds (4 B per
// key value of the bucket) + R rowids (4 B per row) -- four workgroups per CU at L = 12.
#ifndef QE_HJ_NT
#define QE_HJ_NT 1024
#endif
constexpr int HJ_NT = QE_HJ_NT, HJ_NW = HJ_NT / 64;   // 1024: 53 VGPRs, two blocks = 32 waves per CU
constexpr int HJ_I = (TL_CAP + HJ_NT - 1) / HJ_NT;   // rows per thread per side
constexpr int HJ_DBITS = 13;                          // largest in-bucket key domain (2^13 values)
static_assert(HJ_I * HJ_NW <= 128, "the (row-group, wave) table is scanned by one wave, two entries per lane");

__device__ __forceinline__ uint32_t fld(uint64_t w) { return (uint32_t)(w >> 32); }   // the key field

// CARRY: S's rows carry a 64-bit payload (xS, in S's word order): its low half goes to outX0 and
// its high half to outX1 (nullable) beside every pair
template <int DBITS, bool CARRY = false>
__global__ void __launch_bounds__(HJ_NT) __attribute__((amdgpu_waves_per_eu(8))) tl_hjoin_kernel(const uint64_t* __restrict__ wR, const uint32_t* __restrict__ bsR,
                                                         const uint64_t* __restrict__ wS, const uint32_t* __restrict__ bsS,
                                                         int L, uint32_t* __restrict__ outR, uint32_t* __restrict__ outS,
                                                         uint64_t cap, uint64_t* total_out,
                                                         const uint64_t* __restrict__ xS = nullptr,
                                                         uint32_t* __restrict__ outX0 = nullptr,
                                                         uint32_t* __restrict__ outX1 = nullptr) {
    __shared__ uint32_t bnd[1 << DBITS];   // per key value: count, then run start, then run end
    __shared__ uint32_t rr[TL_CAP];        // R rowids grouped by key value
    __shared__ uint32_t tab[HJ_I * HJ_NW];
    __shared__ uint32_t wsum[HJ_NW];
    __shared__ uint64_t s_excl;
    __shared__ uint32_t s_total;
#ifdef QE_DIAG_STAMPS
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
    const uint32_t b = blockIdx.x;   // (XCD-contiguous buckets measured slower: 2.23 -> 2.35 ms per C3 query)
#ifdef QE_DIAG_STAMPS
    if (threadIdx.x == 0 && b < STAMP_TILES) g_hj_stamps[(uint64_t)b * STAMP_SLOTS] = t_start;
#endif
    const uint32_t r0 = bsR[b], mR = bsR[b + 1] - r0, s0 = bsS[b], mS = bsS[b + 1] - s0;
    if (mR > (uint32_t)TL_CAP || mS > (uint32_t)TL_CAP) {   // beyond LDS (the sorts were not checked): flag it
        if (threadIdx.x == 0) atomicOr(reinterpret_cast<unsigned long long*>(total_out + 1), 1ull);
        return;
    }
    const uint32_t D = 1u << L, dmask = D - 1u;
    const int w = wave_id(), l = lane_id();
    const uint64_t* __restrict__ bR = wR + r0;
    const uint64_t* __restrict__ bS = wS + s0;
    // every load of the bucket in flight at once: R's words, S's words, S's payloads (issuing S's
    // after R's scatter and the payloads after the slice atomic left them on the critical path:
    // C3 bucket joins 2.23 -> 2.10 ms, same box)
    uint64_t wr[HJ_I];
#pragma unroll
    for (int j = 0; j < HJ_I; j++) {
        const uint32_t i = (uint32_t)j * HJ_NT + threadIdx.x;
        wr[j] = i < mR ? bR[i] : 0;
    }
    uint64_t ws[HJ_I];
#pragma unroll
    for (int j = 0; j < HJ_I; j++) {
        const uint32_t i = (uint32_t)j * HJ_NT + threadIdx.x;
        ws[j] = i < mS ? bS[i] : 0;
    }
    uint64_t xv[CARRY ? HJ_I : 1];      // S's payloads
    if constexpr (CARRY) {
#pragma unroll
        for (int j = 0; j < HJ_I; j++) {
            const uint32_t i = (uint32_t)j * HJ_NT + threadIdx.x;
            xv[j] = i < mS ? xS[s0 + i] : 0ull;
        }
    }
    for (uint32_t v = threadIdx.x; v < D; v += HJ_NT) bnd[v] = 0;
    __syncthreads();
    QE_STAMP(g_hj_stamps, b, 1);
#pragma unroll
    for (int j = 0; j < HJ_I; j++)
        if ((uint32_t)j * HJ_NT + threadIdx.x < mR) atomicAdd(&bnd[fld(wr[j]) & dmask], 1u);
    __syncthreads();
    QE_STAMP(g_hj_stamps, b, 2);
    {   // exclusive scan of the D counts: PER consecutive values per thread, then a block scan
        const uint32_t PER = (D + HJ_NT - 1) / HJ_NT, v0 = threadIdx.x * PER;
        uint32_t sum = 0;
        for (uint32_t k = 0; k < PER && v0 + k < D; k++) sum += bnd[v0 + k];
        const uint32_t inc = wave_incl_scan_u32(sum);
        if (l == 63) wsum[w] = inc;
        __syncthreads();
        uint32_t run = inc - sum;
        for (int ww = 0; ww < w; ww++) run += wsum[ww];
        for (uint32_t k = 0; k < PER && v0 + k < D; k++) {
            const uint32_t cnt = bnd[v0 + k];
            bnd[v0 + k] = run;
            run += cnt;
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < HJ_I; j++)   // scatter: afterwards bnd[v] is the END of v's run
        if ((uint32_t)j * HJ_NT + threadIdx.x < mR) rr[atomicAdd(&bnd[fld(wr[j]) & dmask], 1u)] = (uint32_t)wr[j];
    __syncthreads();
    QE_STAMP(g_hj_stamps, b, 3);
    uint32_t pre[HJ_I];   // (the runs are looked up again when writing: fewer live registers)
#pragma unroll
    for (int j = 0; j < HJ_I; j++) {
        uint32_t cnt = 0;
        if ((uint32_t)j * HJ_NT + threadIdx.x < mS) {
            const uint32_t v = fld(ws[j]) & dmask;
            cnt = bnd[v] - (v ? bnd[v - 1] : 0u);
        }
        const uint32_t inc = wave_incl_scan_u32(cnt);
        pre[j] = inc - cnt;
        if (l == 63) tab[j * HJ_NW + w] = inc;
    }
    __syncthreads();
    QE_STAMP(g_hj_stamps, b, 4);
    if (w == 0) {   // (row group, wave) totals in row order -> bucket offsets; bucket total -> lookback
        constexpr uint32_t E = HJ_I * HJ_NW;
        const uint32_t a0 = 2u * l < E ? tab[2 * l] : 0u, a1 = 2u * l + 1 < E ? tab[2 * l + 1] : 0u;
        const uint32_t inc = wave_incl_scan_u32(a0 + a1);
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        if (2u * l < E) tab[2 * l] = inc - a0 - a1;
        if (2u * l + 1 < E) tab[2 * l + 1] = inc - a1;
        if (l == 0) {   // the pairs need no order: a bucket reserves its output slice with one atomic
            s_excl = total ? atomicAdd(reinterpret_cast<unsigned long long*>(total_out), (unsigned long long)total)
                           : 0ull;
            s_total = total;
        }
    }
    __syncthreads();
    QE_STAMP(g_hj_stamps, b, 5);
    const uint64_t gofs = s_excl;
    if (gofs + s_total > cap) return;   // outgrew the buffers: the host re-runs with the exact size
#ifndef QE_HJ_LANE_EMIT
    // wave-cooperative emission: item j's pairs of this wave are one contiguous range; lane l
    // writes pairs q0 + l, q0 + 64 + l, ... -- every store instruction covers 64 consecutive
    // pairs (whole lines), where a per-lane loop over its own row's partners left partial lines
    // (PMC: ~2 GB written per C3 bucket join against ~0.6 GB of pairs).  The pair's S row is the
    // last lane whose exclusive prefix is <= q (found by a 6-step shuffle search).
#pragma unroll
    for (int j = 0; j < HJ_I; j++) {
        const bool live = (uint32_t)j * HJ_NT + threadIdx.x < mS;
        const uint32_t v = live ? fld(ws[j]) & dmask : 0u;
        const uint32_t st = live ? (v ? bnd[v - 1] : 0u) : 0u;
        const uint32_t cnt = live ? bnd[v] - st : 0u;
        const uint32_t pj = pre[j];
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)(pj + cnt), 63);
        const uint64_t ob = gofs + tab[j * HJ_NW + w];
        const uint32_t srow = (uint32_t)ws[j];
        for (uint32_t q0 = 0; q0 < tot; q0 += 64) {   // wave-uniform
            const uint32_t q = q0 + (uint32_t)l;
            int owner = 0;
#pragma unroll
            for (int step = 32; step >= 1; step >>= 1) {
                const int cand = owner + step;
                const uint32_t pc = (uint32_t)__shfl((int)pj, cand < 64 ? cand : 63, 64);
                if (cand < 64 && pc <= q) owner = cand;
            }
            const uint32_t k = q - (uint32_t)__shfl((int)pj, owner, 64);
            const uint32_t so = (uint32_t)__shfl((int)st, owner, 64);
            const uint32_t sr = (uint32_t)__shfl((int)srow, owner, 64);
            uint32_t x0 = 0, x1 = 0;
            if constexpr (CARRY) {
                x0 = (uint32_t)__shfl((int)(uint32_t)xv[j], owner, 64);
                x1 = (uint32_t)__shfl((int)(uint32_t)(xv[j] >> 32), owner, 64);
            }
            if (q < tot) {
                outR[ob + q] = rr[so + k];
                outS[ob + q] = sr;
                if constexpr (CARRY) {
                    outX0[ob + q] = x0;
                    if (outX1) outX1[ob + q] = x1;
                }
            }
        }
    }
    QE_STAMP(g_hj_stamps, b, 6);
    return;
#endif
#pragma unroll
    for (int j = 0; j < HJ_I; j++) {
        if ((uint32_t)j * HJ_NT + threadIdx.x >= mS) continue;
        const uint32_t v = fld(ws[j]) & dmask;
        const uint32_t st = v ? bnd[v - 1] : 0u, cnt = bnd[v] - st;
        const uint64_t o = gofs + tab[j * HJ_NW + w] + pre[j];
        const uint32_t srow = (uint32_t)ws[j];
        uint32_t* __restrict__ pR = outR + o;
        uint32_t* __restrict__ pS = outS + o;
        if constexpr (CARRY) {
            const uint64_t x = xv[j];
            uint32_t* __restrict__ p0 = outX0 + o;
#pragma nounroll
            for (uint32_t k = 0; k < cnt; k++) {
                pR[k] = rr[st + k];
                pS[k] = srow;
                p0[k] = (uint32_t)x;
                if (outX1) outX1[o + k] = (uint32_t)(x >> 32);
            }
            continue;
        }
#pragma nounroll
        for (uint32_t k = 0; k < cnt; k++) {   // fan-out ~1: a plain loop (unrolled, it was 118 VGPRs)
            pR[k] = rr[st + k];
            pS[k] = srow;
        }
    }
}

// The same join with R's rows CHAINED by key value instead of counting-sorted: one LDS exchange per
// R row (head[v] <- i, nxt[i] <- old head) replaces the histogram, the scan of the 2^L counts and
// the scatter -- two barrier-separated phases of the ~10.4 us per bucket (3.1 us scan + scatter,
// profiles/r02_hjoin_stamps.log).  An S row counts its partners by walking its value's chain (mean
// length |R bucket| / 2^L, ~0.75 at C3) and the wave-cooperative emission walks it again to the
// pair's partner.  Output is the same multiset of pairs (in no particular order, as before).
// RX: R's rows carry a 32-bit payload too (xR, in R's word order -- a base relation's next join
// key, sorted along with it): staged in LDS beside the rowids (two blocks per CU are the wave
// limit anyway: 67 KB each fits) and written to outRX with the partner.  (Re-reading R's rowids or
// payloads from L2 at emission instead measured 0.2-0.5 ms slower per C3 query.)
constexpr uint32_t HJ_NONE = 0xFFFFu;
// A lane's k-th partner is k links down its key's chain, so emission costs sum(k) per S row:
// quadratic in a long chain (thousands of equal keys on both sides of one bucket).  A bucket with
// a chain longer than HJ_CHAIN_MAX is flagged like one beyond LDS, and the join takes the sorts +
// merge path (linear in the pairs) instead.
constexpr uint32_t HJ_CHAIN_MAX = 64;
#ifndef QE_HJ_RR_GLOBAL
#define QE_HJ_RR_GLOBAL 0
#endif
#ifndef QE_LB_MAXB_LATE   // (build knob, A/B: 0 reads the lookback-form sort's largest bucket before its passes)
#define QE_LB_MAXB_LATE 1
#endif
#ifndef QE_HJ_SKIP
#define QE_HJ_SKIP 1   // (build knob, A/B: 0 walks and scans every item of every wave)
#endif
static_assert(TL_CAP < HJ_NONE, "chain links are 16-bit row indices");

// S32: S's payload is 32-bit (xS32: one carried binding), outX0 only.
// NT: threads per bucket (HJ_NT; 256 for C4-sized joins measured 2 % slower on the batch's wall
// time -- its bucket joins 99 -> 62 ms of kernel time, but 41 re-runs of overflowing buckets and
// more interference with the other lanes, profiles/r03_c4_hjsmall_ab.log)
// IT: rows per thread per side (NT * IT = the largest bucket side it takes; a larger one is flagged)
template <int DBITS, bool CARRY = false, bool RX = false, bool S32 = false, int NT = HJ_NT, int IT = HJ_I>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT >= 1024 ? 8 : 6)))
tl_hjoin_chain_kernel(const uint64_t* __restrict__ wR, const uint32_t* __restrict__ bsR, const uint64_t* __restrict__ wS,
                      const uint32_t* __restrict__ bsS, int L, uint32_t* __restrict__ outR, uint32_t* __restrict__ outS,
                      uint64_t cap, uint64_t* total_out, const uint64_t* __restrict__ xS = nullptr,
                      uint32_t* __restrict__ outX0 = nullptr, uint32_t* __restrict__ outX1 = nullptr,
                      const uint32_t* __restrict__ xR = nullptr, uint32_t* __restrict__ outRX = nullptr,
                      const uint32_t* __restrict__ xS32 = nullptr) {
    __shared__ uint32_t head[1 << DBITS];   // per key value: the last R row inserted (HJ_NONE: none)
    __shared__ uint16_t nxt[NT * IT];        // per R row: the previous row of its value
#if QE_HJ_RR_GLOBAL
    uint32_t* rr = nullptr;                 // (R's rowids re-read from its words, L2-hot, at emission)
#else
    __shared__ uint32_t rr[NT * IT];         // per R row: its rowid
#endif
    __shared__ uint32_t rx[RX ? NT * IT : 1];  // per R row: its payload
    constexpr int NW = NT / 64;
    __shared__ uint32_t tab[IT * NW];
    __shared__ uint64_t s_excl;
    __shared__ uint32_t s_total, s_long;
    // The bucket's bounds are read before the loop as two 8-B scalar loads with the kernel
    // arguments: the straight-line form compiled to three serialized scalar round trips (bounds,
    // then argument pointers, each behind an lgkmcnt(0) wait) before the first word load -- the
    // loop form issues them together (145 -> 93 waits): bucket_join 1.08 -> 1.01 ms per C3 query
    // (profiles/r05w_*, r05x_*).  A grid below TL_BUCKETS (QE_HJ_PERSIST=1) walks the buckets b,
    // b + gridDim.x, ... with the next bucket's bounds in flight -- measured slower (hj_grid).
    uint32_t nr0 = bsR[blockIdx.x], nrE = bsR[blockIdx.x + 1], ns0 = bsS[blockIdx.x], nsE = bsS[blockIdx.x + 1];
    for (uint32_t b = blockIdx.x; b < (uint32_t)TL_BUCKETS; b += gridDim.x) {   // (block-uniform)
    if (b != blockIdx.x) __syncthreads();   // every LDS read of the previous bucket done
#ifdef QE_DIAG_STAMPS
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && b < STAMP_TILES) g_hj_stamps[(uint64_t)b * STAMP_SLOTS] = t_start;
#endif
    const uint32_t r0 = nr0, mR = nrE - nr0, s0 = ns0, mS = nsE - ns0;
    if (b + gridDim.x < (uint32_t)TL_BUCKETS) {
        const uint32_t bn = b + gridDim.x;
        nr0 = bsR[bn];
        nrE = bsR[bn + 1];
        ns0 = bsS[bn];
        nsE = bsS[bn + 1];
    }
    if (mR > (uint32_t)(NT * IT) || mS > (uint32_t)(NT * IT)) {   // beyond LDS (the sorts were not checked): flag it
        if (threadIdx.x == 0) atomicOr(reinterpret_cast<unsigned long long*>(total_out + 1), 1ull);
        continue;
    }
    const uint32_t D = 1u << L, dmask = D - 1u;
    const int w = wave_id(), l = lane_id();
    uint64_t wr[IT], ws[IT];
#pragma unroll
    for (int j = 0; j < IT; j++) {
        const uint32_t i = (uint32_t)j * NT + threadIdx.x;
        wr[j] = i < mR ? wR[r0 + i] : 0;
    }
#pragma unroll
    for (int j = 0; j < IT; j++) {
        const uint32_t i = (uint32_t)j * NT + threadIdx.x;
        ws[j] = i < mS ? wS[s0 + i] : 0;
    }
    uint64_t xv[CARRY ? IT : 1];
    if constexpr (CARRY) {
#pragma unroll
        for (int j = 0; j < IT; j++) {
            const uint32_t i = (uint32_t)j * NT + threadIdx.x;
            xv[j] = i < mS ? (S32 ? (uint64_t)xS32[s0 + i] : xS[s0 + i]) : 0ull;
        }
    }
    uint32_t xr[RX ? IT : 1];
    if constexpr (RX) {
#pragma unroll
        for (int j = 0; j < IT; j++) {
            const uint32_t i = (uint32_t)j * NT + threadIdx.x;
            xr[j] = i < mR ? xR[r0 + i] : 0u;
        }
    }
    for (uint32_t v = threadIdx.x; v < D; v += NT) head[v] = HJ_NONE;
    if (threadIdx.x == 0) s_long = 0;
    __syncthreads();
    QE_STAMP(g_hj_stamps, b, 1);
#pragma unroll
    for (int j = 0; j < IT; j++) {
        const uint32_t i = (uint32_t)j * NT + threadIdx.x;
        if (i < mR) {
            nxt[i] = (uint16_t)atomicExch(&head[fld(wr[j]) & dmask], i);
            if (!QE_HJ_RR_GLOBAL) rr[i] = (uint32_t)wr[j];
            if constexpr (RX) rx[i] = xr[j];
        }
    }
    __syncthreads();
    QE_STAMP(g_hj_stamps, b, 2);
    uint32_t pre[IT], hd[IT], tot[IT];
#pragma unroll
    for (int j = 0; j < IT; j++) {
        if (QE_HJ_SKIP && (uint32_t)j * NT + (uint32_t)w * 64u >= mS) {   // (wave-uniform) no S row of this item in this
            hd[j] = HJ_NONE;                                  // wave: skip its walk and scan (a C3 bucket
            pre[j] = tot[j] = 0;                              // fills 1.4 of the 5 items)
            if (l == 63) tab[j * NW + w] = 0;
            continue;
        }
        uint32_t cnt = 0, h = HJ_NONE;
        if ((uint32_t)j * NT + threadIdx.x < mS) {
            h = head[fld(ws[j]) & dmask];
            // (linear in the pairs: cnt of them) -- and bounded: the walk stops one link past
            // HJ_CHAIN_MAX whatever nxt[] holds, so no chain (a long one, or a cycle through stale
            // links) can keep a wave here (the looped emission that hung in round 4)
            for (uint32_t p = h; p != HJ_NONE && cnt <= HJ_CHAIN_MAX; p = nxt[p]) cnt++;
            if (cnt > HJ_CHAIN_MAX) s_long = 1;
        }
        hd[j] = h;
        const uint32_t inc = wave_incl_scan_u32(cnt);
        pre[j] = inc - cnt;
        tot[j] = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);   // the item's pairs in this wave
        if (l == 63) tab[j * NW + w] = inc;
    }
    __syncthreads();
    QE_STAMP(g_hj_stamps, b, 3);
    if (s_long) {   // block-uniform: a chain too long to emit by walking (the sorts + merge take the join)
        if (threadIdx.x == 0) atomicOr(reinterpret_cast<unsigned long long*>(total_out + 1), 1ull);
        continue;
    }
    if (w == 0) {   // (row group, wave) totals in row order -> bucket offsets; one atomic per bucket
        constexpr uint32_t E = IT * NW;
        const uint32_t a0 = 2u * l < E ? tab[2 * l] : 0u, a1 = 2u * l + 1 < E ? tab[2 * l + 1] : 0u;
        const uint32_t inc = wave_incl_scan_u32(a0 + a1);
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        if (2u * l < E) tab[2 * l] = inc - a0 - a1;
        if (2u * l + 1 < E) tab[2 * l + 1] = inc - a1;
        if (l == 0) {
            s_excl = total ? atomicAdd(reinterpret_cast<unsigned long long*>(total_out), (unsigned long long)total)
                           : 0ull;
            s_total = total;
        }
    }
    __syncthreads();
    QE_STAMP(g_hj_stamps, b, 4);
    const uint64_t gofs = s_excl;
    if (gofs + s_total > cap) continue;   // outgrew the buffers: the host re-runs with the exact size
#pragma unroll
    for (int j = 0; j < IT; j++) {   // wave-cooperative emission, as tl_hjoin_kernel's
        const uint32_t pj = pre[j], all = tot[j];
        const uint64_t ob = gofs + tab[j * NW + w];
        const uint32_t srow = (uint32_t)ws[j];
        for (uint32_t q0 = 0; q0 < all; q0 += 64) {   // wave-uniform
            const uint32_t q = q0 + (uint32_t)l;
            int owner = 0;
#pragma unroll
            for (int step = 32; step >= 1; step >>= 1) {
                const int cand = owner + step;
                const uint32_t pc = (uint32_t)__shfl((int)pj, cand < 64 ? cand : 63, 64);
                if (cand < 64 && pc <= q) owner = cand;
            }
            const uint32_t k = q - (uint32_t)__shfl((int)pj, owner, 64);
            uint32_t p = (uint32_t)__shfl((int)hd[j], owner, 64);
            const uint32_t sr = (uint32_t)__shfl((int)srow, owner, 64);
            uint32_t x0 = 0, x1 = 0;
            if constexpr (CARRY) {
                x0 = (uint32_t)__shfl((int)(uint32_t)xv[j], owner, 64);
                if constexpr (!S32) x1 = (uint32_t)__shfl((int)(uint32_t)(xv[j] >> 32), owner, 64);
            }
            if (q < all) {
                for (uint32_t s = 0; s < k; s++) p = nxt[p];   // the k-th partner on the chain
                outR[ob + q] = QE_HJ_RR_GLOBAL ? (uint32_t)wR[r0 + p] : rr[p];
                outS[ob + q] = sr;
                if constexpr (RX) outRX[ob + q] = rx[p];
                if constexpr (CARRY) {
                    outX0[ob + q] = x0;
                    if (!S32 && outX1) outX1[ob + q] = x1;
                }
            }
        }
    }
    QE_STAMP(g_hj_stamps, b, 5);
    }
}

// the chain join's grid: one block per bucket, or (QE_HJ_PERSIST=1, A/B knob) two per CU walking
// the buckets with the next bucket's bounds in flight -- bucket_join 1.013 -> 1.081 ms per C3
// query and C4 3845 -> 3690 q/s on one box (profiles/r05w_*): the grid of one block per bucket
// keeps every CU's two slots refilled by the dispatcher as buckets finish, whatever their sizes
static unsigned hj_grid() {
    static const unsigned g = [] {
        const char* s = getenv("QE_HJ_PERSIST");
        return s && s[0] == '1' ? 512u : (unsigned)TL_BUCKETS;
    }();
    return g;
}

static bool hj_chain_on() {
    static bool on = [] {   // tuning knob: QE_HJ_CHAIN=0 keeps the counting-sort bucket join
        const char* s = getenv("QE_HJ_CHAIN");
        return !(s && s[0] == '0');
    }();
    return on;
}

// Non-packable pairs (64-bit keys with > 32 varying bits AND a rowid): key and rowid staged
// separately.  Kept simple: rare in this workload (never in the measured configs).
template <typename K, bool VIN>
__global__ void __launch_bounds__(RB) radix_pass_kv_kernel(const K* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                           K* __restrict__ kout, uint32_t* __restrict__ vout, uint64_t n,
                                                           int shift, uint32_t mask,
                                                           const uint32_t* __restrict__ digit_base, uint64_t* status,
                                                           uint32_t* ticket, uint32_t epoch) {
    constexpr int BINS = 256;
    constexpr int WT = 64 * R_ITEMS;
    __shared__ union {
        K keys[KV_TILE];
        uint32_t vals[KV_TILE];
    } stage;
    __shared__ uint32_t whist[RNW][BINS];
    __shared__ uint32_t bexcl[BINS];
    __shared__ uint32_t gofs[BINS];
    __shared__ uint32_t wsum[RNW];
    __shared__ uint32_t s_ticket;

    const uint32_t tile = take_ticket(ticket, &s_ticket);
    const int w = wave_id(), l = lane_id();
    const uint64_t lt = lanemask_lt();
    for (int i = threadIdx.x; i < RNW * BINS; i += RB) (&whist[0][0])[i] = 0;
    __syncthreads();
    const uint64_t wave_base = (uint64_t)tile * KV_TILE + (uint64_t)w * WT;
    K key[R_ITEMS];
    uint32_t val[R_ITEMS], pos[R_ITEMS];
#pragma unroll
    for (int j = 0; j < R_ITEMS; j++) {
        uint64_t i = wave_base + (uint64_t)j * 64 + l;
        bool ok = i < n;
        key[j] = ok ? kin[i] : (K)0;
        val[j] = VIN ? (ok ? vin[i] : 0u) : (uint32_t)i;
    }
#pragma unroll
    for (int j = 0; j < R_ITEMS; j++) {
        uint64_t i = wave_base + (uint64_t)j * 64 + l;
        bool ok = i < n;
        uint32_t d = (uint32_t)((uint64_t)key[j] >> shift) & mask;
        uint64_t peers = __ballot(ok);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            bool bit = (d >> b) & 1u;
            uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        int leader = peers ? (__ffsll((unsigned long long)peers) - 1) : 0;
        uint32_t old = 0;
        if (ok && l == leader) {
            old = whist[w][d];
            whist[w][d] = old + (uint32_t)__popcll(peers);
        }
        old = (uint32_t)__shfl((int)old, leader, 64);
        pos[j] = old + (uint32_t)__popcll(peers & lt);
    }
    __syncthreads();
    const uint32_t d = threadIdx.x;
    uint32_t tot = 0;
#pragma unroll
    for (int ww = 0; ww < RNW; ww++) {
        uint32_t c = whist[ww][d];
        whist[ww][d] = tot;
        tot += c;
    }
    const uint64_t sidx = (uint64_t)tile * BINS + d;
    st_agent(&status[sidx], lb_word(epoch, tile == 0 ? LB_FLAG_INC : LB_FLAG_AGG, tot));
    uint32_t inc = wave_incl_scan_u32(tot);
    if (l == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t add = 0;
    for (int ww = 0; ww < w; ww++) add += wsum[ww];
    const uint32_t be = inc - tot + add;
    bexcl[d] = be;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < R_ITEMS; j++) {
        uint64_t i = wave_base + (uint64_t)j * 64 + l;
        if (i < n) {
            uint32_t dd = (uint32_t)((uint64_t)key[j] >> shift) & mask;
            pos[j] += bexcl[dd] + whist[w][dd];
            stage.keys[pos[j]] = key[j];
        }
    }
    uint64_t excl = 0;
    if (tile > 0) {
        excl = lookback_serial(status, epoch, tile, BINS, d);
        st_agent(&status[sidx], lb_word(epoch, LB_FLAG_INC, excl + tot));
    }
    gofs[d] = digit_base[d] + (uint32_t)excl - be;
    __syncthreads();
    const uint64_t tbase = (uint64_t)tile * KV_TILE;
    const uint32_t tn = (uint32_t)((n - tbase) < (uint64_t)KV_TILE ? (n - tbase) : (uint64_t)KV_TILE);
    uint32_t gp[R_ITEMS];
#pragma unroll
    for (int k = 0; k < R_ITEMS; k++) {
        uint32_t i = (uint32_t)k * RB + threadIdx.x;
        if (i < tn) {
            K kk = stage.keys[i];
            gp[k] = gofs[(uint32_t)((uint64_t)kk >> shift) & mask] + i;
            kout[gp[k]] = kk;
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < R_ITEMS; j++) {
        uint64_t i = wave_base + (uint64_t)j * 64 + l;
        if (i < n) stage.vals[pos[j]] = val[j];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < R_ITEMS; k++) {
        uint32_t i = (uint32_t)k * RB + threadIdx.x;
        if (i < tn) vout[gp[k]] = stage.vals[i];
    }
}

// ---- host side -------------------------------------------------------------------------------

static int sort_maxbits() {
    static int mb = [] {
        // tuning knob (8..11).  Measured on MI355X at 1e8 pairs, 27 key bits: 4 passes of 7 bits
        // 2.72 ms vs 3 passes of 9 bits 3.26 ms -- wider digits cost more per pass than they save.
        const char* s = getenv("QE_SORT_MAXBITS");
        int v = s ? atoi(s) : 8;
        return v < 8 ? 8 : (v > 11 ? 11 : v);
    }();
    return mb;
}

static PassDesc plan_passes(uint64_t kor, uint64_t kand, int maxbits, int* width_out) {
    PassDesc pd{};
    uint64_t vary = kor & ~kand;
    *width_out = 0;
    if (!vary) return pd;
    int lo = __builtin_ctzll(vary);
    int hi = 64 - __builtin_clzll(vary);
    int nbits = hi - lo;
    int np = (nbits + maxbits - 1) / maxbits;
    int width = (nbits + np - 1) / np;
    pd.npass = np;
    for (int p = 0; p < np; p++) {
        pd.shift[p] = lo + p * width;
        int wbits = std::min(width, hi - pd.shift[p]);
        pd.mask[p] = (1u << wbits) - 1u;
    }
    *width_out = width;
    return pd;
}

template <typename K>
static void key_bits_impl(qe_ctx* c, const K* keys, uint64_t n, uint64_t* out) {
    uint64_t* d_bits = c->d_scratch + 8;   // [or, and]
    hipLaunchKernelGGL(set2_kernel, dim3(1), dim3(64), 0, c->stream, d_bits, 0ull, ~0ull);
    QE_HIP(hipGetLastError());
    if (n) {
        Timed t(c, "sort_keybits", (double)sizeof(K) * n);
        hipLaunchKernelGGL(key_bits_kernel<K>, dim3(grid_for(n, 256 * 16, 4096)), dim3(256), 0, c->stream, keys,
                           n, d_bits);
        QE_HIP(hipGetLastError());
    }
    read_words(c, d_bits, out, 2);
}

void key_bits_u64(qe_ctx* c, const uint64_t* keys, uint64_t n, uint64_t* out) { key_bits_impl(c, keys, n, out); }

template <typename K, int RBITS>
static void hist_and_scan(qe_ctx* c, const K* keys, uint64_t n, const PassDesc& pd, uint32_t* hist) {
    QE_HIP(hipMemsetAsync(hist, 0, (size_t)pd.npass * (1u << RBITS) * sizeof(uint32_t), c->stream));
    Timed t(c, "sort_hist", (double)sizeof(K) * n);
    hipLaunchKernelGGL((digit_hist_kernel<K, RBITS>), dim3(grid_for(n, 256 * 32, 2048)), dim3(256), 0, c->stream, keys,
                       n, pd, hist);
    QE_HIP(hipGetLastError());
    hipLaunchKernelGGL((digit_scan_kernel<RBITS>), dim3(pd.npass), dim3(256), 0, c->stream, hist);
    QE_HIP(hipGetLastError());
}

// packed sort: every pass on u64 words; first pass from (key, rowid or iota), last pass back to it
template <typename K, int RBITS>
static SortOut sort_packed(qe_ctx* c, const K* keys, const uint32_t* vals, uint64_t n, const PassDesc& pd, Field f,
                           const char* name) {
    constexpr int BINS = 1 << RBITS;
    uint32_t* hist = dalloc_t<uint32_t>(c, (size_t)MAX_PASS * BINS);
    hist_and_scan<K, RBITS>(c, keys, n, pd, hist);
    const uint64_t nt = (n + RTILE - 1) / RTILE;
    const int P = pd.npass;
    uint64_t* wbuf[2] = {P > 1 ? dalloc_t<uint64_t>(c, n) : nullptr, P > 2 ? dalloc_t<uint64_t>(c, n) : nullptr};
    K* kout = dalloc_t<K>(c, n);
    uint32_t* vout = dalloc_t<uint32_t>(c, n);
    const uint64_t* win = nullptr;
    for (int p = 0; p < P; p++) {
        const bool first = p == 0, last = p == P - 1;
        const int dsh = 32 + pd.shift[p] - f.lo;
        uint64_t* wo = last ? nullptr : wbuf[p & 1];
        LBSlot s = lb_acquire(c, nt * BINS);
        double bytes = (first ? (double)sizeof(K) + 4 : 8.0) * n + (last ? (double)sizeof(K) + 4 : 8.0) * n;
        Timed t(c, name, bytes);
#define QE_RP(IN, OUT)                                                                                             \
    hipLaunchKernelGGL((radix_pass_kernel<K, IN, OUT, true, RBITS, R_ITEMS, R_NT>), dim3((unsigned)nt), dim3(R_NT), 0, \
                       c->stream,                                                                                  \
                       keys, win, vals, kout, wo, vout, n, dsh, pd.mask[p], f, hist + p * BINS, s.status, s.ticket, \
                       s.epoch)
        if (first && last) {
            if (vals) QE_RP(IN_KV, OUT_KV);
            else QE_RP(IN_KIOTA, OUT_KV);
        } else if (first) {
            if (vals) QE_RP(IN_KV, OUT_WORD);
            else QE_RP(IN_KIOTA, OUT_WORD);
        } else if (last) {
            QE_RP(IN_WORD, OUT_KV);
        } else {
            QE_RP(IN_WORD, OUT_WORD);
        }
#undef QE_RP
        QE_HIP(hipGetLastError());
        win = wo;
    }
    dfree(c, hist);
    if (wbuf[0]) dfree(c, wbuf[0]);
    if (wbuf[1]) dfree(c, wbuf[1]);
    return SortOut{kout, vout, true, true};
}

// two-level packed sort (see tl_* kernels); nullopt-style: returns false when a bucket would not
// fit LDS (skew), after which the caller runs the plain LSD passes
static LocalRounds local_rounds(int L) {   // L low bits in rounds of <= 8
    LocalRounds lr{0, {0, 0, 0, 0}};
    while (L > 0 && lr.n < 4) {
        lr.bits[lr.n] = L < 8 ? L : 8;
        L -= lr.bits[lr.n++];
    }
    return lr;
}

// both column scans of a two-level sort: m0 (rows0 x 256), m1 (rows1 x 128)
// cbase (nullable): tl_bstart_kernel's column bases -> the one-pass form
static void column_scans(qe_ctx* c, uint32_t* m0, uint32_t rows0, uint32_t* m1, uint32_t rows1, uint32_t* seg,
                         uint32_t G, uint32_t ntot, const uint32_t* cbase = nullptr) {
    CSJobs js;
    js.j[0] = CSJob{m0, nullptr, rows0, 256u, (rows0 + CS_CH - 1) / CS_CH, seg, G, ntot};
    js.j[1] = CSJob{m1, nullptr, rows1, 128u, (rows1 + CS_CH - 1) / CS_CH, nullptr, 0u, 0u};
    const unsigned nblk = js.j[0].nb + js.j[1].nb;
    if (cbase) {   // one pass (cs_single_kernel): blocks of 1024 / C row groups of CS_CH rows
        CSJobs j1 = js;
        j1.j[0].nb = (rows0 + 4 * CS_CH - 1) / (4 * CS_CH);
        j1.j[1].nb = (rows1 + 8 * CS_CH - 1) / (8 * CS_CH);
        const unsigned nb1 = j1.j[0].nb + j1.j[1].nb;
        LBSlot sl = lb_acquire(c, (size_t)nb1 * 256);
        hipLaunchKernelGGL(cs_single_kernel, dim3(nb1), dim3(1024), 0, c->stream, j1, cbase, sl.status, sl.ticket,
                           sl.epoch);
        QE_HIP(hipGetLastError());
        return;
    }
    uint32_t* part = dalloc_t<uint32_t>(c, (size_t)js.j[0].nb * 256 + (size_t)js.j[1].nb * 128);
    js.j[0].part = part;
    js.j[1].part = part + (size_t)js.j[0].nb * 256;
    hipLaunchKernelGGL(cs_reduce_kernel, dim3(nblk), dim3(256), 0, c->stream, js);
    QE_HIP(hipGetLastError());
    hipLaunchKernelGGL(cs_top_kernel, dim3(2), dim3(1024), 0, c->stream, js);
    QE_HIP(hipGetLastError());
    hipLaunchKernelGGL(cs_apply_kernel, dim3(nblk), dim3(256), 0, c->stream, js);
    QE_HIP(hipGetLastError());
    dfree(c, part);
}

#ifndef QE_PRE_NT
#define QE_PRE_NT 512
#endif
#ifndef QE_PRE_NTU
#define QE_PRE_NTU 512
#endif
// threads of the lookback-free first pass (its tile stays RTILE): 1024 x 8 measured 25 % slower
// than 512 x 16 (fewer loads in flight per thread) when its per-wave rank counters (16 KiB) left
// one workgroup per CU.  The unstable ranks count on one block-wide row: QE_PRE_NTU threads there.
constexpr int PRE_NT = QE_PRE_NT, PRE_NTU = QE_PRE_NTU;
constexpr int pre_nt(bool unstable) { return unstable ? PRE_NTU : PRE_NT; }
// The unstable first pass with a carried payload takes P1_TM = 2 consecutive counted tiles per
// workgroup (1024 threads x 16 words, a 128 KiB LDS stage: one workgroup per CU): each digit run
// it writes is twice as long (~64 words).  Round 5 on MI355X (C3, 1e8 carried rows): the digit
// scatter cost pass 1 a third of its time (a contiguous-write ablation: 598 -> 400 us); paired
// tiles 598 -> 449 us, sort_pass_carry 3.28 -> 3.12 ms per step.  Passes without a payload (half
// the bytes per element, the LDS phases a larger share) measured slower paired, 0.67 -> 0.745 ms
// per step, and keep one tile, as does the stable pass.  QE_P1_TM=1 (build knob): single tiles.
#ifndef QE_P1_TM
#define QE_P1_TM 2
#endif
constexpr int P1_TM = QE_P1_TM;
static_assert(P1_TM == 1 || (P1_TM == 2 && TL_TPG % 2 == 0), "paired tiles stay inside one group");
constexpr int p1_tm(bool unstable, int carry) { return unstable && carry != X_NONE ? P1_TM : 1; }

static bool gather_k32_on() {   // A/B knob: QE_GATHER_K32=0 gathers the plan's keys as u64
    static bool on = [] {
        const char* s = getenv("QE_GATHER_K32");
        return !(s && s[0] == '0');
    }();
    return on;
}

static bool cs_single_on() {   // A/B knob: QE_CS_SINGLE=0 keeps the three-launch count scans
    static bool on = [] {
        const char* s = getenv("QE_CS_SINGLE");
        return !(s && s[0] == '0');
    }();
    return on;
}

static bool prof_split() {   // tuning aid: QE_PROF_SPLIT=1 times the second pass under its own name
    static bool on = [] {
        const char* s = getenv("QE_PROF_SPLIT");
        return s && s[0] == '1';
    }();
    return on;
}

// blocks of tl_hist_kernel.  Each block zeroes a 32 K-bucket LDS table and adds it out with device-
// scope atomics (executed at the memory side: ~0.1 us of chip time per block, on 32 K words every
// block shares), against ~2.7 keys per CU cycle of LDS atomics while counting: B ~ sqrt(n / 720)
// balances the two (round 3 used one block per 4096 keys up to 256: a 1e6-key sort paid 256
// flushes for 4 K keys each).  QE_HIST_C tunes the constant; 0 restores round 3's grid.
static unsigned hist_blocks(uint64_t n) {
    static const double C = [] {
        const char* s = getenv("QE_HIST_C");
        return s ? atof(s) : 720.0;
    }();
    if (C <= 0) return grid_for((n + 3) / 4, 1024, 256);
    const double b = sqrt((double)n / C);
    return b < 8 ? 8u : b > 256 ? 256u : (unsigned)b;
}

static uint64_t sort_pre_min() {   // tuning knob: QE_SORT_PRE_MIN = smallest n for the lookback-free form
    static uint64_t v = [] {
        const char* s = getenv("QE_SORT_PRE_MIN");
        return s ? strtoull(s, nullptr, 0) : (1ull << 22);   // (round 3: 2^25; see sort_two_level)
    }();
    return v;
}

static bool sort_unstable_on() {
    static bool on = [] {   // tuning knob: QE_SORT_UNSTABLE=0 keeps the stable ranks in deferred sorts too
        const char* s = getenv("QE_SORT_UNSTABLE");
        return !(s && s[0] == '0');
    }();
    return on;
}

static bool sort_pre_on() {
    static bool on = [] {   // tuning knob: QE_SORT_PRE=0 keeps the lookback form of the two passes
        const char* s = getenv("QE_SORT_PRE");
        return !(s && s[0] == '0');
    }();
    return on;
}

// the per-bucket LDS step of a two-level sort over packed words: one wave per bucket when the
// largest bucket fits one wave's TL_ITEMS x 64 words (the 15-bit geometry over up to ~20 M keys:
// buckets of tens to hundreds of words), else TL_NT threads per bucket.  QE_LOCAL_WAVE=0 (A/B knob)
// keeps TL_NT threads everywhere.
template <typename K>
static void local_sort_buckets(qe_ctx* c, const uint64_t* words, K* kout, uint32_t* vout, const uint32_t* bstart,
                               unsigned nbuckets, Field f, LocalRounds lr, uint64_t maxb, bool unstable0 = false) {
    static const bool wave_on = !(getenv("QE_LOCAL_WAVE") && getenv("QE_LOCAL_WAVE")[0] == '0');
    const bool one_wave = wave_on && maxb <= 64u * TL_ITEMS;
#define QE_LOCAL(NTH, UN)                                                                                                \
    hipLaunchKernelGGL((tl_local_kernel<K, IN_WORD, NTH, UN>), dim3(nbuckets), dim3(NTH), 0, c->stream, words, nullptr, \
                       nullptr, kout, vout, bstart, 0u, f, lr)
    if (one_wave && unstable0) QE_LOCAL(64, true);
    else if (one_wave) QE_LOCAL(64, false);
    else if (unstable0) QE_LOCAL(TL_NT, true);
    else QE_LOCAL(TL_NT, false);
#undef QE_LOCAL
    QE_HIP(hipGetLastError());
}

// where a histogram kernel stores its group counts: gcnt itself when every group has one block, else
// Q slices that hist_fold adds into gcnt (and frees), also writing the bucket histogram when asked
static uint32_t* hist_slices(qe_ctx* c, uint32_t* gcnt, uint32_t Q, uint32_t nseg) {
    return Q > 1 ? dalloc_t<uint32_t>(c, (size_t)Q * nseg * 128) : gcnt;
}
static void hist_fold(qe_ctx* c, uint32_t* gout, uint32_t Q, uint32_t G, uint32_t* gcnt, uint32_t* hist,
                      uint32_t* d1part = nullptr) {
    if (gout != gcnt || hist) {
        hipLaunchKernelGGL(tl_gfold_kernel, dim3(1024), dim3(256), 0, c->stream, gout, gout != gcnt ? Q : 1u, G, gcnt,
                           hist, d1part);
        QE_HIP(hipGetLastError());
    }
    if (gout != gcnt) dfree(c, gout);
}

// the two-level sort (H = TL_H) with both global passes lookback-free (see tl_hist_tiles_kernel)
template <typename K>
static bool sort_two_level_pre(qe_ctx* c, const K* keys, const uint32_t* vals, uint64_t n, int bits, Field f,
                               const char* name, SortOut* out, bool defer = false) {
    const int L = bits - TL_H;
    const LocalRounds lr = local_rounds(L);
    const uint32_t nt = (uint32_t)((n + RTILE - 1) / RTILE);
    const uint32_t G = (nt + TL_TPG - 1) / TL_TPG;
    const uint32_t Q = G >= 256 ? 1u : 256u / G;   // ~one histogram block per CU
    const uint32_t nseg = 256u * G;
    uint32_t* tcnt = dalloc_t<uint32_t>(c, (size_t)nt * 256);
    uint32_t* gcnt = dalloc_t<uint32_t>(c, (size_t)nseg * 128);
    uint32_t* hist = dalloc_t<uint32_t>(c, TL_BUCKETS);
    // (+ the count scans' column bases and the d1 partial sums they come from, 16-B aligned)
    uint32_t* bstart = dalloc_t<uint32_t>(c, TL_BUCKETS + 4 + (cs_single_on() ? 384 + 1024 : 0));
    uint32_t* cbase = cs_single_on() ? bstart + TL_BUCKETS + 4 : nullptr;
    uint32_t* d1part = cs_single_on() ? cbase + 384 : nullptr;
    uint32_t* seg = dalloc_t<uint32_t>(c, (size_t)nseg + 1);   // the second pass's segment starts
    // a deferred sort keeps its largest bucket on the device: the consumer checks it there
    // (bucket_join) or reads it when it completes the sort (pairs_need_keys) -- no round trip here
    const bool dfr = defer && sizeof(K) == 8;
    uint64_t* d_max = dfr ? dalloc_t<uint64_t>(c, 1) : c->d_scratch + 34;
    auto release = [&] {
        dfree(c, tcnt);
        dfree(c, gcnt);
        dfree(c, hist);
        dfree(c, bstart);
        dfree(c, seg);
    };
    // a base column with a u32 copy (Relation::cols32): the histogram and the first pass read that
    // -- along with the u32 copies of its payload / value columns -- when every one of them has one
    const uint32_t* kn = dfr && !vals && sizeof(K) == 8 ? narrow_of(c, keys, n) : nullptr;
    if (kn) {
        if (c->carry_xa || (c->carry_c64 && !narrow_of(c, c->carry_c64, n)) || (c->sort_v64 && !narrow_of(c, c->sort_v64, n)))
            kn = nullptr;
    }
    auto ph = c->prehist.find(keys);   // counted while the keys were gathered?
    const bool have = ph != c->prehist.end() && ph->second.lo == f.lo && ph->second.L == L &&
                      ph->second.fmask == f.fmask;
    // keys gathered as u32 only (PreHist::k32): this sort's first pass reads them when it is the
    // unstable deferred form that reads u32 keys with u32 values (its rowids) -- else they are
    // widened into the key buffer first
    const uint32_t* k32 = nullptr;
    {
        const bool k32_ok = have && ph->second.k32 && dfr && vals && sort_unstable_on() && !c->carry_c64 &&
                            !c->sort_v64;
        if (k32_ok) k32 = ph->second.k32;
        else if (ph != c->prehist.end()) keys_need_u64(c, keys);
    }
    if (have) {
        dfree(c, tcnt);
        dfree(c, gcnt);
        tcnt = ph->second.tcnt;
        gcnt = ph->second.gcnt;
        if (k32) {   // the u32 keys stay with the key buffer: a later sort of the same buffer (a
            ph->second.tcnt = ph->second.gcnt = nullptr;   // join's fallback) widens them, and
            ph->second.lo = -1;                            // the buffer's release frees them
        } else {
            c->prehist.erase(ph);
        }
    }
    if (k32) kn = k32;
    {
        Timed t(c, "sort_hist", have ? 0.0 : (kn ? 4.0 : (double)sizeof(K)) * n);
        uint32_t* gout = have ? gcnt : hist_slices(c, gcnt, Q, nseg);
        if (!have && kn)
            hipLaunchKernelGGL((tl_hist_tiles_kernel<uint32_t>), dim3(G * Q), dim3(1024), 0, c->stream, kn, n, f, L, nt,
                               G, Q, tcnt, gout);
        else if (!have)
            hipLaunchKernelGGL((tl_hist_tiles_kernel<K>), dim3(G * Q), dim3(1024), 0, c->stream, keys, n, f, L, nt, G,
                               Q, tcnt, gout);
        QE_HIP(hipGetLastError());
        hist_fold(c, gout, have ? 1u : Q, G, gcnt, hist, d1part);
        hipLaunchKernelGGL(tl_bstart_kernel, dim3(1), dim3(1024), 0, c->stream, hist, bstart, d_max, cbase, d1part);
        QE_HIP(hipGetLastError());
    }
    {
        Timed t(c, "sort_scan", 8.0 * ((double)nt * 256 + (double)nseg * 128));
        column_scans(c, tcnt, nt, gcnt, nseg, seg, G, (uint32_t)n, cbase);
    }
    uint64_t* w1 = dalloc_t<uint64_t>(c, n);
    uint64_t* w2 = dalloc_t<uint64_t>(c, n);
    K* kout = dalloc_t<K>(c, n);
    uint32_t* vout = dalloc_t<uint32_t>(c, n);
    // a payload to carry (join_pairs_carry asked for it on this deferred sort)
    // (X64: S's carried bindings; X32 / XCOL: one 32-bit payload, R's next join key)
    const uint32_t* cxa = dfr ? c->carry_xa : nullptr;
    const uint32_t* cxb = dfr ? c->carry_xb : nullptr;
    const int xm = !dfr ? X_NONE : c->carry_xa ? X64 : c->carry_x32 ? X32 : c->carry_c64 ? XCOL : X_NONE;
    if (xm == X32) cxa = c->carry_x32;
    if (xm == XCOL) cxa = reinterpret_cast<const uint32_t*>(c->carry_c64);
    c->carry_xa = c->carry_xb = c->carry_x32 = nullptr;
    c->carry_c64 = nullptr;
    // the packed value: a u64 column's low words instead of the row index (a base relation whose
    // binding is read later only through that column: its values ride in place of the rowids)
    const uint64_t* cv64 = dfr && !vals && (xm == XCOL || xm == X_NONE) ? c->sort_v64 : nullptr;
    c->sort_v64 = nullptr;
    const uint32_t* v64w = reinterpret_cast<const uint32_t*>(cv64);
    // key-only words (the consumer counts this side's keys and never reads its rows: the last
    // join's aggregate form): u32 fields through both passes, half the bytes
    const bool w32 = dfr && !vals && xm == X_NONE && !cv64 && sort_unstable_on() && c->sort_keys_only;
    c->sort_keys_only = false;
    const size_t xsz = xm == X64 ? 8 : 4;
    uint64_t* x1 = xm ? static_cast<uint64_t*>(dalloc(c, n * xsz)) : nullptr;
    uint64_t* x2 = xm ? static_cast<uint64_t*>(dalloc(c, n * xsz)) : nullptr;
    if (xm && alloc_log_on())
        fprintf(stderr, "[qe sort_pass_carry] n=%llu w1=%p w2=%p x1=%p x2=%p keys=%p\n", (unsigned long long)n,
                (void*)w1, (void*)w2, (void*)x1, (void*)x2, (const void*)keys);
    // a deferred sort's consumer needs its buckets, not an order inside them: unstable ranks
    const bool uns = dfr && sort_unstable_on();
#define QE_P1(IN, CR, UN, XA, XB, XO)                                                                                   \
    hipLaunchKernelGGL((radix_pass_kernel<K, IN, OUT_WORD, true, 8, RTILE / pre_nt(UN), pre_nt(UN) * p1_tm(UN, CR), true, CR, UN, p1_tm(UN, CR)>),  \
                       dim3(xcd_grid((nt + p1_tm(UN, CR) - 1) / p1_tm(UN, CR))), dim3(pre_nt(UN) * p1_tm(UN, CR)), 0, c->stream, keys, nullptr, vals, kout, w1, vout, n, 32 + L, \
                       255u, f, tcnt, nullptr, nullptr, 0u, XA, XB, XO)
#define QE_P1N(IN, CR, VIN, XA, XB)                                                                                     \
    hipLaunchKernelGGL((radix_pass_kernel<uint32_t, IN, OUT_WORD, true, 8, RTILE / pre_nt(true), pre_nt(true) * p1_tm(true, CR), true, CR, true, p1_tm(true, CR)>),      \
                       dim3(xcd_grid((nt + p1_tm(true, CR) - 1) / p1_tm(true, CR))), dim3(pre_nt(true) * p1_tm(true, CR)), 0, c->stream, kn, nullptr, VIN, nullptr, w1, vout, n, 32 + L,     \
                       255u, f, tcnt, nullptr, nullptr, 0u, XA, XB, x1)
#ifdef QE_DIAG_STAMPS
    stamp_select(c, "p1", n);
#endif
    if (kn && uns) {
        // u32 key (+ u32 value: a base column's values riding as rows, or a gathered side's rowids)
        // (+ u32 payload, or X64's one or two u32 columns) in, word (+ payload) out
        const uint32_t* vt = vals ? vals : cv64 ? narrow_of(c, cv64, n) : nullptr;
        const uint32_t* xt = xm == XCOL ? narrow_of(c, reinterpret_cast<const uint64_t*>(cxa), n) : xm == X32 ? cxa : nullptr;
        const double xin = xm == X64 ? 4.0 + (cxb ? 4.0 : 0.0) : xt ? 4.0 : 0.0, xout = xm == X64 ? 8.0 : xt ? 4.0 : 0.0;
        Timed t(c, xm ? "sort_pass_carry" : name, (4.0 + (vt ? 4.0 : 0.0) + xin + (w32 ? 4.0 : 8.0) + xout) * n);
        if (xm == X64 && vt) QE_P1N(IN_KV, X64, vt, cxa, cxb);
        else if (xm == X64) QE_P1N(IN_KIOTA, X64, nullptr, cxa, cxb);
        else if (w32)
            hipLaunchKernelGGL((radix_pass_kernel<uint32_t, IN_KIOTA, OUT_W32, true, 8, RTILE / pre_nt(true), pre_nt(true) * p1_tm(true, X_NONE), true, X_NONE, true, p1_tm(true, X_NONE)>),
                               dim3(xcd_grid((nt + p1_tm(true, X_NONE) - 1) / p1_tm(true, X_NONE))), dim3(pre_nt(true) * p1_tm(true, X_NONE)), 0, c->stream, kn, nullptr, nullptr, nullptr, w1, vout, n,
                               32 + L, 255u, f, tcnt, nullptr, nullptr, 0u, nullptr, nullptr, nullptr);
        else if (vt && xt) QE_P1N(IN_KV, X32, vt, xt, nullptr);
        else if (vt) QE_P1N(IN_KV, X_NONE, vt, nullptr, nullptr);
        else if (xt) QE_P1N(IN_KIOTA, X32, nullptr, xt, nullptr);
        else QE_P1N(IN_KIOTA, X_NONE, nullptr, nullptr, nullptr);
        QE_HIP(hipGetLastError());
    } else if (w32) {
        Timed t(c, name, ((double)sizeof(K) + 4.0) * n);
        hipLaunchKernelGGL((radix_pass_kernel<K, IN_KIOTA, OUT_W32, true, 8, RTILE / pre_nt(true), pre_nt(true) * p1_tm(true, X_NONE), true, X_NONE, true, p1_tm(true, X_NONE)>),
                           dim3(xcd_grid((nt + p1_tm(true, X_NONE) - 1) / p1_tm(true, X_NONE))), dim3(pre_nt(true) * p1_tm(true, X_NONE)), 0, c->stream, keys, nullptr, nullptr, kout, w1, vout, n,
                           32 + L, 255u, f, tcnt, nullptr, nullptr, 0u, nullptr, nullptr, nullptr);
        QE_HIP(hipGetLastError());
    } else if (cv64) {
        Timed t(c, xm ? "sort_pass_carry" : name, ((double)sizeof(K) + 8.0 + (xm ? 8.0 : 0.0) + 8.0 + (xm ? 4.0 : 0.0)) * n);
        if (xm)
            hipLaunchKernelGGL((radix_pass_kernel<K, IN_KV64, OUT_WORD, true, 8, RTILE / pre_nt(true), pre_nt(true) * p1_tm(true, XCOL), true, XCOL, true, p1_tm(true, XCOL)>),
                               dim3(xcd_grid((nt + p1_tm(true, XCOL) - 1) / p1_tm(true, XCOL))), dim3(pre_nt(true) * p1_tm(true, XCOL)), 0, c->stream, keys, nullptr, v64w, kout, w1, vout, n,
                               32 + L, 255u, f, tcnt, nullptr, nullptr, 0u, cxa, nullptr, x1);
        else
            hipLaunchKernelGGL((radix_pass_kernel<K, IN_KV64, OUT_WORD, true, 8, RTILE / pre_nt(true), pre_nt(true) * p1_tm(true, X_NONE), true, X_NONE, true, p1_tm(true, X_NONE)>),
                               dim3(xcd_grid((nt + p1_tm(true, X_NONE) - 1) / p1_tm(true, X_NONE))), dim3(pre_nt(true) * p1_tm(true, X_NONE)), 0, c->stream, keys, nullptr, v64w, kout, w1, vout, n,
                               32 + L, 255u, f, tcnt, nullptr, nullptr, 0u, nullptr, nullptr, nullptr);
        QE_HIP(hipGetLastError());
    } else if (xm == X64) {
        const double xb = cxb ? 8.0 : 4.0;
        Timed t(c, "sort_pass_carry", ((double)sizeof(K) + (vals ? 4.0 : 0.0) + 8.0 + xb + 8.0) * n);
        if (vals && uns) QE_P1(IN_KV, X64, true, cxa, cxb, x1);
        else if (vals) QE_P1(IN_KV, X64, false, cxa, cxb, x1);
        else if (uns) QE_P1(IN_KIOTA, X64, true, cxa, cxb, x1);
        else QE_P1(IN_KIOTA, X64, false, cxa, cxb, x1);
        QE_HIP(hipGetLastError());
    } else if (xm) {
        // key (+ rowid) in, + the payload's 4 (X32) or 8 (XCOL: a u64 column) bytes; word + 4 B out
        Timed t(c, "sort_pass_carry", ((double)sizeof(K) + (vals ? 4.0 : 0.0) + (xm == XCOL ? 8.0 : 4.0) + 12.0) * n);
        if (xm == X32 && vals) QE_P1(IN_KV, X32, true, cxa, nullptr, x1);
        else if (xm == X32) QE_P1(IN_KIOTA, X32, true, cxa, nullptr, x1);
        else if (vals) QE_P1(IN_KV, XCOL, true, cxa, nullptr, x1);
        else QE_P1(IN_KIOTA, XCOL, true, cxa, nullptr, x1);
        QE_HIP(hipGetLastError());
    } else {
        // algorithmic bytes: key (+ rowid when given; generated otherwise) in, packed word out
        Timed t(c, name, ((double)sizeof(K) + (vals ? 4.0 : 0.0) + 8.0) * n);
        if (vals && uns) QE_P1(IN_KV, false, true, nullptr, nullptr, nullptr);
        else if (vals) QE_P1(IN_KV, false, false, nullptr, nullptr, nullptr);
        else if (uns) QE_P1(IN_KIOTA, false, true, nullptr, nullptr, nullptr);
        else QE_P1(IN_KIOTA, false, false, nullptr, nullptr, nullptr);
        QE_HIP(hipGetLastError());
    }
#undef QE_P1
#undef QE_P1N
    {
        Timed t(c, xm ? "sort_pass_carry" : prof_split() ? "sort_pass2" : name,
                (w32 ? 8.0 : 16.0 + 2.0 * (double)(xm ? xsz : 0)) * n);
        auto kern = w32       ? tl_pass2_kernel<K, X_NONE, true, true>
                    : xm == X64 ? (uns ? (x64_staged() ? tl_pass2_kernel<K, X64, true, false, true> : tl_pass2_kernel<K, X64, true>)
                                       : (x64_staged() ? tl_pass2_kernel<K, X64, false, false, true> : tl_pass2_kernel<K, X64, false>))
                    : xm      ? tl_pass2_kernel<K, X32, true>   // (the X32 / XCOL first pass is unstable too)
                              : (uns ? tl_pass2_kernel<K, X_NONE, true> : tl_pass2_kernel<K, X_NONE, false>);
#ifdef QE_DIAG_STAMPS
        stamp_select(c, "p2", n);
#endif
        hipLaunchKernelGGL(kern, dim3(xcd_grid(nseg)), dim3(TL2_NT), 0, c->stream, w1, w2, n, 32 + L + 8, seg, gcnt, G,
                           x1, x2);
        QE_HIP(hipGetLastError());
        if (xm) dfree(c, x1);
    }
    // the two passes are valid whatever the bucket sizes, so they are queued before the host
    // reads the largest bucket: the GPU stays busy through that round trip
    const uint64_t maxb = dfr ? 0 : read_u64(c, d_max);
    if (!dfr && maxb > (uint64_t)TL_CAP) {   // a bucket beyond LDS (skew): plain LSD passes
        dfree(c, w1);
        dfree(c, w2);
        dfree(c, kout);
        dfree(c, vout);
        release();
        return false;
    }
    if constexpr (sizeof(K) == 8) {
        if (dfr) {   // the per-bucket step waits for the consumer (bucket_join / pairs_need_keys)
            DeferredSort d;
            d.words = w2;
            d.bstart = bstart;
            d.d_max = d_max;
            d.x = xm == X64 ? x2 : nullptr;
            d.v64 = cv64;
            d.w32 = w32;
            d.x32 = xm && xm != X64 ? reinterpret_cast<uint32_t*>(x2) : nullptr;
            d.kout = (uint64_t*)kout;
            d.vout = vout;
            d.lo = f.lo;
            d.L = L;
            d.fmask = f.fmask;
            d.kconst = f.kconst;
            d.lr_n = lr.n;
            for (int r = 0; r < 4; r++) d.lr_bits[r] = lr.bits[r];
            c->deferred[kout] = d;
            dfree(c, w1);
            dfree(c, tcnt);
            dfree(c, gcnt);
            dfree(c, hist);
            dfree(c, seg);
            *out = SortOut{kout, vout, true, true};
            return true;
        }
    }
    {
        Timed t(c, "sort_local", 8.0 * n + ((double)sizeof(K) + 4) * n);
        local_sort_buckets<K>(c, w2, kout, vout, bstart, TL_BUCKETS, f, lr, maxb);
    }
    dfree(c, w1);
    dfree(c, w2);
    release();
    *out = SortOut{kout, vout, true, true};
    return true;
}

// H = TL_H (15 high bits by two global passes) for large inputs; H = 8 (ONE global pass) for
// inputs whose 256 buckets fit LDS (<= ~1 M keys)
template <typename K>
static bool sort_two_level(qe_ctx* c, const K* keys, const uint32_t* vals, uint64_t n, int bits, Field f,
                           const char* name, SortOut* out, int H = TL_H, bool defer = false) {
    // the lookback-free form saves ~1 us per million keys per pass but adds the count scans: round
    // 3 measured it paying from a few 10^7 keys (C4's 1-10 M-key sorts slower); with round 4's
    // cheaper scans and histograms it pays from 2^22 keys (C4 3724 -> 3748 q/s averaged over four
    // same-box pairs, 2^21 and 2^23 no better: profiles/r04q_c4_knobs_ab.log, r04r_c4_knobs_ab.log)
    if (H == TL_H && sort_pre_on() && n >= sort_pre_min())
        return sort_two_level_pre<K>(c, keys, vals, n, bits, f, name, out, defer);
    const int L = bits - H;   // low bits sorted in LDS (<= 24)
    const LocalRounds lr = local_rounds(L);
    if (!c->d_zhist) {   // once per context; every scan below leaves it zeroed again
        QE_HIP(hipMalloc(&c->d_zhist, (TL_BUCKETS + 256) * sizeof(uint32_t)));
        c->zhist_dirty = true;
    }
    // a throw between a histogram launch and its scan's (which re-zeroes the table) leaves counts
    // behind: the flag, set from the one to the other, makes the next sort clear the table first
    if (c->zhist_dirty) QE_HIP(hipMemsetAsync(c->d_zhist, 0, (TL_BUCKETS + 256) * sizeof(uint32_t), c->stream));
    c->zhist_dirty = true;
    uint32_t* hist = H == 8 ? c->d_zhist + TL_BUCKETS : c->d_zhist;
    // digit bases: 256 entries each (the pass kernel reads one per possible 8-bit digit)
    uint32_t* bstart = dalloc_t<uint32_t>(c, TL_BUCKETS + 1 + 512);
    uint32_t* base1 = bstart + TL_BUCKETS + 1;
    uint32_t* base2 = base1 + 256;
    const bool dfr = defer && H == TL_H && sizeof(K) == 8;   // largest bucket checked by the consumer
    uint64_t* d_max = dfr ? dalloc_t<uint64_t>(c, 1) : c->d_scratch + 34;
    if (H == 8) {
        base1 = bstart;   // one pass: its digit IS the bucket
        Timed t(c, "sort_hist", (double)sizeof(K) * n);
        hipLaunchKernelGGL((tl_hist8_kernel<K>), dim3(grid_for(n, 256 * 16, 1024)), dim3(256), 0, c->stream, keys, n, f,
                           L, hist);
        QE_HIP(hipGetLastError());
        hipLaunchKernelGGL(tl_scan8_kernel, dim3(1), dim3(256), 0, c->stream, hist, bstart, d_max);
        QE_HIP(hipGetLastError());
        c->zhist_dirty = false;
    } else {
        Timed t(c, "sort_hist", (double)sizeof(K) * n);
        hipLaunchKernelGGL((tl_hist_kernel<K>), dim3(hist_blocks(n)), dim3(1024), 0, c->stream, keys, n, f, L, hist);
        QE_HIP(hipGetLastError());
        hipLaunchKernelGGL(tl_scan_kernel, dim3(1), dim3(1024), 0, c->stream, hist, bstart, base1, base2, d_max);
        QE_HIP(hipGetLastError());
        c->zhist_dirty = false;
    }
#if !QE_LB_MAXB_LATE
    const uint64_t maxb = dfr ? 0 : read_u64(c, d_max);
    if (!dfr && maxb > (uint64_t)TL_CAP) {
        dfree(c, bstart);
        return false;
    }
#endif
    const uint64_t nt = (n + RTILE - 1) / RTILE;
    uint64_t* w1 = dalloc_t<uint64_t>(c, n);
    uint64_t* w2 = H == TL_H ? dalloc_t<uint64_t>(c, n) : nullptr;
    K* kout = dalloc_t<K>(c, n);
    uint32_t* vout = dalloc_t<uint32_t>(c, n);
    // a deferred sort's consumer (the plan's join) needs buckets, not an order inside them: the
    // first pass ranks unstably (one LDS atomic per element instead of 8 ballots).  The second
    // stays stable -- in this lookback form a tile holds several first digits, and an unstable
    // rank would interleave their buckets
    const bool uns = dfr && sort_unstable_on() && H == TL_H;
    for (int p = 0; p < (H == TL_H ? 2 : 1); p++) {
        const int dsh = 32 + L + 8 * p;
        const uint32_t pmask = p == 0 ? 255u : 127u;
        LBSlot sl = lb_acquire(c, nt * 256);
        Timed t(c, name, p == 0 ? ((double)sizeof(K) + 4 + 8) * n : 16.0 * n);
        if (p == 1)
            hipLaunchKernelGGL((radix_pass_kernel<K, IN_WORD, OUT_WORD, true, 8, R_ITEMS, R_NT>), dim3((unsigned)nt),
                               dim3(R_NT), 0, c->stream, keys, w1, vals, kout, w2, vout, n, dsh, pmask, f, base2,
                               sl.status, sl.ticket, sl.epoch);
        else if (vals && uns)
            hipLaunchKernelGGL((radix_pass_kernel<K, IN_KV, OUT_WORD, true, 8, R_ITEMS, R_NT, false, X_NONE, true>),
                               dim3((unsigned)nt), dim3(R_NT), 0, c->stream, keys, nullptr, vals, kout, w1, vout, n, dsh,
                               pmask, f, base1, sl.status, sl.ticket, sl.epoch);
        else if (vals)
            hipLaunchKernelGGL((radix_pass_kernel<K, IN_KV, OUT_WORD, true, 8, R_ITEMS, R_NT>), dim3((unsigned)nt),
                               dim3(R_NT), 0, c->stream, keys, nullptr, vals, kout, w1, vout, n, dsh, pmask, f, base1,
                               sl.status, sl.ticket, sl.epoch);
        else if (uns)
            hipLaunchKernelGGL((radix_pass_kernel<K, IN_KIOTA, OUT_WORD, true, 8, R_ITEMS, R_NT, false, X_NONE, true>),
                               dim3((unsigned)nt), dim3(R_NT), 0, c->stream, keys, nullptr, vals, kout, w1, vout, n, dsh,
                               pmask, f, base1, sl.status, sl.ticket, sl.epoch);
        else
            hipLaunchKernelGGL((radix_pass_kernel<K, IN_KIOTA, OUT_WORD, true, 8, R_ITEMS, R_NT>), dim3((unsigned)nt),
                               dim3(R_NT), 0, c->stream, keys, nullptr, vals, kout, w1, vout, n, dsh, pmask, f, base1,
                               sl.status, sl.ticket, sl.epoch);
        QE_HIP(hipGetLastError());
    }
#if QE_LB_MAXB_LATE
    // the passes are valid whatever the bucket sizes (their digit bases come from the histogram):
    // queued before the host reads the largest bucket, as in the lookback-free form, so the GPU
    // works through the round trip instead of waiting for the next launch
    const uint64_t maxb = dfr ? 0 : read_u64(c, d_max);
    if (!dfr && maxb > (uint64_t)TL_CAP) {   // a bucket beyond LDS (skew): plain LSD passes
        dfree(c, w1);
        if (w2) dfree(c, w2);
        dfree(c, kout);
        dfree(c, vout);
        dfree(c, bstart);
        return false;
    }
#endif
    if constexpr (sizeof(K) == 8) {
        if (dfr) {   // the per-bucket step waits for the consumer (bucket_join / pairs_need_keys)
            DeferredSort d;
            d.words = w2;
            d.bstart = bstart;
            d.d_max = d_max;
            d.kout = (uint64_t*)kout;
            d.vout = vout;
            d.lo = f.lo;
            d.L = L;
            d.fmask = f.fmask;
            d.kconst = f.kconst;
            d.lr_n = lr.n;
            for (int r = 0; r < 4; r++) d.lr_bits[r] = lr.bits[r];
            c->deferred[kout] = d;
            dfree(c, w1);
            *out = SortOut{kout, vout, true, true};
            return true;
        }
    }
    {
        Timed t(c, "sort_local", 8.0 * n + ((double)sizeof(K) + 4) * n);
        local_sort_buckets<K>(c, H == TL_H ? w2 : w1, kout, vout, bstart, 1u << H, f, lr, maxb);
    }
    dfree(c, w1);
    if (w2) dfree(c, w2);
    dfree(c, bstart);
    *out = SortOut{kout, vout, true, true};
    return true;
}

static bool two_level_on() {
    static bool on = [] {   // tuning knob: QE_SORT_TWO_LEVEL=0 keeps every pass global
        const char* s = getenv("QE_SORT_TWO_LEVEL");
        return !(s && s[0] == '0');
    }();
    return on;
}

// key-only sort of 64-bit words (dedup of packed pairs): the word is the key
template <int RBITS>
static SortOut sort_keys_only(qe_ctx* c, const uint64_t* keys, uint64_t n, const PassDesc& pd, const char* name) {
    constexpr int BINS = 1 << RBITS;
    uint32_t* hist = dalloc_t<uint32_t>(c, (size_t)MAX_PASS * BINS);
    hist_and_scan<uint64_t, RBITS>(c, keys, n, pd, hist);
    const uint64_t nt = (n + RTILE - 1) / RTILE;
    uint64_t* buf[2] = {dalloc_t<uint64_t>(c, n), pd.npass > 1 ? dalloc_t<uint64_t>(c, n) : nullptr};
    const uint64_t* in = keys;
    Field f{0, 0, 0};
    for (int p = 0; p < pd.npass; p++) {
        uint64_t* out = buf[p & 1];
        LBSlot s = lb_acquire(c, nt * BINS);
        Timed t(c, name, 16.0 * n);
        hipLaunchKernelGGL((radix_pass_kernel<uint64_t, IN_WORD, OUT_WORD, false, RBITS, R_ITEMS, R_NT>), dim3((unsigned)nt), dim3(R_NT),
                           0, c->stream, nullptr, in, nullptr, nullptr, out, nullptr, n, pd.shift[p], pd.mask[p], f,
                           hist + p * BINS, s.status, s.ticket, s.epoch);
        QE_HIP(hipGetLastError());
        in = out;
    }
    dfree(c, hist);
    int last = (pd.npass - 1) & 1;
    if (pd.npass > 1) dfree(c, buf[last ^ 1]);
    return SortOut{buf[last], nullptr, true, false};
}

template <typename K>
static SortOut sort_kv_unpacked(qe_ctx* c, const K* keys, const uint32_t* vals, uint64_t n, const PassDesc& pd,
                                const char* name) {
    uint32_t* hist = dalloc_t<uint32_t>(c, (size_t)MAX_PASS * 256);
    hist_and_scan<K, 8>(c, keys, n, pd, hist);
    const uint64_t nt = (n + KV_TILE - 1) / KV_TILE;
    K* kbuf[2] = {dalloc_t<K>(c, n), pd.npass > 1 ? dalloc_t<K>(c, n) : nullptr};
    uint32_t* vbuf[2] = {dalloc_t<uint32_t>(c, n), pd.npass > 1 ? dalloc_t<uint32_t>(c, n) : nullptr};
    const K* kin = keys;
    const uint32_t* vin = vals;
    for (int p = 0; p < pd.npass; p++) {
        LBSlot s = lb_acquire(c, nt * 256);
        Timed t(c, name, 2.0 * n * (sizeof(K) + 4));
        if (vin)
            hipLaunchKernelGGL((radix_pass_kv_kernel<K, true>), dim3((unsigned)nt), dim3(RB), 0, c->stream, kin, vin,
                               kbuf[p & 1], vbuf[p & 1], n, pd.shift[p], pd.mask[p], hist + p * 256, s.status,
                               s.ticket, s.epoch);
        else
            hipLaunchKernelGGL((radix_pass_kv_kernel<K, false>), dim3((unsigned)nt), dim3(RB), 0, c->stream, kin,
                               nullptr, kbuf[p & 1], vbuf[p & 1], n, pd.shift[p], pd.mask[p], hist + p * 256,
                               s.status, s.ticket, s.epoch);
        QE_HIP(hipGetLastError());
        kin = kbuf[p & 1];
        vin = vbuf[p & 1];
    }
    dfree(c, hist);
    int last = (pd.npass - 1) & 1;
    if (pd.npass > 1) {
        dfree(c, kbuf[last ^ 1]);
        dfree(c, vbuf[last ^ 1]);
    }
    return SortOut{kbuf[last], vbuf[last], true, true};
}

// true when radix_sort_impl's plan for these keys is the lookback-free two-level sort (the one that
// may read a gathered side's u32 keys, PreHist::k32) -- the conditions gather_hist_impl checks
static bool takes_pre_two_level(uint64_t n, const uint64_t* bits, bool with_vals, bool defer) {
    if (!bits || !with_vals || !defer || n < 2 || n >= 0xFFFFFFFFull) return false;
    const uint64_t vary = bits[0] & ~bits[1];
    if (!vary) return false;
    const int lo = __builtin_ctzll(vary), hi = 64 - __builtin_clzll(vary), nb = hi - lo;
    if (nb > 32 || !two_level_on() || n <= (uint64_t)TL_CAP) return false;
    if (nb >= 12 && nb <= 8 + 24 && n <= 700000) return false;
    if (!(nb >= 20 && nb <= TL_H + 16 && n >= (1u << 20) && n <= 4000ull * TL_BUCKETS)) return false;
    return sort_pre_on() && n >= sort_pre_min();
}

template <typename K>
static SortOut radix_sort_impl(qe_ctx* c, const K* keys, const uint32_t* vals, uint64_t n, bool with_vals,
                               const char* name, const uint64_t* bits, bool defer = false) {
    SortOut so{(void*)keys, (uint32_t*)vals, false, false};
    // keys gathered as u32 only: widened now unless the sort that reads them comes next
    if (sizeof(K) == 8 && !c->prehist.empty() && !takes_pre_two_level(n, bits, with_vals, defer)) keys_need_u64(c, keys);
    if (n < 2) return so;
    if (n >= 0xFFFFFFFFull) throw Error(QE_EINVAL, "sort input too large");
    uint64_t kb[2];
    if (bits) {
        kb[0] = bits[0];
        kb[1] = bits[1];
    } else {
        key_bits_impl(c, keys, n, kb);
    }
    const uint64_t vary = kb[0] & ~kb[1];
    if (!vary) return so;   // every key equal: already sorted (and stable)
    const int lo = __builtin_ctzll(vary), hi = 64 - __builtin_clzll(vary);
    const bool pack = with_vals && hi - lo <= 32;
    int width = 0;
    if (pack) {
        const int mb = sort_maxbits();
        PassDesc pd = plan_passes(kb[0], kb[1], mb, &width);
        const uint64_t fmask = (1ull << (hi - lo)) - 1;   // hi - lo <= 32 here
        Field f{lo, fmask, kb[1] & ~(fmask << lo)};         // constant key bits come back from the AND
        // two-level when the buckets can average well under LDS's TL_CAP = 8192 words (the
        // histogram's maximum decides; a skewed input falls through to the LSD passes)
        const int nb = hi - lo;
        if (two_level_on() && n <= (uint64_t)TL_CAP) {
            // small: one workgroup sorts everything in LDS, rounds of <= 8 bits, one launch
            K* kout = dalloc_t<K>(c, n);
            uint32_t* vout = dalloc_t<uint32_t>(c, n);
            Timed t(c, "sort_small", ((double)sizeof(K) + 4) * 2.0 * n);
            const LocalRounds lr = local_rounds(nb);
            if (vals)
                hipLaunchKernelGGL((tl_local_kernel<K, IN_KV>), dim3(1), dim3(TL_NT), 0, c->stream, nullptr, keys, vals,
                                   kout, vout, nullptr, (uint32_t)n, f, lr);
            else
                hipLaunchKernelGGL((tl_local_kernel<K, IN_KIOTA>), dim3(1), dim3(TL_NT), 0, c->stream, nullptr, keys,
                                   nullptr, kout, vout, nullptr, (uint32_t)n, f, lr);
            QE_HIP(hipGetLastError());
            return SortOut{kout, vout, true, true};
        }
        if (two_level_on() && nb >= 12 && nb <= 8 + 24 && n <= 700000) {   // ~2.7 K per bucket: room for unfilled ranges
            SortOut so2;   // one global pass of 8 bits + LDS buckets (falls through on skew)
            if (sort_two_level<K>(c, keys, vals, n, nb, f, name, &so2, 8)) return so2;
        }
        if (two_level_on() && nb >= 20 && nb <= TL_H + 16 && n >= (1u << 20) && n <= 4000ull * TL_BUCKETS) {
            SortOut so2;
            if (sort_two_level<K>(c, keys, vals, n, nb, f, name, &so2, TL_H, defer)) return so2;
        }
        switch (width <= 8 ? 8 : width) {
        case 8: return sort_packed<K, 8>(c, keys, vals, n, pd, f, name);
        case 9: return sort_packed<K, 9>(c, keys, vals, n, pd, f, name);
        case 10: return sort_packed<K, 10>(c, keys, vals, n, pd, f, name);
        default: return sort_packed<K, 11>(c, keys, vals, n, pd, f, name);
        }
    }
    PassDesc pd = plan_passes(kb[0], kb[1], 8, &width);
    if (!with_vals) {
        if constexpr (sizeof(K) == 8) return sort_keys_only<8>(c, (const uint64_t*)keys, n, pd, name);
        throw Error(QE_EINVAL, "key-only sort needs 64-bit keys");
    }
    return sort_kv_unpacked<K>(c, keys, vals, n, pd, name);
}

SortOut radix_sort_u64(qe_ctx* c, const uint64_t* keys, const uint32_t* vals, uint64_t n, bool with_vals,
                       const uint64_t* bits, bool defer) {
    return radix_sort_impl<uint64_t>(c, keys, vals, n, with_vals, with_vals ? "sort_pass_k64v32" : "sort_pass_k64",
                                     bits, defer && with_vals);
}

SortOut radix_sort_u32(qe_ctx* c, const uint32_t* keys, const uint32_t* vals, uint64_t n, const uint64_t* bits) {
    return radix_sort_impl<uint32_t>(c, keys, vals, n, true, "sort_pass_k32v32", bits);
}

static LocalRounds rounds_of(const DeferredSort& d) {
    LocalRounds lr{d.lr_n, {d.lr_bits[0], d.lr_bits[1], d.lr_bits[2], d.lr_bits[3]}};
    return lr;
}

static void drop(qe_ctx* c, const DeferredSort& d) {
    if (!d.shared) {   // a batch's shared sort (qe_sort_cache): other lanes read it until the batch ends
        dfree(c, d.words);
        dfree(c, d.bstart);
        dfree(c, d.d_max);
    }
    dfree(c, d.x);
    dfree(c, d.x32);
}

// A deferred sort with a bucket beyond LDS (skew) completes by plain LSD passes over the packed
// words' whole field, the last one unpacking into the pairs' key / rowid buffers.  The words are
// bucket-partitioned and stable, so ties keep their input order, as in every other sort path.
static void complete_lsd(qe_ctx* c, const DeferredSort& d, uint64_t n) {
    const int nb = d.L + TL_H;
    PassDesc pd{};
    pd.npass = (nb + 7) / 8;
    const int width = (nb + pd.npass - 1) / pd.npass;
    for (int p = 0; p < pd.npass; p++) {
        pd.shift[p] = 32 + p * width;
        pd.mask[p] = (1u << std::min(width, nb - p * width)) - 1u;
    }
    constexpr int BINS = 256;
    uint32_t* hist = dalloc_t<uint32_t>(c, (size_t)MAX_PASS * BINS);
    hist_and_scan<uint64_t, 8>(c, d.words, n, pd, hist);
    const uint64_t nt = (n + RTILE - 1) / RTILE;
    uint64_t* buf[2] = {dalloc_t<uint64_t>(c, n), pd.npass > 2 ? dalloc_t<uint64_t>(c, n) : nullptr};
    const Field f{d.lo, d.fmask, d.kconst};
    const uint64_t* in = d.words;
    for (int p = 0; p < pd.npass; p++) {
        const bool last = p == pd.npass - 1;
        LBSlot s = lb_acquire(c, nt * BINS);
        Timed t(c, "sort_pass_skew", last ? 8.0 * n + 12.0 * n : 16.0 * n);
        if (last)
            hipLaunchKernelGGL((radix_pass_kernel<uint64_t, IN_WORD, OUT_KV, true, 8, R_ITEMS, R_NT>), dim3((unsigned)nt),
                               dim3(R_NT), 0, c->stream, nullptr, in, nullptr, d.kout, nullptr, d.vout, n, pd.shift[p],
                               pd.mask[p], f, hist + p * BINS, s.status, s.ticket, s.epoch);
        else
            hipLaunchKernelGGL((radix_pass_kernel<uint64_t, IN_WORD, OUT_WORD, true, 8, R_ITEMS, R_NT>),
                               dim3((unsigned)nt), dim3(R_NT), 0, c->stream, nullptr, in, nullptr, nullptr, buf[p & 1],
                               nullptr, n, pd.shift[p], pd.mask[p], f, hist + p * BINS, s.status, s.ticket, s.epoch);
        QE_HIP(hipGetLastError());
        if (!last) in = buf[p & 1];
    }
    dfree(c, hist);
    dfree(c, buf[0]);
    if (buf[1]) dfree(c, buf[1]);
}

// (field << 32 | (uint32_t) val[i]) words of a base column, sorted by the key field
// (key >> lo) & (2^nb - 1): the aggregate join's sides (qe_join_aggregate), whose select column
// rides in the word where the other sorts carry the rowid.  vals == null packs the row index.
uint64_t* sort_words_kv64(qe_ctx* c, const uint64_t* keys, const uint64_t* vals, uint64_t n, int lo, int nb,
                          const uint32_t* vals32) {
    if (n >= 0xFFFFFFFFull) throw Error(QE_EINVAL, "sort input too large");
    PassDesc pd{};
    const uint64_t fmask = nb >= 32 ? 0xFFFFFFFFull : (1ull << nb) - 1;
    if (nb == 0) {   // every key equal: one pass packs the words (digit 0 everywhere, order kept)
        pd.npass = 1;
        pd.shift[0] = lo;
        pd.mask[0] = 0;
    } else {
        pd.npass = (nb + 7) / 8;
        const int width = (nb + pd.npass - 1) / pd.npass;
        for (int p = 0; p < pd.npass; p++) {
            pd.shift[p] = lo + p * width;
            pd.mask[p] = (1u << std::min(width, nb - p * width)) - 1u;
        }
    }
    const Field f{lo, fmask, 0};
    constexpr int BINS = 256;
    uint32_t* hist = dalloc_t<uint32_t>(c, (size_t)MAX_PASS * BINS);
    hist_and_scan<uint64_t, 8>(c, keys, n, pd, hist);
    const uint64_t nt = (n + RTILE - 1) / RTILE;
    uint64_t* buf[2] = {dalloc_t<uint64_t>(c, std::max<uint64_t>(n, 1)),
                        pd.npass > 1 ? dalloc_t<uint64_t>(c, n) : nullptr};
    const uint64_t* win = nullptr;
    for (int p = 0; p < pd.npass; p++) {
        uint64_t* wo = buf[p & 1];
        const int dsh = 32 + pd.shift[p] - lo;
        LBSlot s = lb_acquire(c, nt * BINS);
        Timed t(c, "sort_pass_agg", (p == 0 ? (vals ? 16.0 : vals32 ? 12.0 : 8.0) : 8.0) * n + 8.0 * n);
        if (p > 0)
            hipLaunchKernelGGL((radix_pass_kernel<uint64_t, IN_WORD, OUT_WORD, true, 8, R_ITEMS, R_NT>), dim3((unsigned)nt),
                               dim3(R_NT), 0, c->stream, keys, win, nullptr, nullptr, wo, nullptr, n, dsh, pd.mask[p], f,
                               hist + p * BINS, s.status, s.ticket, s.epoch);
        // the first pass has no earlier order to keep, and the aggregate join needs none among
        // equal keys: unstable ranks there (the later LSD passes must keep theirs)
        else if (vals32)   // (values already narrowed to 32 bits: a bucket's, qe_bucket_select_values)
            hipLaunchKernelGGL((radix_pass_kernel<uint64_t, IN_KV, OUT_WORD, true, 8, R_ITEMS, R_NT, false, false, true>),
                               dim3((unsigned)nt), dim3(R_NT), 0, c->stream, keys, nullptr, vals32, nullptr, wo, nullptr,
                               n, dsh, pd.mask[p], f, hist + p * BINS, s.status, s.ticket, s.epoch);
        else if (vals)
            hipLaunchKernelGGL((radix_pass_kernel<uint64_t, IN_KV64, OUT_WORD, true, 8, R_ITEMS, R_NT, false, false, true>),
                               dim3((unsigned)nt), dim3(R_NT), 0, c->stream, keys, nullptr,
                               reinterpret_cast<const uint32_t*>(vals), nullptr, wo, nullptr, n, dsh, pd.mask[p], f,
                               hist + p * BINS, s.status, s.ticket, s.epoch);
        else
            hipLaunchKernelGGL((radix_pass_kernel<uint64_t, IN_KIOTA, OUT_WORD, true, 8, R_ITEMS, R_NT, false, false, true>),
                               dim3((unsigned)nt), dim3(R_NT), 0, c->stream, keys, nullptr, nullptr, nullptr, wo, nullptr, n,
                               dsh, pd.mask[p], f, hist + p * BINS, s.status, s.ticket, s.epoch);
        QE_HIP(hipGetLastError());
        win = wo;
    }
    dfree(c, hist);
    const int last = (pd.npass - 1) & 1;
    if (buf[last ^ 1]) dfree(c, buf[last ^ 1]);
    return buf[last];
}

// The two global passes of the two-level sort, alone, over (key field << 32 | value) words: the
// words come out partitioned into the TL_BUCKETS buckets of the field's top TL_H bits (bucket b =
// words [bstart[b], bstart[b+1]), no order inside a bucket), lookback-free (tl_hist_tiles_kernel
// counts + column scans).  The aggregate join (qe_agg.hip) needs exactly that: inside a bucket a
// key is its field's L = nb - TL_H low bits, a dense domain it counts in LDS -- no per-bucket
// sort.  Values: a u64 column's low words (v64), u32 (v32), or neither (the row index).
void partition_words_kv(qe_ctx* c, const uint64_t* keys, const uint64_t* v64, const uint32_t* v32, uint64_t n, int lo,
                        int nb, uint64_t** words, uint32_t** bstart_out) {
    if (n == 0 || n >= 0xFFFFFFFFull || nb <= TL_H || nb > TL_H + 16) throw Error(QE_ENOTSUP, "partition geometry");
    const uint64_t fmask = nb >= 32 ? 0xFFFFFFFFull : (1ull << nb) - 1;
    const Field f{lo, fmask, 0};
    const int L = nb - TL_H;
    const uint32_t nt = (uint32_t)((n + RTILE - 1) / RTILE);
    const uint32_t G = (nt + TL_TPG - 1) / TL_TPG;
    const uint32_t Q = G >= 256 ? 1u : 256u / G;
    const uint32_t nseg = 256u * G;
    uint32_t* tcnt = dalloc_t<uint32_t>(c, (size_t)nt * 256);
    uint32_t* gcnt = dalloc_t<uint32_t>(c, (size_t)nseg * 128);
    uint32_t* hist = dalloc_t<uint32_t>(c, TL_BUCKETS);
    uint32_t* bstart = dalloc_t<uint32_t>(c, TL_BUCKETS + 1);
    uint32_t* seg = dalloc_t<uint32_t>(c, (size_t)nseg + 1);
    // base columns with u32 copies (Relation::cols32): the histogram and the first pass read those
    const uint32_t* kn = narrow_of(c, keys, n);
    const uint32_t* vn = v64 ? narrow_of(c, v64, n) : nullptr;
    {
        Timed t(c, "sort_hist", (kn ? 4.0 : 8.0) * n);
        uint32_t* gout = hist_slices(c, gcnt, Q, nseg);
        if (kn)
            hipLaunchKernelGGL((tl_hist_tiles_kernel<uint32_t>), dim3(G * Q), dim3(1024), 0, c->stream, kn, n, f, L, nt,
                               G, Q, tcnt, gout);
        else
            hipLaunchKernelGGL((tl_hist_tiles_kernel<uint64_t>), dim3(G * Q), dim3(1024), 0, c->stream, keys, n, f, L, nt,
                               G, Q, tcnt, gout);
        QE_HIP(hipGetLastError());
        hist_fold(c, gout, Q, G, gcnt, hist);
        hipLaunchKernelGGL(tl_bstart_kernel, dim3(1), dim3(1024), 0, c->stream, hist, bstart, c->d_scratch + 34);
        QE_HIP(hipGetLastError());
    }
    {
        Timed t(c, "sort_scan", 8.0 * ((double)nt * 256 + (double)nseg * 128));
        column_scans(c, tcnt, nt, gcnt, nseg, seg, G, (uint32_t)n);
    }
    uint64_t* w1 = dalloc_t<uint64_t>(c, n);
    uint64_t* w2 = dalloc_t<uint64_t>(c, n);
    {
        Timed t(c, "sort_pass_agg", ((kn ? 4.0 : 8.0) + (vn ? 4.0 : v64 ? 8.0 : v32 ? 4.0 : 0.0) + 8.0) * n);
#define QE_PW1(KT, KP, IN, V)                                                                                            \
    hipLaunchKernelGGL((radix_pass_kernel<KT, IN, OUT_WORD, true, 8, RTILE / pre_nt(true), pre_nt(true) * p1_tm(true, X_NONE), true, X_NONE, true, p1_tm(true, X_NONE)>),        \
                       dim3(xcd_grid((nt + p1_tm(true, X_NONE) - 1) / p1_tm(true, X_NONE))), dim3(pre_nt(true) * p1_tm(true, X_NONE)), 0, c->stream, KP, nullptr, V, nullptr, w1, nullptr, n,         \
                       32 + L, 255u, f, tcnt, nullptr, nullptr, 0u, nullptr, nullptr, nullptr)
        if (kn && (vn || v32)) QE_PW1(uint32_t, kn, IN_KV, vn ? vn : v32);
        else if (kn && !v64) QE_PW1(uint32_t, kn, IN_KIOTA, nullptr);
        else if (v64) QE_PW1(uint64_t, keys, IN_KV64, reinterpret_cast<const uint32_t*>(v64));
        else if (v32) QE_PW1(uint64_t, keys, IN_KV, v32);
        else QE_PW1(uint64_t, keys, IN_KIOTA, nullptr);
#undef QE_PW1
        QE_HIP(hipGetLastError());
    }
    {
        Timed t(c, "sort_pass_agg", 16.0 * n);
        hipLaunchKernelGGL((tl_pass2_kernel<uint64_t, false, true>), dim3(xcd_grid(nseg)), dim3(TL2_NT), 0, c->stream, w1,
                           w2, n, 32 + L + 8, seg, gcnt, G, nullptr, nullptr);
        QE_HIP(hipGetLastError());
    }
    dfree(c, w1);
    dfree(c, tcnt);
    dfree(c, gcnt);
    dfree(c, hist);
    dfree(c, seg);
    *words = w2;
    *bstart_out = bstart;
}

void pairs_need_keys(qe_ctx* c, const qe_pairs* p) {
    if (!p || !p->key) return;
    // keys gathered as u32 for a deferred sort that has not run (PreHist::k32): the u64 buffer is
    // unwritten until widened -- every reader of p->key comes through here, so none sees it
    keys_need_u64(c, p->key);
    auto it = c->deferred.find(p->key);
    if (it == c->deferred.end()) return;
    const DeferredSort d = it->second;
    if (d.w32) throw Error(QE_EINVAL, "internal: a key-only deferred sort has no rows to complete");
    c->deferred.erase(it);
    const Field f{d.lo, d.fmask, d.kconst};
    const uint64_t maxb = read_u64(c, d.d_max);
    if (maxb > (uint64_t)TL_CAP) {
        complete_lsd(c, d, p->n);
    } else {
        Timed t(c, "sort_local", 8.0 * p->n + 12.0 * p->n);
        // (a deferred sort is the plan's: no order among equal keys is needed)
        local_sort_buckets<uint64_t>(c, d.words, d.kout, d.vout, d.bstart, TL_BUCKETS, f, rounds_of(d), maxb,
                                     sort_unstable_on());
    }
    drop(c, d);
}

void pairs_need_vals(qe_ctx* c, const qe_pairs* p) { pairs_need_keys(c, p); }

void pairs_drop_deferred(qe_ctx* c, const qe_pairs* p, bool keep_k32) {
    if (!p || !p->key) return;
    auto ph = c->prehist.find(p->key);   // gathered with a histogram but never sorted (a scan join)
    if (ph != c->prehist.end()) {
        dfree(c, ph->second.tcnt);
        dfree(c, ph->second.gcnt);
        if (keep_k32 && ph->second.k32) {
            ph->second.tcnt = ph->second.gcnt = nullptr;
            ph->second.lo = -1;
        } else {
            if (ph->second.k32) dfree(c, ph->second.k32);
            c->prehist.erase(ph);
        }
    }
    auto it = c->deferred.find(p->key);
    if (it == c->deferred.end()) return;
    drop(c, it->second);
    c->deferred.erase(it);
}

// adopt (DIRECT only, nullable): `rows` are the keys as u32 in a dalloc block the caller hands over --
// they become the PreHist::k32 copy as they are (no write) when the keys are kept as u32; *adopted
// says whether they were (else the caller still owns the block)
static bool gather_hist_impl(qe_ctx* c, const uint64_t* col, const uint32_t* rows, uint64_t n, uint64_t kor,
                             uint64_t kand, uint64_t* keys, const uint32_t* col32 = nullptr, bool adopt = false,
                             bool* adopted = nullptr) {
    if (adopted) *adopted = false;
    // exactly the plan radix_sort_impl will choose for these keys and bounds: the packed
    // two-level sort in its lookback-free form
    if (n < 2 || n >= 0xFFFFFFFFull) return false;
    const uint64_t vary = kor & ~kand;
    if (!vary) return false;
    const int lo = __builtin_ctzll(vary), hi = 64 - __builtin_clzll(vary), nb = hi - lo;
    if (nb > 32 || !two_level_on() || n <= (uint64_t)TL_CAP) return false;
    if (nb >= 12 && nb <= 8 + 24 && n <= 700000) return false;
    if (!(nb >= 20 && nb <= TL_H + 16 && n >= (1u << 20) && n <= 4000ull * TL_BUCKETS)) return false;
    if (!sort_pre_on() || n < sort_pre_min()) return false;
    const uint64_t fmask = (1ull << nb) - 1;
    const Field f{lo, fmask, kand & ~(fmask << lo)};
    const int L = nb - TL_H;
    const uint32_t nt = (uint32_t)((n + RTILE - 1) / RTILE);
    const uint32_t G = (nt + TL_TPG - 1) / TL_TPG;
    const uint32_t Q = G >= 256 ? 1u : 256u / G;
    const uint32_t nseg = 256u * G;
    uint32_t* tcnt = dalloc_t<uint32_t>(c, (size_t)nt * 256);
    uint32_t* gcnt = dalloc_t<uint32_t>(c, (size_t)nseg * 128);
    uint32_t* gout = hist_slices(c, gcnt, Q, nseg);
    // the plan engine's keys below 2^32 are gathered as u32 (PreHist::k32): its deferred sort's
    // first pass reads 4 B per key instead of 8, and the gather writes 4
    const bool keep32 = c->gather_k32 && !(kor >> 32) && gather_k32_on();
    const bool take = adopt && !col && keep32;
    uint32_t* k32 = take ? const_cast<uint32_t*>(rows) : keep32 ? dalloc_t<uint32_t>(c, n) : nullptr;
    if (adopted) *adopted = take;
    const double kw = take ? 0.0 : k32 ? 4.0 : 8.0;
    if (col) {
        Timed t(c, "gather_keys", (col32 ? 8.0 : 12.0) * n + kw * n);
        hipLaunchKernelGGL(tl_gather_hist_kernel<false>, dim3(G * Q), dim3(1024), 0, c->stream, col, rows, n, keys, f, L,
                           nt, G, Q, tcnt, gout, col32, k32);
        QE_HIP(hipGetLastError());
    } else {
        Timed t(c, "widen_keys", 4.0 * n + kw * n);
        hipLaunchKernelGGL(tl_gather_hist_kernel<true>, dim3(G * Q), dim3(1024), 0, c->stream, nullptr, rows, n, keys, f,
                           L, nt, G, Q, tcnt, gout, nullptr, k32);
        QE_HIP(hipGetLastError());
    }
    hist_fold(c, gout, Q, G, gcnt, nullptr);   // (the sort that reads these counts makes the histogram)
    PreHist ph;
    ph.tcnt = tcnt;
    ph.gcnt = gcnt;
    ph.lo = lo;
    ph.L = L;
    ph.fmask = fmask;
    ph.k32 = k32;
    ph.n = n;
    c->prehist[keys] = ph;
    return true;
}

__global__ void __launch_bounds__(256) widen_keys_kernel(const uint32_t* __restrict__ k32, uint64_t n,
                                                         uint64_t* __restrict__ keys) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) keys[i] = k32[i];
}

const uint32_t* keys_pending_u32(qe_ctx* c, const void* keys) {
    auto it = c->prehist.find(keys);
    return it == c->prehist.end() ? nullptr : it->second.k32;
}

void keys_need_u64(qe_ctx* c, const void* keys) {
    auto it = c->prehist.find(keys);
    if (it == c->prehist.end() || !it->second.k32) return;
    PreHist& ph = it->second;
    if (ph.n) {
        Timed t(c, "widen_keys", 12.0 * ph.n);
        hipLaunchKernelGGL(widen_keys_kernel, dim3(grid_for(ph.n, 256 * 8, 8192)), dim3(256), 0, c->stream, ph.k32, ph.n,
                           static_cast<uint64_t*>(const_cast<void*>(keys)));
        QE_HIP(hipGetLastError());
    }
    dfree(c, ph.k32);
    ph.k32 = nullptr;
}

bool gather_with_hist(qe_ctx* c, const uint64_t* col, const uint32_t* rows, uint64_t n, uint64_t kor, uint64_t kand,
                      uint64_t* keys, uint64_t col_rows) {
    return gather_hist_impl(c, col, rows, n, kor, kand, keys, narrow_of(c, col, col_rows));
}

bool widen_with_hist(qe_ctx* c, const uint32_t* vals, uint64_t n, uint64_t kor, uint64_t kand, uint64_t* keys,
                     bool* adopted) {
    return gather_hist_impl(c, nullptr, vals, n, kor, kand, keys, nullptr, adopted != nullptr, adopted);
}

// the bucket geometry radix_sort_impl would give a deferred sort of p (its pass plan, from the
// key bounds), or false when p's sort would not be a deferred two-level one (need_pre: the
// lookback-free form, the only one that carries a payload)
static bool deferred_geometry(const qe_pairs* p, bool need_pre, int* lo, int* nb, uint64_t* kconst) {
    const uint64_t n = p->n;
    if (!(p->flags & QE_PAIRS_BITS) || n < 2 || n >= 0xFFFFFFFFull || !two_level_on() || n <= (uint64_t)TL_CAP)
        return false;
    const uint64_t vary = p->kor & ~p->kand;
    if (!vary) return false;
    *lo = __builtin_ctzll(vary);
    *nb = 64 - __builtin_clzll(vary) - *lo;
    if (*nb > 32) return false;
    if (*nb >= 12 && *nb <= 8 + 24 && n <= 700000) return false;   // the one-pass form
    if (!(*nb >= 20 && *nb <= TL_H + 16 && n >= (1u << 20) && n <= 4000ull * TL_BUCKETS)) return false;
    if (need_pre && !(sort_pre_on() && n >= sort_pre_min())) return false;
    const uint64_t fmask = (1ull << *nb) - 1;
    *kconst = p->kand & ~(fmask << *lo);
    return true;
}

// Two join sides whose key bounds differ (two columns' load-time OR / AND: the C4 batch's key
// columns share one domain but not one maximum) get different bucket geometries, and the join falls
// back to complete sorts + the merge.  Any superset of a side's bounds is valid for its sort, so
// both take the union bounds when each would then still be a deferred two-level sort with an
// in-bucket domain the bucket join holds in LDS.
void unify_geometry(qe_pairs* R, qe_pairs* S) {
    if (!(R->flags & QE_PAIRS_BITS) || !(S->flags & QE_PAIRS_BITS)) return;
    if (R->kor == S->kor && R->kand == S->kand) return;
    if ((R->flags | S->flags) & QE_PAIRS_SORTED) return;
    qe_pairs r = *R, s = *S;
    r.kor = s.kor = R->kor | S->kor;
    r.kand = s.kand = R->kand & S->kand;
    int lo, nb, lo2, nb2;
    uint64_t kc, kc2;
    if (!deferred_geometry(&r, false, &lo, &nb, &kc) || !deferred_geometry(&s, false, &lo2, &nb2, &kc2)) return;
    if (nb - TL_H > HJ_DBITS) return;
    R->kor = S->kor = r.kor;
    R->kand = S->kand = r.kand;
}

bool carry_eligible(const qe_pairs* R, const qe_pairs* S, bool rpay) {
    int loR, nbR, loS, nbS;
    uint64_t kcR, kcS;
    if (!deferred_geometry(R, rpay, &loR, &nbR, &kcR) || !deferred_geometry(S, true, &loS, &nbS, &kcS)) return false;
    return loR == loS && nbR == nbS && kcR == kcS && nbR - TL_H <= HJ_DBITS;
}

bool bucket_join(qe_ctx* c, const qe_pairs* R, const qe_pairs* S, qe_list* outR, qe_list* outS, qe_list* outX0,
                 qe_list* outX1, qe_list* outRX) {
    auto iR = c->deferred.find(R->key), iS = c->deferred.find(S->key);
    if (iR == c->deferred.end() || iS == c->deferred.end() || R->key == S->key) return false;
    const DeferredSort& dR = iR->second;
    const DeferredSort& dS = iS->second;
    if (dR.lo != dS.lo || dR.L != dS.L || dR.fmask != dS.fmask || dR.kconst != dS.kconst || dR.L > HJ_DBITS)
        return false;   // different bucket geometry, or a bucket domain beyond LDS
    if (dR.w32 || dS.w32) return false;   // key-only words: the aggregate form only
    const bool carry = outX0 != nullptr, rx = outRX != nullptr;
    if (carry && !dS.x && !dS.x32) return false;   // S's sort did not carry the payload
    const bool s32 = carry && !dS.x;                // ... or carried one 32-bit column (chain kernel only)
    if (s32 && (outX1 || !hj_chain_on() || dR.L > 12)) return false;
    // R's neither (or no chain kernel to take it, or a 2^13-value bucket domain: 82 KB of LDS)
    if (rx && (!dR.x32 || !hj_chain_on() || dR.L > 12)) return false;
    const uint64_t nR = R->n, nS = S->n;
    uint64_t cap = nR + nS;   // optimistic (fan-out ~1); an outgrown launch re-runs with the exact size
    // (512-thread workgroups taking bucket sides of <= 3584 rows, three per CU, measured 1.63 vs
    // 1.00 ms per C3 query: profiles/r06q_c3_bench.log)
    for (int attempt = 0; attempt < 2; attempt++) {
        uint32_t* oR = dalloc_t<uint32_t>(c, std::max<uint64_t>(cap, 1));
        uint32_t* oS = dalloc_t<uint32_t>(c, std::max<uint64_t>(cap, 1));
        uint32_t* x0 = carry ? dalloc_t<uint32_t>(c, std::max<uint64_t>(cap, 1)) : nullptr;
        uint32_t* x1 = carry && outX1 ? dalloc_t<uint32_t>(c, std::max<uint64_t>(cap, 1)) : nullptr;
        uint32_t* xr = rx ? dalloc_t<uint32_t>(c, std::max<uint64_t>(cap, 1)) : nullptr;
        hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(64), 0, c->stream, c->d_scratch + 17, 2);   // [pairs, oversize]
        QE_HIP(hipGetLastError());
        {
            // algorithmic bytes: both sides' words in (+ 8 B per pair below; + the payloads)
            Timed t(c, "bucket_join", 8.0 * (double)(nR + nS) + (carry ? (s32 ? 4.0 : 8.0) * (double)nS : 0.0) +
                                          (rx ? 4.0 * (double)nR : 0.0));
            // (256-thread workgroups with only the chain in LDS, R's rows read back from global memory at
            // emission: 2.32 vs 1.01 ms per C3 query, profiles/r06k_c3_bench.log -- removed)
            if (s32 && rx) {
                hipLaunchKernelGGL((tl_hjoin_chain_kernel<12, true, true, true>), dim3(hj_grid()), dim3(HJ_NT), 0,
                                   c->stream, dR.words, dR.bstart, dS.words, dS.bstart, dR.L, oR, oS, cap,
                                   c->d_scratch + 17, nullptr, x0, nullptr, dR.x32, xr, dS.x32);
            } else if (s32) {
                hipLaunchKernelGGL((tl_hjoin_chain_kernel<12, true, false, true>), dim3(hj_grid()), dim3(HJ_NT), 0,
                                   c->stream, dR.words, dR.bstart, dS.words, dS.bstart, dR.L, oR, oS, cap,
                                   c->d_scratch + 17, nullptr, x0, nullptr, nullptr, nullptr, dS.x32);
            } else if (rx) {
                const uint64_t* xs = carry ? dS.x : nullptr;
                if (carry)
                    hipLaunchKernelGGL((tl_hjoin_chain_kernel<12, true, true>), dim3(hj_grid()), dim3(HJ_NT), 0,
                                       c->stream, dR.words, dR.bstart, dS.words, dS.bstart, dR.L, oR, oS, cap,
                                       c->d_scratch + 17, xs, x0, x1, dR.x32, xr);
                else
                    hipLaunchKernelGGL((tl_hjoin_chain_kernel<12, false, true>), dim3(hj_grid()), dim3(HJ_NT), 0,
                                       c->stream, dR.words, dR.bstart, dS.words, dS.bstart, dR.L, oR, oS, cap,
                                       c->d_scratch + 17, nullptr, nullptr, nullptr, dR.x32, xr);
            } else if (hj_chain_on()) {
                if (carry && dR.L <= 12)
                    hipLaunchKernelGGL((tl_hjoin_chain_kernel<12, true>), dim3(hj_grid()), dim3(HJ_NT), 0, c->stream,
                                       dR.words, dR.bstart, dS.words, dS.bstart, dR.L, oR, oS, cap, c->d_scratch + 17,
                                       dS.x, x0, x1);
                else if (carry)
                    hipLaunchKernelGGL((tl_hjoin_chain_kernel<HJ_DBITS, true>), dim3(hj_grid()), dim3(HJ_NT), 0,
                                       c->stream, dR.words, dR.bstart, dS.words, dS.bstart, dR.L, oR, oS, cap,
                                       c->d_scratch + 17, dS.x, x0, x1);
                else if (dR.L <= 12)
                    hipLaunchKernelGGL(tl_hjoin_chain_kernel<12>, dim3(hj_grid()), dim3(HJ_NT), 0, c->stream, dR.words,
                                       dR.bstart, dS.words, dS.bstart, dR.L, oR, oS, cap, c->d_scratch + 17);
                else
                    hipLaunchKernelGGL(tl_hjoin_chain_kernel<HJ_DBITS>, dim3(hj_grid()), dim3(HJ_NT), 0, c->stream,
                                       dR.words, dR.bstart, dS.words, dS.bstart, dR.L, oR, oS, cap, c->d_scratch + 17);
            } else if (carry && dR.L <= 12)
                hipLaunchKernelGGL((tl_hjoin_kernel<12, true>), dim3(TL_BUCKETS), dim3(HJ_NT), 0, c->stream, dR.words,
                                   dR.bstart, dS.words, dS.bstart, dR.L, oR, oS, cap, c->d_scratch + 17, dS.x, x0, x1);
            else if (carry)
                hipLaunchKernelGGL((tl_hjoin_kernel<HJ_DBITS, true>), dim3(TL_BUCKETS), dim3(HJ_NT), 0, c->stream,
                                   dR.words, dR.bstart, dS.words, dS.bstart, dR.L, oR, oS, cap, c->d_scratch + 17, dS.x,
                                   x0, x1);
            else if (dR.L <= 12)
                hipLaunchKernelGGL(tl_hjoin_kernel<12>, dim3(TL_BUCKETS), dim3(HJ_NT), 0, c->stream, dR.words, dR.bstart,
                                   dS.words, dS.bstart, dR.L, oR, oS, cap, c->d_scratch + 17);
            else
                hipLaunchKernelGGL(tl_hjoin_kernel<HJ_DBITS>, dim3(TL_BUCKETS), dim3(HJ_NT), 0, c->stream, dR.words,
                                   dR.bstart, dS.words, dS.bstart, dR.L, oR, oS, cap, c->d_scratch + 17);
            QE_HIP(hipGetLastError());
        }
        uint64_t h[2];
        read_words(c, c->d_scratch + 17, h, 2);   // the ONE round trip of the join
        const uint64_t P = h[0];
        if (h[1]) {   // a bucket beyond LDS (skew): the sides complete their sorts, the merge joins them
            dfree(c, oR);
            dfree(c, oS);
            dfree(c, x0);
            dfree(c, x1);
            dfree(c, xr);
            return false;
        }
        if (P <= cap) {
            // the pairs (4 + 4 B) and every carried output column (4 B each) written per pair
            add_bytes(c, "bucket_join", (8.0 + (carry ? 4.0 : 0.0) + (outX1 ? 4.0 : 0.0) + (rx ? 4.0 : 0.0)) * (double)P);
            if (P > c->mat_limit) {   // the reference's DArray cannot hold it either (src/DArray.h:14-15)
                dfree(c, oR);
                dfree(c, oS);
                dfree(c, x0);
                dfree(c, x1);
                dfree(c, xr);
                char msg[160];
                snprintf(msg, sizeof msg, "join of %llu pairs exceeds the materialisation limit %llu",
                         (unsigned long long)P, (unsigned long long)c->mat_limit);
                throw Error(QE_ETOOBIG, msg);
            }
            outR->d = oR;
            outS->d = oS;
            outR->n = outS->n = P;
            outR->cap = outS->cap = cap;
            outR->flags = outS->flags = 0;
            for (auto [ol, xd] : {std::pair<qe_list*, uint32_t*>{outX0, x0}, {outX1, x1}, {outRX, xr}})
                if (ol) {
                    ol->d = xd;
                    ol->n = P;
                    ol->cap = cap;
                    ol->flags = 0;
                }
            return true;
        }
        dfree(c, oR);
        dfree(c, oS);
        dfree(c, x0);
        dfree(c, x1);
        dfree(c, xr);
        cap = P;
    }
    throw Error(QE_EINVAL, "internal: bucket join outgrew its exact size");
}

// ---- the bucket join in aggregate form (the plan's last join, read only by the checksums) ----
// print_sums (src/utilities.c:197-224) reads a finished query's lists only through sums mod 2^64,
// and each S row appears in the join's output once per R partner: so the output's checksum over
// column V of one of S's bindings is sum_s cnt_R(key_s) * V[rowid_s], and its length sum_s cnt_R.
// Per bucket: R's key values counted in LDS (no scan, no scatter of R's rowids), every S row
// looks up its count and gathers its selected values once -- no pairs, no payloads written, no
// checksum pass reading them back.  Each block writes its partial sums (plain stores); a second
// launch adds them up (one atomic per block on one word would serialise at the memory side).
// PERSIST: a resident grid, each workgroup walking buckets blockIdx.x, + gridDim.x, ... with its
// sums kept in registers across them and reduced once (the per-bucket form reduces and stores
// five u64 sums per bucket); part is indexed by workgroup in both forms.
// XK: S's carried payload -- 0 none, 1 u32 (xS32), 2 u64 (xS).  Every S word and payload is held as
// 32-bit halves, so a row's key field dies at its count lookup and no payload register exists when
// no select reads one: with five u64 sums across the walk, the form that held (word, payload) as
// u64 pairs spilled 17 VGPRs at the 64-register occupancy target (0.31 GB of scratch writes per
// C3 launch).
template <bool PERSIST = false, int XK = 2>
__global__ void __launch_bounds__(HJ_NT) __attribute__((amdgpu_waves_per_eu(8)))
tl_hjoin_sums_kernel(const uint64_t* __restrict__ wR, const uint32_t* __restrict__ bsR,
                     const uint64_t* __restrict__ wS, const uint32_t* __restrict__ bsS, int L,
                     const uint64_t* __restrict__ xS, HjSums sc, uint64_t* __restrict__ part,
                     unsigned long long* __restrict__ flag, const uint32_t* __restrict__ xS32, int r32) {
    __shared__ uint32_t cnt[1 << HJ_DBITS];
    __shared__ uint64_t red[HJ_NW][HJ_SUMS + 1];
    const uint32_t D = 1u << L, dmask = D - 1u;
    const int w = wave_id(), l = lane_id();
    // the sums as five named registers: an array of them became one padded 16-VGPR vector
    // register tuple (copied whole on every update) in the persistent loop
    uint64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0, ap = 0;
    static_assert(HJ_SUMS == 4, "one named accumulator per select");
#define QE_ACC(s) (*((s) == 0 ? &a0 : (s) == 1 ? &a1 : (s) == 2 ? &a2 : &a3))
    const uint32_t step = PERSIST ? gridDim.x : (uint32_t)TL_BUCKETS;
    const uint32_t o8 = threadIdx.x * 8u, o4 = threadIdx.x * 4u;   // the loads' only per-lane addressing
    // R's key fields: a u32 array, or the high halves of its u64 words
    const uint32_t rstride = r32 ? 4u : 8u, oR = r32 ? o4 : o8 + 4u;
    for (uint32_t b = blockIdx.x; b < (uint32_t)TL_BUCKETS; b += step) {   // block-uniform
        const uint32_t r0 = bsR[b], mR = bsR[b + 1] - r0, s0 = bsS[b], mS = bsS[b + 1] - s0;
        if (mR > (uint32_t)TL_CAP || mS > (uint32_t)TL_CAP) {   // beyond LDS: the host takes the other path
            if (threadIdx.x == 0) atomicOr(flag, 1ull);
            continue;
        }
        // this bucket's slices as buffer descriptors: rows past the bucket read as 0
        const auto rR = buf_rsrc(reinterpret_cast<const uint32_t*>(wR) + (r32 ? r0 : 2u * r0), mR * rstride);
        const auto rS = buf_rsrc(wS + s0, mS * 8u);
        uint32_t fr[HJ_I];   // R's key fields only (its rows are never read)
        uint32_t fs[HJ_I], sl[HJ_I];   // S's key field, S's word's low half (rowid or value)
        uint32_t xl[XK ? HJ_I : 1], xh[XK == 2 ? HJ_I : 1];   // S's payload halves
#pragma unroll
        for (int j = 0; j < HJ_I; j++) {
            fr[j] = buf_load_u32(rR, oR, (uint32_t)j * HJ_NT * rstride);
            const uint2 ws = buf_load_u2(rS, o8, (uint32_t)j * HJ_NT * 8u);
            fs[j] = ws.y;
            sl[j] = ws.x;
        }
        if constexpr (XK == 1) {
            const auto rX = buf_rsrc(xS32 + s0, mS * 4u);
#pragma unroll
            for (int j = 0; j < HJ_I; j++) xl[j] = buf_load_u32(rX, o4, (uint32_t)j * HJ_NT * 4u);
        }
        if constexpr (XK == 2) {
            const auto rX = buf_rsrc(xS + s0, mS * 8u);
#pragma unroll
            for (int j = 0; j < HJ_I; j++) {
                const uint2 x = buf_load_u2(rX, o8, (uint32_t)j * HJ_NT * 8u);
                xl[j] = x.x;
                xh[j] = x.y;
            }
        }
        if (PERSIST) __syncthreads();   // the previous bucket's lookups are done with cnt
        for (uint32_t v = threadIdx.x; v < D; v += HJ_NT) cnt[v] = 0;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < HJ_I; j++)
            if ((uint32_t)j * HJ_NT + threadIdx.x < mR) atomicAdd(&cnt[fr[j] & dmask], 1u);
        __syncthreads();
        uint32_t c[HJ_I];
#pragma unroll
        for (int j = 0; j < HJ_I; j++) {
            c[j] = (uint32_t)j * HJ_NT + threadIdx.x < mS ? cnt[fs[j] & dmask] : 0u;
            ap += c[j];
        }
#pragma unroll
        for (int s = 0; s < HJ_SUMS; s++) {
            if (s < sc.n) {   // block-uniform
                const uint64_t* __restrict__ col = sc.col[s];
                const int src = sc.src[s] & 3;
                const bool own = (sc.src[s] & 4) != 0;   // the carried list holds the values (QE_PLAN_VALUES_SRC)
                uint32_t id[HJ_I];
#pragma unroll
                for (int j = 0; j < HJ_I; j++) {
                    if constexpr (XK == 0) id[j] = sl[j];
                    else if constexpr (XK == 1) id[j] = src == 0 ? sl[j] : xl[j];
                    else id[j] = src == 0 ? sl[j] : src == 1 ? xl[j] : xh[j];
                }
                if (own) {   // c * value: one 32 x 32 -> 64 multiply-add per row
#pragma unroll
                    for (int j = 0; j < HJ_I; j++) QE_ACC(s) += (uint64_t)c[j] * id[j];
                } else {
                    uint64_t v[HJ_I];
#pragma unroll
                    for (int j = 0; j < HJ_I; j++) v[j] = c[j] ? col[id[j]] : 0ull;   // every gather in flight together
#pragma unroll
                    for (int j = 0; j < HJ_I; j++) QE_ACC(s) += (uint64_t)c[j] * v[j];
                }
            }
        }
    }
#pragma unroll
    for (int s = 0; s <= HJ_SUMS; s++) {
        const uint64_t t = wave_sum_u64(s == HJ_SUMS ? ap : QE_ACC(s));
        if (l == 0) red[w][s] = t;
    }
#undef QE_ACC
    __syncthreads();
    if (threadIdx.x <= HJ_SUMS) {
        uint64_t t = 0;
        for (int ww = 0; ww < HJ_NW; ww++) t += red[ww][threadIdx.x];
        part[(uint64_t)blockIdx.x * (HJ_SUMS + 1) + threadIdx.x] = t;
    }
}

// The aggregate join with small workgroups (the default; QE_HJ_SUMS_SMALL=0: the 1024-thread form
// above): 256 threads, eight resident per CU, each bucket's rows STREAMED in chunks (4 rows a thread
// in flight) instead of held in registers -- a bucket's three barriers stall an eighth of a CU's
// waves, not half of them.  bucket_join_sums 0.373 -> 0.262 ms per C3 query, same box
// (profiles/r06i_c3_bench.log).
#ifndef QE_HJS_NT
#define QE_HJS_NT 256
#endif
#ifndef QE_HJS_U
#define QE_HJS_U 4
#endif
// Both sides' words are read once, as non-temporal loads: bucket_join_sums 0.260-0.265 -> 0.239 ms
// per C3 query, same box, two rounds (profiles/r06ze_c3_bench.log; the next query's filter scan,
// the kernel after it, +0.007).  QE_HJS_NTLOAD=0 (A/B build): default-policy loads.  (The chain
// join's loads as non-temporal: neutral there, and the kernel after it slower -- not used.)
#ifndef QE_HJS_NTLOAD
#define QE_HJS_NTLOAD 1
#endif
#if QE_HJS_NTLOAD
#define QE_HJS_LD(p) __builtin_nontemporal_load(p)
#else
#define QE_HJS_LD(p) (*(p))
#endif
constexpr int HJS_NT = QE_HJS_NT, HJS_NW = HJS_NT / 64, HJS_U = QE_HJS_U;
template <int XK>
__global__ void __launch_bounds__(HJS_NT) __attribute__((amdgpu_waves_per_eu(8)))
tl_hjoin_sums_small_kernel(const uint64_t* __restrict__ wR, const uint32_t* __restrict__ bsR,
                           const uint64_t* __restrict__ wS, const uint32_t* __restrict__ bsS, int L,
                           const uint64_t* __restrict__ xS, HjSums sc, uint64_t* __restrict__ part,
                           unsigned long long* __restrict__ flag, const uint32_t* __restrict__ xS32, int r32) {
    __shared__ alignas(16) uint32_t cnt[1 << 12];
    __shared__ uint64_t red[HJS_NW][HJ_SUMS + 1];
    const uint32_t D = 1u << L, dmask = D - 1u;
    const int w = wave_id(), l = lane_id();
    uint64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0, ap = 0;
#define QE_ACC(s) (*((s) == 0 ? &a0 : (s) == 1 ? &a1 : (s) == 2 ? &a2 : &a3))
    const uint32_t* wR32 = reinterpret_cast<const uint32_t*>(wR);
    for (uint32_t b = blockIdx.x; b < (uint32_t)TL_BUCKETS; b += gridDim.x) {   // block-uniform
        const uint32_t r0 = bsR[b], mR = bsR[b + 1] - r0, s0 = bsS[b], mS = bsS[b + 1] - s0;
        if (mR > (uint32_t)TL_CAP || mS > (uint32_t)TL_CAP) {
            if (threadIdx.x == 0) atomicOr(flag, 1ull);
            continue;
        }
        if (b != blockIdx.x) __syncthreads();   // the previous bucket's lookups are done with cnt
        for (uint32_t v = threadIdx.x * 4u; v < D; v += HJS_NT * 4u)
            *reinterpret_cast<uint4*>(&cnt[v]) = make_uint4(0, 0, 0, 0);
        __syncthreads();
        for (uint32_t i0 = 0; i0 < mR; i0 += HJS_NT * HJS_U) {
            uint32_t f[HJS_U];
#pragma unroll
            for (int u = 0; u < HJS_U; u++) {
                const uint32_t i = i0 + (uint32_t)u * HJS_NT + threadIdx.x;
                f[u] = i < mR ? QE_HJS_LD(r32 ? &wR32[r0 + i] : &wR32[2u * (r0 + i) + 1u]) : 0u;
            }
#pragma unroll
            for (int u = 0; u < HJS_U; u++)
                if (i0 + (uint32_t)u * HJS_NT + threadIdx.x < mR) atomicAdd(&cnt[f[u] & dmask], 1u);
        }
        __syncthreads();
        for (uint32_t i0 = 0; i0 < mS; i0 += HJS_NT * HJS_U) {
            uint64_t ws[HJS_U], xv[HJS_U];
#pragma unroll
            for (int u = 0; u < HJS_U; u++) {
                const uint32_t i = i0 + (uint32_t)u * HJS_NT + threadIdx.x;
                ws[u] = i < mS ? QE_HJS_LD(&wS[s0 + i]) : 0ull;
                if constexpr (XK == 1) xv[u] = i < mS ? QE_HJS_LD(&xS32[s0 + i]) : 0u;
                else if constexpr (XK == 2) xv[u] = i < mS ? QE_HJS_LD(&xS[s0 + i]) : 0ull;
                else xv[u] = 0;
            }
#pragma unroll
            for (int u = 0; u < HJS_U; u++) {
                const uint32_t i = i0 + (uint32_t)u * HJS_NT + threadIdx.x;
                const uint32_t c = i < mS ? cnt[(uint32_t)(ws[u] >> 32) & dmask] : 0u;
                ap += c;
#pragma unroll
                for (int s = 0; s < HJ_SUMS; s++) {
                    if (s < sc.n) {   // block-uniform
                        const int src = sc.src[s] & 3;
                        const uint32_t id = src == 0 ? (uint32_t)ws[u] : src == 1 ? (uint32_t)xv[u] : (uint32_t)(xv[u] >> 32);
                        if (sc.src[s] & 4) QE_ACC(s) += (uint64_t)c * id;
                        else if (c) QE_ACC(s) += (uint64_t)c * sc.col[s][id];
                    }
                }
            }
        }
    }
#pragma unroll
    for (int s = 0; s <= HJ_SUMS; s++) {
        const uint64_t t = wave_sum_u64(s == HJ_SUMS ? ap : QE_ACC(s));
        if (l == 0) red[w][s] = t;
    }
#undef QE_ACC
    __syncthreads();
    if (threadIdx.x <= HJ_SUMS) {
        uint64_t t = 0;
        for (int ww = 0; ww < HJS_NW; ww++) t += red[ww][threadIdx.x];
        part[(uint64_t)blockIdx.x * (HJ_SUMS + 1) + threadIdx.x] = t;
    }
}

// out[k] = sum over blocks of part[b][k] (mod 2^64), one workgroup per k
__global__ void __launch_bounds__(256) hjoin_sums_reduce_kernel(const uint64_t* __restrict__ part, uint32_t nb,
                                                                uint64_t* __restrict__ out) {
    const uint32_t k = blockIdx.x;
    uint64_t t = 0;
    for (uint32_t b = threadIdx.x; b < nb; b += 256) t += part[(uint64_t)b * (HJ_SUMS + 1) + k];
    t = wave_sum_u64(t);
    __shared__ uint64_t red[4];
    if (lane_id() == 0) red[wave_id()] = t;
    __syncthreads();
    if (threadIdx.x == 0) out[k] = red[0] + red[1] + red[2] + red[3];
}

bool bucket_join_sums(qe_ctx* c, const qe_pairs* R, const qe_pairs* S, const HjSums& sc, uint64_t* pairs,
                      uint64_t* sums) {
    auto iR = c->deferred.find(R->key), iS = c->deferred.find(S->key);
    if (iR == c->deferred.end() || iS == c->deferred.end() || R->key == S->key) return false;
    const DeferredSort& dR = iR->second;
    const DeferredSort& dS = iS->second;
    if (dR.lo != dS.lo || dR.L != dS.L || dR.fmask != dS.fmask || dR.kconst != dS.kconst || dR.L > HJ_DBITS)
        return false;
    if (sc.n < 0 || sc.n > HJ_SUMS) return false;
    bool carry = false;
    for (int s = 0; s < sc.n; s++) carry |= (sc.src[s] & 3) != 0;
    if (carry && !dS.x && !dS.x32) return false;   // S's sort did not carry the payload
    if (dS.w32) return false;
    for (int s = 0; s < sc.n; s++)
        if (!dS.x && (sc.src[s] & 3) == 2) return false;   // (a 32-bit payload has no high half)
    uint64_t* part = dalloc_t<uint64_t>(c, (size_t)TL_BUCKETS * (HJ_SUMS + 1));
    uint64_t* out = dalloc_t<uint64_t>(c, 8);   // [pairs-free sums..., pairs, oversize]
    hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(64), 0, c->stream, out, 8);
    QE_HIP(hipGetLastError());
    {
        // algorithmic bytes: R's words (u32 fields when key-only), S's words and carried payload;
        // the gathered select values are added below
        Timed t(c, "bucket_join_sums", (dR.w32 ? 4.0 : 8.0) * (double)R->n + 8.0 * (double)S->n +
                                           (carry ? (dS.x ? 8.0 : 4.0) * (double)S->n : 0.0));
        // a resident grid (two 1024-thread workgroups per CU) walking the buckets, its sums reduced
        // once per workgroup (QE_HJ_SUMS_PERSIST=0: one workgroup per bucket)
        static const uint32_t resident = [&] {
            int ncu = 0;
            QE_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device));
            return (uint32_t)std::max(1, 2 * ncu);
        }();
        static const bool persist = !(getenv("QE_HJ_SUMS_PERSIST") && getenv("QE_HJ_SUMS_PERSIST")[0] == '0');
        const bool small = dR.L <= 12 && !(getenv("QE_HJ_SUMS_SMALL") && getenv("QE_HJ_SUMS_SMALL")[0] == '0');
        // (one barrier per bucket -- three count tables used round robin -- with or without the next
        // bucket's loads in flight at one workgroup per CU measured slower: 0.375 -> 0.424 / 0.431 ms
        // per C3 query, profiles/r06e_c3_bench.log)
        const uint32_t grid = small ? std::min<uint32_t>(resident * (1024 / HJS_NT), TL_BUCKETS)
                              : persist ? std::min<uint32_t>(resident, TL_BUCKETS) : (uint32_t)TL_BUCKETS;
        // S's payload as the kernel holds it: none when no select reads one, else u32 or u64
        const int xk = !carry ? 0 : dS.x32 ? 1 : 2;
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(grid), dim3(HJ_NT), 0, c->stream, dR.words, dR.bstart, dS.words, dS.bstart,
                               dR.L, carry ? dS.x : nullptr, sc, part,
                               reinterpret_cast<unsigned long long*>(out + HJ_SUMS + 1), carry ? dS.x32 : nullptr,
                               dR.w32 ? 1 : 0);
        };
        auto gos = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(grid), dim3(HJS_NT), 0, c->stream, dR.words, dR.bstart, dS.words, dS.bstart,
                               dR.L, carry ? dS.x : nullptr, sc, part,
                               reinterpret_cast<unsigned long long*>(out + HJ_SUMS + 1), carry ? dS.x32 : nullptr,
                               dR.w32 ? 1 : 0);
        };
        if (small)
            xk == 0 ? gos(tl_hjoin_sums_small_kernel<0>) : xk == 1 ? gos(tl_hjoin_sums_small_kernel<1>)
                                                         : gos(tl_hjoin_sums_small_kernel<2>);
        else if (persist)
            xk == 0 ? go(tl_hjoin_sums_kernel<true, 0>) : xk == 1 ? go(tl_hjoin_sums_kernel<true, 1>)
                                                        : go(tl_hjoin_sums_kernel<true, 2>);
        else
            xk == 0 ? go(tl_hjoin_sums_kernel<false, 0>) : xk == 1 ? go(tl_hjoin_sums_kernel<false, 1>)
                                                         : go(tl_hjoin_sums_kernel<false, 2>);
        QE_HIP(hipGetLastError());
        hipLaunchKernelGGL(hjoin_sums_reduce_kernel, dim3(HJ_SUMS + 1), dim3(256), 0, c->stream, part, grid, out);
        QE_HIP(hipGetLastError());
    }
    uint64_t h[HJ_SUMS + 2];
    read_words(c, out, h, HJ_SUMS + 2);   // the ONE round trip of the join and its sums
    dfree(c, part);
    dfree(c, out);
    if (h[HJ_SUMS + 1]) return false;     // a bucket beyond LDS (skew)
    *pairs = h[HJ_SUMS];
    for (int s = 0; s < sc.n; s++) sums[s] = h[s];
    // a select whose values ride in the carried list is summed in place; the others gather one 8-B
    // value per S row with a partner (at most min(pairs, |S|) of them)
    int gathered = 0;
    for (int s = 0; s < sc.n; s++) gathered += sc.col[s] && !(sc.src[s] & 4) ? 1 : 0;   // (4: QE_PLAN_VALUES_SRC)
    add_bytes(c, "bucket_join_sums", 8.0 * gathered * (double)std::min<uint64_t>(h[HJ_SUMS], S->n));
    return true;
}

}  // namespace qe

#ifdef QE_DIAG_STAMPS
extern "C" int qe_diag_stamps_sort(const char* which, uint64_t* out, uint64_t n) {
    if (!strcmp(which, "hj")) return hipMemcpyFromSymbol(out, HIP_SYMBOL(qe::g_hj_stamps), n * 8) == hipSuccess ? 0 : -2;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(qe::g_sort_stamps), n * 8) == hipSuccess ? 0 : -2;
}
#endif
