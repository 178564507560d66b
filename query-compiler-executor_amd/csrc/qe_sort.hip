// qe_sort.hip -- stable LSD radix sort of (key, rowid) pairs on gfx950.
//
// Replaces the reference's iterative_sort (MSD radix with a FIFO of buckets, src/join.c:5-94)
// and its randomised quicksort for small buckets (src/quicksort.c:7-64).  The reference's tie
// order depends on rand(); ours is stable (input order), which is one of the orders the
// reference can produce and unobservable on the rand-invariant domain.
//
// Pipeline for n pairs:
//   1. key_bits     -- OR / AND reduction: only bits that vary across keys are sorted
//                      (keys < 2^27 at 100 M rows: 27 bits, 4 passes of <= 8 bits, not 8).
//   2. digit_hist   -- one read of the keys builds the 256-bin histograms of every pass in LDS.
//   3. digit_scan   -- exclusive scan per pass -> global base offset of each digit.
//   4. radix_pass   -- per digit pass, ONE read + ONE write of the pairs: a tile of 256 x ITEMS
//                      pairs is ranked in registers (8 ballots per element = wave match-any,
//                      per-wave LDS counters), per-digit tile totals go through a decoupled
//                      lookback (thread d owns digit d), and the tile is re-ordered by digit
//                      in LDS so the global scatter writes runs of equal digits.
// HBM per pass: 12 B read + 12 B write per pair (u64 key + u32 rowid).
#include <algorithm>

#include "qe_device.h"
#include "qe_internal.h"

namespace qe {

constexpr int RB = 256;          // block
constexpr int RNW = RB / 64;     // waves per block
constexpr int RBINS = 256;       // 8-bit digits (narrower passes use a mask)
constexpr int R_ITEMS = 16;      // pairs per thread per tile
constexpr int RTILE = RB * R_ITEMS;

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
    int shift[8];
    uint32_t mask[8];
};

template <typename K>
__global__ void __launch_bounds__(256) digit_hist_kernel(const K* __restrict__ keys, uint64_t n, PassDesc pd,
                                                         uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[8][RBINS];
    for (int i = threadIdx.x; i < 8 * RBINS; i += blockDim.x) (&h[0][0])[i] = 0;
    __syncthreads();
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint64_t k = (uint64_t)keys[i];
        for (int p = 0; p < pd.npass; p++) atomicAdd(&h[p][(uint32_t)(k >> pd.shift[p]) & pd.mask[p]], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < pd.npass * RBINS; i += blockDim.x) {
        uint32_t v = (&h[0][0])[i];
        if (v) atomicAdd(&hist[i], v);
    }
}

// one block per pass: exclusive scan of 256 counts
__global__ void __launch_bounds__(256) digit_scan_kernel(uint32_t* hist) {
    __shared__ uint32_t wsum[RNW];
    uint32_t* h = hist + blockIdx.x * RBINS;
    uint32_t v = h[threadIdx.x];
    uint32_t inc = wave_incl_scan_u32(v);
    if (lane_id() == 63) wsum[wave_id()] = inc;
    __syncthreads();
    uint32_t add = 0;
    for (int w = 0; w < wave_id(); w++) add += wsum[w];
    h[threadIdx.x] = inc - v + add;
}

template <typename K, bool VIN, bool VOUT>
__global__ void __launch_bounds__(RB) radix_pass_kernel(const K* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                        K* __restrict__ kout, uint32_t* __restrict__ vout, uint64_t n,
                                                        int shift, uint32_t mask,
                                                        const uint32_t* __restrict__ digit_base, uint64_t* status,
                                                        uint32_t* ticket, uint32_t epoch) {
    constexpr int WT = 64 * R_ITEMS;   // pairs per wave
    __shared__ union {
        K keys[RTILE];
        uint32_t vals[RTILE];
    } stage;
    __shared__ uint32_t whist[RNW][RBINS];   // per-wave digit counts -> exclusive over waves
    __shared__ uint32_t bexcl[RBINS];        // tile-local exclusive offset of each digit
    __shared__ uint32_t gofs[RBINS];         // global position of digit run start - bexcl
    __shared__ uint32_t wsum[RNW];
    __shared__ uint32_t s_ticket;

    const uint32_t tile = take_ticket(ticket, &s_ticket);
    const int w = wave_id(), l = lane_id();
    const uint64_t lt = lanemask_lt();
    for (int i = threadIdx.x; i < RNW * RBINS; i += RB) (&whist[0][0])[i] = 0;
    __syncthreads();

    const uint64_t wave_base = (uint64_t)tile * RTILE + (uint64_t)w * WT;
    K key[R_ITEMS];
    uint32_t val[R_ITEMS];
    uint32_t pos[R_ITEMS];
#pragma unroll
    for (int j = 0; j < R_ITEMS; j++) {
        uint64_t i = wave_base + (uint64_t)j * 64 + l;
        bool ok = i < n;
        key[j] = ok ? kin[i] : (K)0;
        if (VOUT) val[j] = VIN ? (ok ? vin[i] : 0u) : (uint32_t)i;
    }
    // rank inside the wave, stable: element order is (j, lane)
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
        pos[j] = old + (uint32_t)__popcll(peers & lt);   // rank within (wave, digit)
    }
    __syncthreads();
    // thread d owns digit d
    const uint32_t d = threadIdx.x;
    uint32_t tot = 0;
#pragma unroll
    for (int ww = 0; ww < RNW; ww++) {
        uint32_t c = whist[ww][d];
        whist[ww][d] = tot;
        tot += c;
    }
    // publish this tile's count of digit d, then look back for the predecessors'
    const uint64_t sidx = (uint64_t)tile * RBINS + d;
    if (tile == 0) st_agent(&status[sidx], lb_word(epoch, LB_FLAG_INC, tot));
    else st_agent(&status[sidx], lb_word(epoch, LB_FLAG_AGG, tot));
    // tile-local exclusive scan over digits
    uint32_t inc = wave_incl_scan_u32(tot);
    if (l == 63) wsum[w] = inc;
    uint64_t excl = 0;
    if (tile > 0) {
        excl = lookback_serial(status, epoch, tile, RBINS, d);
        st_agent(&status[sidx], lb_word(epoch, LB_FLAG_INC, excl + tot));
    }
    __syncthreads();
    uint32_t add = 0;
    for (int ww = 0; ww < w; ww++) add += wsum[ww];
    const uint32_t be = inc - tot + add;
    bexcl[d] = be;
    gofs[d] = digit_base[d] + (uint32_t)excl - be;
    __syncthreads();
    // stage keys in digit order
#pragma unroll
    for (int j = 0; j < R_ITEMS; j++) {
        uint64_t i = wave_base + (uint64_t)j * 64 + l;
        if (i < n) {
            uint32_t dd = (uint32_t)((uint64_t)key[j] >> shift) & mask;
            pos[j] += bexcl[dd] + whist[w][dd];
            stage.keys[pos[j]] = key[j];
        }
    }
    __syncthreads();
    const uint64_t tbase = (uint64_t)tile * RTILE;
    const uint32_t tn = (uint32_t)((n - tbase) < (uint64_t)RTILE ? (n - tbase) : (uint64_t)RTILE);
    uint32_t gp[R_ITEMS];
#pragma unroll
    for (int k = 0; k < R_ITEMS; k++) {
        uint32_t i = (uint32_t)k * RB + threadIdx.x;
        if (i < tn) {
            K kk = stage.keys[i];
            uint32_t dd = (uint32_t)((uint64_t)kk >> shift) & mask;
            gp[k] = gofs[dd] + i;
            kout[gp[k]] = kk;
        }
    }
    if (VOUT) {
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
}

static PassDesc plan_passes(uint64_t kor, uint64_t kand) {
    PassDesc pd{};
    uint64_t vary = kor & ~kand;
    if (!vary) return pd;
    int lo = __builtin_ctzll(vary);
    int hi = 64 - __builtin_clzll(vary);
    int nbits = hi - lo;
    int np = (nbits + 7) / 8;
    int width = (nbits + np - 1) / np;
    pd.npass = np;
    for (int p = 0; p < np; p++) {
        pd.shift[p] = lo + p * width;
        int wbits = std::min(width, hi - pd.shift[p]);
        pd.mask[p] = (1u << wbits) - 1u;
    }
    return pd;
}

template <typename K>
static void key_bits_impl(qe_ctx* c, const K* keys, uint64_t n, uint64_t* out) {
    uint64_t* d_bits = c->d_scratch + 8;   // [or, and]
    uint64_t init[2] = {0ull, ~0ull};
    QE_HIP(hipMemcpyAsync(d_bits, init, sizeof(init), hipMemcpyHostToDevice, c->stream));
    if (n) {
        Timed t(c, "sort_keybits", (double)sizeof(K) * n);
        hipLaunchKernelGGL(key_bits_kernel<K>, dim3(grid_for(n, 256 * 16, 4096)), dim3(256), 0, c->stream, keys,
                           n, d_bits);
        QE_HIP(hipGetLastError());
    }
    read_words(c, d_bits, out, 2);
}

void key_bits_u64(qe_ctx* c, const uint64_t* keys, uint64_t n, uint64_t* out) { key_bits_impl(c, keys, n, out); }

template <typename K>
static SortOut radix_sort_impl(qe_ctx* c, const K* keys, const uint32_t* vals, uint64_t n, bool with_vals,
                               const char* name, const uint64_t* bits) {
    SortOut so{(void*)keys, (uint32_t*)vals, false, false};
    if (n < 2) return so;
    if (n >= 0xFFFFFFFFull) throw Error(QE_EINVAL, "sort input too large");
    uint64_t kb[2];
    if (bits) {
        kb[0] = bits[0];
        kb[1] = bits[1];
    } else {
        key_bits_impl(c, keys, n, kb);
    }
    PassDesc pd = plan_passes(kb[0], kb[1]);
    if (pd.npass == 0) return so;   // every key equal: already sorted (and stable)

    uint32_t* hist = dalloc_t<uint32_t>(c, 8 * RBINS);
    QE_HIP(hipMemsetAsync(hist, 0, 8 * RBINS * sizeof(uint32_t), c->stream));
    {
        Timed t(c, "sort_hist", (double)sizeof(K) * n);
        hipLaunchKernelGGL(digit_hist_kernel<K>, dim3(grid_for(n, 256 * 32, 2048)), dim3(256), 0, c->stream, keys,
                           n, pd, hist);
        QE_HIP(hipGetLastError());
        hipLaunchKernelGGL(digit_scan_kernel, dim3(pd.npass), dim3(256), 0, c->stream, hist);
        QE_HIP(hipGetLastError());
    }
    const uint64_t nt = (n + RTILE - 1) / RTILE;
    K* kbuf[2] = {dalloc_t<K>(c, n), pd.npass > 1 ? dalloc_t<K>(c, n) : nullptr};
    uint32_t* vbuf[2] = {nullptr, nullptr};
    if (with_vals) {
        vbuf[0] = dalloc_t<uint32_t>(c, n);
        if (pd.npass > 1) vbuf[1] = dalloc_t<uint32_t>(c, n);
    }
    const K* kin = keys;
    const uint32_t* vin = vals;
    const double pass_bytes = 2.0 * n * (sizeof(K) + (with_vals ? 4 : 0));
    for (int p = 0; p < pd.npass; p++) {
        K* kout = kbuf[p & 1];
        uint32_t* vout = vbuf[p & 1];
        LBSlot s = lb_acquire(c, nt * RBINS);
        Timed t(c, name, pass_bytes);
        if (!with_vals)
            hipLaunchKernelGGL((radix_pass_kernel<K, false, false>), dim3((unsigned)nt), dim3(RB), 0, c->stream, kin,
                               nullptr, kout, nullptr, n, pd.shift[p], pd.mask[p], hist + p * RBINS, s.status,
                               s.ticket, s.epoch);
        else if (vin)
            hipLaunchKernelGGL((radix_pass_kernel<K, true, true>), dim3((unsigned)nt), dim3(RB), 0, c->stream, kin,
                               vin, kout, vout, n, pd.shift[p], pd.mask[p], hist + p * RBINS, s.status, s.ticket,
                               s.epoch);
        else
            hipLaunchKernelGGL((radix_pass_kernel<K, false, true>), dim3((unsigned)nt), dim3(RB), 0, c->stream, kin,
                               nullptr, kout, vout, n, pd.shift[p], pd.mask[p], hist + p * RBINS, s.status,
                               s.ticket, s.epoch);
        QE_HIP(hipGetLastError());
        kin = kout;
        vin = vout;
    }
    dfree(c, hist);
    int last = (pd.npass - 1) & 1;
    if (pd.npass > 1) {
        dfree(c, kbuf[last ^ 1]);
        if (with_vals) dfree(c, vbuf[last ^ 1]);
    }
    so.keys = kbuf[last];
    so.vals = with_vals ? vbuf[last] : nullptr;
    so.keys_new = true;
    so.vals_new = with_vals;
    return so;
}

SortOut radix_sort_u64(qe_ctx* c, const uint64_t* keys, const uint32_t* vals, uint64_t n, bool with_vals,
                       const uint64_t* bits) {
    return radix_sort_impl<uint64_t>(c, keys, vals, n, with_vals, with_vals ? "sort_pass_k64v32" : "sort_pass_k64",
                                     bits);
}

SortOut radix_sort_u32(qe_ctx* c, const uint32_t* keys, const uint32_t* vals, uint64_t n, const uint64_t* bits) {
    return radix_sort_impl<uint32_t>(c, keys, vals, n, true, "sort_pass_k32v32", bits);
}

}  // namespace qe
