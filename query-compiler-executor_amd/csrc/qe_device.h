// qe_device.h -- device helpers for gfx950 (wave64): lane masks, wave scans, and the
// decoupled-lookback chained scan used by every single-pass compaction / radix pass.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "qe_internal.h"

namespace qe {

constexpr int WAVE = 64;

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }
__device__ __forceinline__ int wave_id() { return (int)(threadIdx.x >> 6); }

__device__ __forceinline__ uint64_t lanemask_lt() {
    int l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    lo = (uint32_t)__shfl((int)lo, src, 64);
    hi = (uint32_t)__shfl((int)hi, src, 64);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    lo = (uint32_t)__shfl_xor((int)lo, m, 64);
    hi = (uint32_t)__shfl_xor((int)hi, m, 64);
    return ((uint64_t)hi << 32) | lo;
}

// A buffer descriptor over [p, p + bytes) built from wave-uniform inputs (readfirstlane'd so the
// compiler can prove it: no waterfall loop around the loads).  Loads through it take a 32-bit
// per-lane byte offset + a scalar one (one VGPR of addressing per stream instead of a 64-bit
// address per load); elements past `bytes` are masked by their kernels.  The raw-buffer range
// check covers the per-lane offset + the instruction's immediate but NOT the scalar soffset
// (ADVICE r4), so a lane may read up to its stride past `bytes`: allowed because every buffer a
// kernel reads is libqe-allocated with DALLOC_SLACK bytes of slack (qe_internal.h).  (Folding
// the stride into the checked offset instead cost pass 1 up to 6 VGPRs and ~2 % of
// sort_pass_carry: profiles/r05d_c3_bench.log.)
typedef unsigned int qe_v2u __attribute__((ext_vector_type(2)));
// cache policy of the streaming buffer loads (build knob, A/B: QE_LOAD_NT=1 marks them
// non-temporal, aux = 2 -- MI355X_MICROARCH "nt-weights": read-once streams land earlier)
#ifndef QE_LOAD_NT
#define QE_LOAD_NT 0
#endif
constexpr int QE_LOAD_AUX = QE_LOAD_NT ? 2 : 0;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, uint32_t bytes) {
    const uint64_t a = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const uint32_t n = __builtin_amdgcn_readfirstlane(bytes);
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, (int)n, 0x00020000);
}
template <int AUX = QE_LOAD_AUX>
__device__ __forceinline__ uint2 buf_load_u2(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    const qe_v2u x = __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, (int)soff, AUX);
    return make_uint2(x.x, x.y);
}
template <int AUX = QE_LOAD_AUX>
__device__ __forceinline__ uint32_t buf_load_u32(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, AUX);
}
typedef unsigned int qe_v4u __attribute__((ext_vector_type(4)));
// (a 16-B load that crosses the end of the range: use it only where the range is whole 16-B units)
__device__ __forceinline__ uint4 buf_load_u4(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    const qe_v4u x = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, QE_LOAD_AUX);
    return make_uint4(x.x, x.y, x.z, x.w);
}

// a few device words zeroed by a kernel of ours instead of a runtime memset (hipMemsetAsync is a
// separate fill launch through the runtime's own path; the small scalar-result words need none)
static __global__ void __launch_bounds__(64) __attribute__((unused)) zero_words_kernel(uint64_t* d, int n) {
    for (int i = threadIdx.x; i < n; i += 64) d[i] = 0;
}

// two device words set from kernel arguments: an [OR, AND] accumulator's start, instead of an
// async copy from a host stack buffer (pageable: the runtime stages it on every call)
static __global__ void __launch_bounds__(64) __attribute__((unused)) set2_kernel(uint64_t* d, uint64_t a, uint64_t b) {
    if (threadIdx.x == 0) {
        d[0] = a;
        d[1] = b;
    }
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += shfl_xor_u64(v, m);
    return v;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += (uint32_t)__shfl_xor((int)v, m, 64);
    return v;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        uint32_t o = (uint32_t)__shfl_xor((int)v, m, 64);
        v = o > v ? o : v;
    }
    return v;
}

// Inclusive wave scans.  QE_DPP_SCAN (default): six DPP adds -- row_shr 1/2/4/8 inside each
// 16-lane row, then row_bcast:15 (rows 1, 3 take row 0's / row 2's total) and row_bcast:31 (rows
// 2, 3 take rows 0-1's total), GFX9's wave64 broadcasts -- no LDS round trip per step; the
// __shfl_up form was six dependent ds_bpermute + waits (~100 cycles each).  A source lane out of
// its row reads 0 (bound_ctrl), a row masked off keeps its value.
#ifndef QE_DPP_SCAN
#define QE_DPP_SCAN 1
#endif
__device__ __forceinline__ uint32_t dpp_add_u32(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);   // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);   // row_bcast:31
    return v;
}
#define QE_DPP64(v, CTRL, RM)                                                                                   \
    do {                                                                                                        \
        const uint32_t lo_ = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v), CTRL, RM, 0xf, false);  \
        const uint32_t hi_ = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)((v) >> 32), CTRL, RM, 0xf, false); \
        (v) += ((uint64_t)hi_ << 32) | lo_;                                                                     \
    } while (0)

// inclusive wave scan (u32); DPP = false: the ds_bpermute form (a kernel at its register limit
// may allocate better around it)
template <bool DPP = (QE_DPP_SCAN != 0)>
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
    if (DPP) return dpp_add_u32(v);
    int l = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t o = (uint32_t)__shfl_up((int)v, d, 64);
        if (l >= d) v += o;
    }
    return v;
}

__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t v) {
    if (QE_DPP_SCAN) {
        QE_DPP64(v, 0x111, 0xf);
        QE_DPP64(v, 0x112, 0xf);
        QE_DPP64(v, 0x114, 0xf);
        QE_DPP64(v, 0x118, 0xf);
        QE_DPP64(v, 0x142, 0xa);
        QE_DPP64(v, 0x143, 0xc);
        return v;
    }
    int l = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v, d, 64);
        uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), d, 64);
        uint64_t o = ((uint64_t)hi << 32) | lo;
        if (l >= d) v += o;
    }
    return v;
}

__device__ __forceinline__ uint64_t ld_agent(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// status word = [epoch:16 | flag:2 | value:46]: one 8-byte agent-scope store carries both the
// value and its flag (the data is the flag, MI355X_MICROARCH "R2 granule"), so no fence is
// needed and a word from an older launch (other epoch) reads as "not ready".
__device__ __forceinline__ uint64_t lb_word(uint32_t epoch, uint64_t flag, uint64_t v) {
    return ((uint64_t)epoch << 48) | (flag << 46) | (v & LB_VAL_MASK);
}
__device__ __forceinline__ uint32_t lb_flag(uint64_t w, uint32_t epoch) {
    return ((uint32_t)(w >> 48) == epoch) ? (uint32_t)((w >> 46) & 3u) : 0u;
}

// Dynamic tile id: blocks take tickets in the order they start, so every predecessor of a
// running tile is itself resident -- the lookback below cannot deadlock whatever the
// dispatch order (cdna_hip_programming.md §1: dispatch order is undefined).
__device__ __forceinline__ uint32_t take_ticket(uint32_t* ticket, uint32_t* lds_slot) {
    if (threadIdx.x == 0) *lds_slot = atomicAdd(ticket, 1u);
    __syncthreads();
    uint32_t t = *lds_slot;
    return t;
}

// Wave-parallel lookback for ONE running total per tile, in two halves so a tile can publish its
// aggregate early and do independent work (e.g. stage its output in LDS) before it waits.
__device__ __forceinline__ void lookback_publish(uint64_t* status, uint32_t epoch, uint32_t tile, uint64_t agg) {
    if (lane_id() == 0) st_agent(&status[tile], lb_word(epoch, tile == 0 ? LB_FLAG_INC : LB_FLAG_AGG, agg));
}

// called by a whole wave after lookback_publish; returns the exclusive prefix (same in every
// lane) and publishes the inclusive one.  Each step reads LB_K predecessors per lane (64 x LB_K
// tiles per step).  Measured on MI355X (filter scan, 1e8 rows, persistent grid): LB_K = 1
// 0.321 ms, 4 0.392 ms, 8 0.464 ms -- wider polls cost more in traffic than they save in steps.
#ifndef QE_LB_K
#define QE_LB_K 1
#endif
constexpr int LB_K = QE_LB_K;
__device__ __forceinline__ uint64_t lookback_wait(uint64_t* status, uint32_t epoch, uint32_t tile, uint64_t agg) {
    const int l = lane_id();
    if (tile == 0) return 0;
    uint64_t excl = 0;
    int64_t base = (int64_t)tile - 1;
    for (;;) {
        // lane l looks at tiles base - (l * LB_K + q), q < LB_K; only the words up to the nearest
        // inclusive prefix matter, so a slow tile further back never holds this one up
        uint64_t w[LB_K];
        int qi, first;
        uint32_t spins = 0;
        for (;;) {
            uint32_t fl[LB_K];
#pragma unroll
            for (int q = 0; q < LB_K; q++) {
                const int64_t idx = base - (int64_t)(l * LB_K + q);
                if (idx >= 0) {
                    w[q] = ld_agent(&status[idx]);
                    fl[q] = lb_flag(w[q], epoch);
                } else {
                    w[q] = 0;
                    fl[q] = (uint32_t)LB_FLAG_INC;
                }
            }
            qi = LB_K;   // this lane's nearest inclusive prefix
            bool blocked = false;
#pragma unroll
            for (int q = 0; q < LB_K; q++) {
                if (qi == LB_K && fl[q] == (uint32_t)LB_FLAG_INC) qi = q;
                if (qi == LB_K && fl[q] == 0) blocked = true;   // not published, before any prefix
            }
            const uint64_t inc = __ballot(qi < LB_K);
            first = inc ? (__ffsll((unsigned long long)inc) - 1) : 64;
            const uint64_t need = first >= 63 ? ~0ull : ((2ull << first) - 1);   // lanes 0..first
            if (!(__ballot(blocked) & need)) break;
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1u << 24)) break;   // bounded spin: never hang the GPU
        }
        uint64_t v = 0;
        const int upto = l < first ? LB_K : (l == first ? qi + 1 : 0);
#pragma unroll
        for (int q = 0; q < LB_K; q++)
            if (q < upto) v += w[q] & LB_VAL_MASK;
        excl += wave_sum_u64(v);
        if (first < 64) break;
        base -= 64 * LB_K;
    }
    if (l == 0) st_agent(&status[tile], lb_word(epoch, LB_FLAG_INC, excl + agg));
    return excl;
}

__device__ __forceinline__ uint64_t lookback_wave(uint64_t* status, uint32_t epoch, uint32_t tile,
                                                  uint64_t agg) {
    lookback_publish(status, epoch, tile, agg);
    return lookback_wait(status, epoch, tile, agg);
}

// Thread-serial lookback for one of many per-tile totals (radix digits): `stride` words per
// tile, this thread owns column `col`.  The aggregate must already be published.
// Each step reads the next LB_WIN predecessors' words at once (independent loads in flight), so
// a walk over k aggregate-only tiles costs ~k/LB_WIN load latencies instead of k.
#ifndef QE_LB_WIN
#define QE_LB_WIN 8
#endif
constexpr int LB_WIN = QE_LB_WIN;
template <int WIN = LB_WIN>
__device__ __forceinline__ uint64_t lookback_serial(uint64_t* status, uint32_t epoch, uint32_t tile,
                                                    uint32_t stride, uint32_t col, uint32_t* diag = nullptr) {
    uint64_t excl = 0;
    int64_t idx = (int64_t)tile - 1;
    uint32_t spins = 0, rounds = 0;
    while (idx >= 0) {
        rounds++;
        uint64_t w[WIN];
#pragma unroll
        for (int q = 0; q < WIN; q++)
            w[q] = idx - q >= 0 ? ld_agent(&status[(uint64_t)(idx - q) * stride + col])
                                : lb_word(epoch, LB_FLAG_INC, 0);
        int used = 0;
        bool done = false, stall = false;
#pragma unroll
        for (int q = 0; q < WIN; q++) {
            if (done || stall) continue;
            uint32_t f = lb_flag(w[q], epoch);
            if (f == 0) {
                stall = true;       // predecessor idx - q has not published yet: re-poll from there
                continue;
            }
            excl += w[q] & LB_VAL_MASK;
            used++;
            if (f == LB_FLAG_INC) done = true;
        }
        if (done) break;
        idx -= used;
        if (stall) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1u << 24)) break;   // bounded spin: never hang the GPU
        }
    }
    if (diag) {   // tuning builds: load rounds, stalled rounds, tiles walked
        diag[0] = rounds;
        diag[1] = spins;
        diag[2] = (uint32_t)((int64_t)tile - 1 - idx);
    }
    return excl;
}

// Phase timestamps for tuning builds only (tools/build_variant.sh NAME -DQE_DIAG_STAMPS):
// thread 0 of a tile records s_memrealtime (100 MHz) after each barrier-separated phase.
#ifdef QE_DIAG_STAMPS
constexpr uint32_t STAMP_TILES = 1u << 16, STAMP_SLOTS = 8;
#define QE_STAMP(arr, tile, k)                                                        \
    do {                                                                              \
        if (threadIdx.x == 0 && (tile) < STAMP_TILES)                                 \
            (arr)[(uint64_t)(tile) * STAMP_SLOTS + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define QE_STAMP(arr, tile, k) ((void)0)
#endif

}  // namespace qe
