// qe_scan.hip -- order-preserving stream compaction on gfx950, one pass over HBM.
//
// Used for the filter scan (reference src/filter.c:37-64), the order-preserving filter
// refinement (src/filter.c:3-35, whose O(n^2) DArray_remove it replaces), scan_join
// (src/join.c:395-423) and join_payloads' zero-count pruning.
//
// One workgroup = 256 threads = 4 waves owns a tile of ITEMS x VEC x 256 consecutive elements.
// Each lane loads VEC elements per step with one 16-byte load (coalesced: a wave moves 1 KiB
// per instruction).  Flags are ranked with one ballot per (step, vec slot) + popcount -- no LDS
// scan -- then the tile total goes through a wave-parallel decoupled lookback (qe_device.h) to
// get the tile's output offset.  Survivors are staged in LDS in order and written out as one
// contiguous, coalesced run.  HBM traffic = input bytes + output bytes (+ gathers for refine).
#include "qe_device.h"
#include "qe_internal.h"

namespace qe {

#ifndef QE_CB
#define QE_CB 512
#endif
#ifndef QE_FS_ITEMS
#define QE_FS_ITEMS 12
#endif
constexpr int CB = QE_CB;   // block
constexpr int FS_ITEMS = QE_FS_ITEMS;   // filter scan: steps of 2 x CB rows per tile (12: 3.29 TB/s vs 3.02 at 8, same box)
#ifndef QE_RF_ITEMS
#define QE_RF_ITEMS 8
#endif
#ifndef QE_NZ_ITEMS
#define QE_NZ_ITEMS 8
#endif
constexpr int RF_ITEMS = QE_RF_ITEMS;   // filter refine: steps per tile (TILE = CB * ITEMS * VEC)
constexpr int NZ_ITEMS = QE_NZ_ITEMS;   // join_payloads pruning: steps per tile
constexpr int CNW = CB / 64;

enum { OP_EQ = 0, OP_GT = 1, OP_LT = 2 };

template <int OP>
__device__ __forceinline__ bool cmp_op(uint64_t k, uint64_t v) {
    if (OP == OP_EQ) return k == v;
    if (OP == OP_GT) return k > v;
    return k < v;
}

// ---- element producers ------------------------------------------------------------------------
// load(base, n, f[VEC], v0[VEC], v1[VEC]) for elements base..base+VEC-1 (valid when < n)

template <int OP>
struct FilterScanOp {          // exec_filter_rel_no_exists: rowid i if col[i] op v
    static constexpr int VEC = 2;
    const uint64_t* col;
    uint64_t v;
    __device__ __forceinline__ void load(uint64_t base, uint64_t n, bool* f, uint32_t* v0, uint32_t*) const {
        if (base + 1 < n) {
            ulonglong2 x = *reinterpret_cast<const ulonglong2*>(col + base);
            f[0] = cmp_op<OP>(x.x, v);
            f[1] = cmp_op<OP>(x.y, v);
        } else {
            f[0] = base < n && cmp_op<OP>(col[base], v);
            f[1] = false;
        }
        v0[0] = (uint32_t)base;
        v0[1] = (uint32_t)(base + 1);
    }
};

__device__ __forceinline__ bool cmp_rt(uint32_t op, uint64_t k, uint64_t v) {
    return op == OP_EQ ? k == v : (op == OP_GT ? k > v : k < v);
}

struct FilterScan2Op {         // a scan and a refine of the same binding: rowid i if both hold
    static constexpr int VEC = 2;
    const uint64_t *c1, *c2;
    uint64_t v1, v2;
    uint32_t o1, o2;
    // (second output, when the launch has one: the survivor's c1 value as u32 -- the values a
    // binding read only by selects of c1 carries instead of its rowids, engine `values`)
    __device__ __forceinline__ void load(uint64_t base, uint64_t n, bool* f, uint32_t* v0, uint32_t* vv) const {
        if (base + 1 < n) {
            const ulonglong2 x = *reinterpret_cast<const ulonglong2*>(c1 + base);
            const ulonglong2 y = c2 == c1 ? x : *reinterpret_cast<const ulonglong2*>(c2 + base);
            f[0] = cmp_rt(o1, x.x, v1) && cmp_rt(o2, y.x, v2);
            f[1] = cmp_rt(o1, x.y, v1) && cmp_rt(o2, y.y, v2);
            vv[0] = (uint32_t)x.x;
            vv[1] = (uint32_t)x.y;
        } else {
            const uint64_t x0 = base < n ? c1[base] : 0;
            f[0] = base < n && cmp_rt(o1, x0, v1) && cmp_rt(o2, c2[base], v2);
            f[1] = false;
            vv[0] = (uint32_t)x0;
            vv[1] = 0;
        }
        v0[0] = (uint32_t)base;
        v0[1] = (uint32_t)(base + 1);
    }
};

template <int OP>
struct FilterRefineOp {        // exec_filter_rel_exists: keep rowid r if col[r] op v, in order
    static constexpr int VEC = 4;
    const uint64_t* col;
    const uint32_t* in;
    uint64_t v;
    __device__ __forceinline__ void load(uint64_t base, uint64_t n, bool* f, uint32_t* v0, uint32_t*) const {
        uint32_t r[4];
        if (base + 3 < n) {
            uint4 x = *reinterpret_cast<const uint4*>(in + base);
            r[0] = x.x; r[1] = x.y; r[2] = x.z; r[3] = x.w;
#pragma unroll
            for (int k = 0; k < 4; k++) f[k] = true;
        } else {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                f[k] = base + k < n;
                r[k] = f[k] ? in[base + k] : 0;
            }
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (f[k]) f[k] = cmp_op<OP>(col[r[k]], v);
            v0[k] = r[k];
        }
    }
};

struct ScanJoinOp {            // scan_join: positional key equality, both payloads out
    static constexpr int VEC = 2;
    const uint64_t *rk, *sk;
    const uint32_t *rv, *sv;   // nullable: iota (base column)
    __device__ __forceinline__ void load(uint64_t base, uint64_t n, bool* f, uint32_t* v0, uint32_t* v1) const {
#pragma unroll
        for (int k = 0; k < 2; k++) {
            uint64_t i = base + k;
            bool ok = i < n;
            f[k] = ok && rk[i] == sk[i];
            v0[k] = ok ? (rv ? rv[i] : (uint32_t)i) : 0;
            v1[k] = ok ? (sv ? sv[i] : (uint32_t)i) : 0;
        }
    }
};

struct NonzeroPairsOp {        // join_payloads: keep (last[i], edit[i] or i) whose driver count > 0
    static constexpr int VEC = 4;
    const uint32_t *nz, *last, *edit;   // nz: bit r set <=> count[r] > 0; edit == null: emit i
    uint64_t nzw;                        // words in nz (a rowid past the driver's rows never matches)
    __device__ __forceinline__ void load(uint64_t base, uint64_t n, bool* f, uint32_t* v0, uint32_t* v1) const {
        uint32_t l[4], e[4];
        if (base + 3 < n) {
            uint4 x = *reinterpret_cast<const uint4*>(last + base);
            l[0] = x.x; l[1] = x.y; l[2] = x.z; l[3] = x.w;
            if (edit) {
                uint4 y = *reinterpret_cast<const uint4*>(edit + base);
                e[0] = y.x; e[1] = y.y; e[2] = y.z; e[3] = y.w;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                l[k] = base + k < n ? last[base + k] : 0;
                if (edit) e[k] = base + k < n ? edit[base + k] : 0;
            }
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            uint64_t i = base + k;
            bool ok = i < n;
            f[k] = ok && (l[k] >> 5) < nzw && ((nz[l[k] >> 5] >> (l[k] & 31)) & 1u);
            v0[k] = l[k];
            v1[k] = ok ? (edit ? e[k] : (uint32_t)i) : 0;
        }
    }
};

struct PrefixMaxHitOp {         // unsorted merge: index i where key[i] equals the running max at i
    static constexpr int VEC = 2;   // (and, with `limit`, that max is <= limit)
    const uint64_t *key, *pmax;
    uint64_t limit;
    __device__ __forceinline__ void load(uint64_t base, uint64_t n, bool* f, uint32_t* v0, uint32_t*) const {
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const uint64_t i = base + k;
            const bool ok = i < n;
            const uint64_t m = ok ? pmax[i] : 0;
            f[k] = ok && key[i] == m && m <= limit;
            v0[k] = (uint32_t)i;
        }
    }
};

// ---- the kernel -------------------------------------------------------------------------------
#ifdef QE_DIAG_STAMPS
__device__ uint64_t g_cp_stamps[STAMP_TILES * STAMP_SLOTS];
#endif

template <int ITEMS, int NOUT, class Op>
__global__ void __launch_bounds__(CB) compact_kernel(Op op, uint64_t n, uint32_t ntiles, uint64_t* status,
                                                     uint32_t* ticket, uint32_t epoch, uint32_t* __restrict__ out0,
                                                     uint32_t* __restrict__ out1, uint64_t* total_out) {
    constexpr int VEC = Op::VEC;
    constexpr int TILE = CB * ITEMS * VEC;
    static_assert(ITEMS * CNW <= 128, "one wave scans the (step, wave) table, two entries per lane");
    __shared__ uint32_t s_vals[NOUT][TILE];
    __shared__ uint32_t s_cnt[ITEMS * CNW];
    __shared__ uint32_t s_ticket;
    __shared__ uint64_t s_excl;
    __shared__ uint32_t s_total;

#ifdef QE_DIAG_STAMPS
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
    const uint32_t tile = take_ticket(ticket, &s_ticket);
#ifdef QE_DIAG_STAMPS
    if (threadIdx.x == 0 && tile < STAMP_TILES) g_cp_stamps[(uint64_t)tile * STAMP_SLOTS] = t_start;
#endif
    QE_STAMP(g_cp_stamps, tile, 1);
    const uint64_t tile_base = (uint64_t)tile * TILE;
    const int w = wave_id(), l = lane_id();
    const uint64_t lt = lanemask_lt();

    bool f[ITEMS][VEC];
    uint32_t v0[ITEMS][VEC], v1[ITEMS][VEC];
    uint32_t rank[ITEMS][VEC];
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        uint64_t base = tile_base + (uint64_t)j * (CB * VEC) + (uint64_t)threadIdx.x * VEC;
        op.load(base, n, f[j], v0[j], v1[j]);
    }
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        uint32_t pre = 0, tot = 0;
#pragma unroll
        for (int k = 0; k < VEC; k++) {
            uint64_t m = __ballot(f[j][k]);
            pre += (uint32_t)__popcll(m & lt);
            tot += (uint32_t)__popcll(m);
        }
        uint32_t r = pre;
#pragma unroll
        for (int k = 0; k < VEC; k++) {
            rank[j][k] = r;
            r += f[j][k] ? 1u : 0u;
        }
        if (l == 0) s_cnt[j * CNW + w] = tot;
    }
    __syncthreads();
    QE_STAMP(g_cp_stamps, tile, 2);
    if (w == 0) {
        constexpr uint32_t E = ITEMS * CNW;
        const uint32_t c0 = 2u * l < E ? s_cnt[2 * l] : 0u, c1 = 2u * l + 1 < E ? s_cnt[2 * l + 1] : 0u;
        uint32_t inc = wave_incl_scan_u32(c0 + c1);
        uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        if (2u * l < E) s_cnt[2 * l] = inc - c0 - c1;
        if (2u * l + 1 < E) s_cnt[2 * l + 1] = inc - c1;
        uint64_t excl = lookback_wave(status, epoch, tile, total);
        if (l == 0) {
            s_excl = excl;
            s_total = total;
            if (tile == ntiles - 1) *total_out = excl + total;
        }
    }
    __syncthreads();
    QE_STAMP(g_cp_stamps, tile, 3);
#pragma unroll
    for (int j = 0; j < ITEMS; j++) {
        uint32_t b = s_cnt[j * CNW + w];
#pragma unroll
        for (int k = 0; k < VEC; k++) {
            if (f[j][k]) {
                s_vals[0][b + rank[j][k]] = v0[j][k];
                if (NOUT == 2) s_vals[NOUT - 1][b + rank[j][k]] = v1[j][k];
            }
        }
    }
    __syncthreads();
    QE_STAMP(g_cp_stamps, tile, 4);
    const uint32_t total = s_total;
    const uint64_t off = s_excl;
    for (uint32_t i = threadIdx.x; i < total; i += CB) {
        out0[off + i] = s_vals[0][i];
        if (NOUT == 2) out1[off + i] = s_vals[NOUT - 1][i];
    }
    QE_STAMP(g_cp_stamps, tile, 5);
}

// Persistent, software-pipelined form of compact_kernel: a resident grid of workgroups loops
// over tiles taken by ticket.  Per tile: rank, scan the (step, wave) counts, PUBLISH the tile's
// aggregate, stage the survivors in LDS with tile-local offsets, and only then wait for the
// lookback -- meanwhile waves 1.. already load the next tile (its ticket was taken at the top of
// the iteration), wave 0 after its wait (a wave's loads complete in order, so its polls must not
// queue behind a tile of loads).  The lookback latency, the whole "scan+lookback" phase of the
// one-tile-per-workgroup form (7 of its ~22 us per tile, tools/stamps.py), overlaps HBM loads.
// Deadlock-free by ticket order: a workgroup holds its current tile and the next one, the
// current one taken first, so the smallest unfinished tile is always some workgroup's current
// tile whose predecessors are all complete.
template <int ITEMS, int NOUT, class Op>
__global__ void __launch_bounds__(CB) compact_pipe_kernel(Op op, uint64_t n, uint32_t ntiles, uint64_t* status,
                                                          uint32_t* ticket, uint32_t epoch, uint32_t* __restrict__ out0,
                                                          uint32_t* __restrict__ out1, uint64_t* total_out) {
    constexpr int VEC = Op::VEC;
    constexpr int TILE = CB * ITEMS * VEC;
    static_assert(ITEMS * CNW <= 128, "one wave scans the (step, wave) table, two entries per lane");
    __shared__ uint32_t s_vals[NOUT][TILE];
    __shared__ uint32_t s_cnt[ITEMS * CNW];
    __shared__ uint32_t s_tk[2];
    __shared__ uint64_t s_excl;
    __shared__ uint32_t s_total;
    const int w = wave_id(), l = lane_id();
    const uint64_t lt = lanemask_lt();
    if (threadIdx.x == 0) s_tk[0] = atomicAdd(ticket, 1u);
    __syncthreads();
    uint32_t tile = s_tk[0];
    bool f[ITEMS][VEC];
    uint32_t v0[ITEMS][VEC], v1[ITEMS][VEC];
    auto load_tile = [&](uint32_t t) {
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint64_t base = (uint64_t)t * TILE + (uint64_t)j * (CB * VEC) + (uint64_t)threadIdx.x * VEC;
            op.load(base, n, f[j], v0[j], v1[j]);
        }
    };
    if (tile < ntiles) load_tile(tile);
    int par = 0;
    while (tile < ntiles) {
        QE_STAMP(g_cp_stamps, tile, 0);
        if (threadIdx.x == 0) s_tk[par ^ 1] = atomicAdd(ticket, 1u);   // the next tile, taken early
        uint32_t rank[ITEMS][VEC];
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            uint32_t pre = 0, tot = 0;
#pragma unroll
            for (int k = 0; k < VEC; k++) {
                const uint64_t m = __ballot(f[j][k]);
                pre += (uint32_t)__popcll(m & lt);
                tot += (uint32_t)__popcll(m);
            }
            uint32_t r = pre;
#pragma unroll
            for (int k = 0; k < VEC; k++) {
                rank[j][k] = r;
                r += f[j][k] ? 1u : 0u;
            }
            if (l == 0) s_cnt[j * CNW + w] = tot;
        }
        __syncthreads();   // s_cnt complete, s_tk[par ^ 1] visible
        QE_STAMP(g_cp_stamps, tile, 1);
        if (w == 0) {
            constexpr uint32_t E = ITEMS * CNW;
            const uint32_t c0 = 2u * l < E ? s_cnt[2 * l] : 0u, c1 = 2u * l + 1 < E ? s_cnt[2 * l + 1] : 0u;
            const uint32_t inc = wave_incl_scan_u32(c0 + c1);
            const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
            if (2u * l < E) s_cnt[2 * l] = inc - c0 - c1;
            if (2u * l + 1 < E) s_cnt[2 * l + 1] = inc - c1;
            lookback_publish(status, epoch, tile, total);
            if (l == 0) s_total = total;
        }
        __syncthreads();   // tile-local offsets visible
        QE_STAMP(g_cp_stamps, tile, 2);
#pragma unroll
        for (int j = 0; j < ITEMS; j++) {
            const uint32_t b = s_cnt[j * CNW + w];
#pragma unroll
            for (int k = 0; k < VEC; k++) {
                if (f[j][k]) {
                    s_vals[0][b + rank[j][k]] = v0[j][k];
                    if (NOUT == 2) s_vals[NOUT - 1][b + rank[j][k]] = v1[j][k];
                }
            }
        }
        const uint32_t total = s_total;
        const uint32_t next = s_tk[par ^ 1];
        if (w != 0 && next < ntiles) load_tile(next);   // in flight during the lookback
        if (w == 0) {
            const uint64_t excl = lookback_wait(status, epoch, tile, total);
            if (l == 0) {
                s_excl = excl;
                if (tile == ntiles - 1) *total_out = excl + total;
            }
            if (next < ntiles) load_tile(next);
        }
        __syncthreads();   // staged values and the tile's offset visible
        QE_STAMP(g_cp_stamps, tile, 3);
        const uint64_t off = s_excl;
        for (uint32_t i = threadIdx.x; i < total; i += CB) {
            out0[off + i] = s_vals[0][i];
            if (NOUT == 2) out1[off + i] = s_vals[NOUT - 1][i];
        }
        __syncthreads();   // s_vals / s_cnt / s_tk[par] are rewritten by the next iteration
        QE_STAMP(g_cp_stamps, tile, 4);
        tile = next;
        par ^= 1;
    }
}

static uint32_t op_code(char op);

// ---- wave-tile filter scan ----------------------------------------------------------------------
// The column scans (filter scan, the fused scan + refine, with or without the survivors' values)
// as WAVE-granular tiles: each wave owns WS_STEPS x 64 consecutive rows, loads them all at once
// (one 8-byte element per lane per step: a wave instruction reads 512 contiguous bytes), ranks its
// survivors with one ballot per step (kept in scalar registers), publishes its count, takes its
// exclusive offset from the wave-parallel lookback and stores every step's survivors straight from
// registers -- one instruction per step and output writes popcount(ballot) consecutive words.  No
// LDS, no __syncthreads after the ticket: the four waves of a workgroup are independent, tens of
// thousands of tiles stay in flight, and no phase of one tile waits for another wave's phase.
// Deadlock-free by ticket order: a workgroup's ticket names its four consecutive tiles, and a wave
// waits only for lower tiles, all taken by workgroups already running.
#ifndef QE_WS_STEPS
#define QE_WS_STEPS 32
#endif
constexpr int WS_STEPS = QE_WS_STEPS;
constexpr int WS_B = 256;

template <int STEPS, bool TWO, bool VALS>
__global__ void __launch_bounds__(WS_B) wscan_kernel(FilterScan2Op op, uint64_t n, uint32_t ntiles, uint64_t* status,
                                                    uint32_t* ticket, uint32_t epoch, uint32_t* __restrict__ out0,
                                                    uint32_t* __restrict__ out1, uint64_t* total_out) {
#ifdef QE_DIAG_STAMPS
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#define QE_WSTAMP(k, v)                                                                          \
    do {                                                                                         \
        if (l == 0 && tile < STAMP_TILES) g_cp_stamps[(uint64_t)tile * STAMP_SLOTS + (k)] = (v); \
    } while (0)
#else
#define QE_WSTAMP(k, v) ((void)0)
#endif
    __shared__ uint32_t s_t;
    if (threadIdx.x == 0) s_t = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t tile = s_t * (WS_B / WAVE) + (uint32_t)wave_id();
    if (tile >= ntiles) return;
    const int l = lane_id();
    QE_WSTAMP(0, t_start);
    QE_WSTAMP(1, __builtin_amdgcn_s_memrealtime());
    const uint64_t lt = lanemask_lt();
    const uint64_t base = (uint64_t)tile * (STEPS * WAVE) + (uint64_t)l;
    uint64_t x[STEPS], y[TWO ? STEPS : 1];
#pragma unroll
    for (int j = 0; j < STEPS; j++) {
        const uint64_t i = base + (uint64_t)j * WAVE;
        x[j] = i < n ? __builtin_nontemporal_load(op.c1 + i) : 0;
        if (TWO) y[j] = i < n ? __builtin_nontemporal_load(op.c2 + i) : 0;
    }
    uint64_t m[STEPS];
    uint32_t val[VALS ? STEPS : 1];
    uint32_t total = 0;
#pragma unroll
    for (int j = 0; j < STEPS; j++) {
        const uint64_t i = base + (uint64_t)j * WAVE;
        const bool f = i < n && cmp_rt(op.o1, x[j], op.v1) && cmp_rt(op.o2, TWO ? y[j] : x[j], op.v2);
        m[j] = __ballot(f);
        if (VALS) val[j] = (uint32_t)x[j];
        total += (uint32_t)__popcll(m[j]);
    }
    QE_WSTAMP(2, __builtin_amdgcn_s_memrealtime());
    lookback_publish(status, epoch, tile, total);
    uint64_t off = lookback_wait(status, epoch, tile, total);
    QE_WSTAMP(3, __builtin_amdgcn_s_memrealtime());
    if (tile == ntiles - 1 && l == 0) *total_out = off + total;
    const uint32_t row0 = (uint32_t)base;
#pragma unroll
    for (int j = 0; j < STEPS; j++) {
        if ((m[j] >> l) & 1ull) {
            const uint64_t o = off + (uint64_t)__popcll(m[j] & lt);
            out0[o] = row0 + (uint32_t)(j * WAVE);
            if (VALS) out1[o] = val[j];
        }
        off += (uint64_t)__popcll(m[j]);
    }
    QE_WSTAMP(4, __builtin_amdgcn_s_memrealtime());
#undef QE_WSTAMP
}

static bool wscan_on() {
    static bool on = [] {   // tuning knob: QE_WSCAN=0 keeps the workgroup-tile compaction for scans
        const char* s = getenv("QE_WSCAN");
        return !(s && s[0] == '0');
    }();
    return on;
}

// the scans through wscan_kernel: rowids (and c1's low words when outv) of the rows passing both
// predicates; `bytes` = algorithmic input bytes (4 B per output per survivor added here)
static uint64_t run_wscan(qe_ctx* c, double bytes, const FilterScan2Op& op, uint64_t n, uint32_t* out,
                          uint32_t* outv) {
    if (n == 0) return 0;
    const bool two = op.c2 != op.c1;
    constexpr uint64_t TILE = (uint64_t)WS_STEPS * WAVE;
    const uint64_t nt = (n + TILE - 1) / TILE;
    if (nt >= (1ull << 31)) throw Error(QE_EINVAL, "input too large");
    LBSlot s = lb_acquire(c, nt);
    uint64_t* d_total = c->d_scratch;
    const unsigned grid = (unsigned)((nt + WS_B / WAVE - 1) / (WS_B / WAVE));
    {
        Timed t(c, "filter_scan", bytes);
#define QE_WS_LAUNCH(TWO, VALS)                                                                                \
    hipLaunchKernelGGL((wscan_kernel<WS_STEPS, TWO, VALS>), dim3(grid), dim3(WS_B), 0, c->stream, op, n,       \
                       (uint32_t)nt, s.status, s.ticket, s.epoch, out, outv, d_total)
        if (two) {
            if (outv) QE_WS_LAUNCH(true, true);
            else QE_WS_LAUNCH(true, false);
        } else {
            if (outv) QE_WS_LAUNCH(false, true);
            else QE_WS_LAUNCH(false, false);
        }
#undef QE_WS_LAUNCH
        QE_HIP(hipGetLastError());
    }
    const uint64_t m = read_u64(c, d_total);
    add_bytes(c, "filter_scan", (outv ? 8.0 : 4.0) * m);
    return m;
}

// ---- unordered filter scan (the partitioned plan's) ---------------------------------------------
// The plan's filter lists feed only order-free consumers (key gathers whose sort follows, the
// bucket join, sums): so its scans need no lookback.  Each wave loads its US_STEPS x 64 rows and
// ranks its survivors by ballot as above; the workgroup adds up its waves' counts, reserves its
// output run with ONE atomic on a global counter and every wave stores its part -- no ticket (a
// workgroup waits for nobody: tile = block id), no status words.  The ordered form's per-tile
// time was 38.5 us: 4.2 ticket, 13.7 loads, 15.7 lookback wait, 4.9 stores (tools/stamps.py "ws",
// profiles/r03_wscan_stamps.log).  One atomic per WAVE measured slower than the ordered form
// (0.625 vs 0.347 ms per 1e8 rows, profiles/r03_uscan_wave_ab.log): 48.8 k returning atomics on one
// address serialise at the memory side (~12 ns each), so the reservation is per workgroup of
// US_B / 64 waves.  A run is ascending, the runs are in no particular order.  row_base is added
// to every rowid (a rank's slice numbered globally).
#ifndef QE_US_B
#define QE_US_B 1024
#endif
#ifndef QE_US_STEPS
#define QE_US_STEPS 16
#endif
constexpr int US_B = QE_US_B, US_STEPS = QE_US_STEPS;

// KEYS: a third output -- the survivors' values of another u32 column (kin, the binding's next join
// key: its key side then needs no gather), loaded for the surviving lanes only, right after the
// predicate, so their latency runs under the workgroup's barrier and output reservation
#ifndef QE_USCAN_KEYS_EARLY
#define QE_USCAN_KEYS_EARLY 0
#endif
template <int STEPS, bool TWO, bool VALS, bool KEYS = false>
__global__ void __launch_bounds__(US_B) uscan_kernel(FilterScan2Op op, uint64_t n, uint32_t row_base,
                                                    uint32_t* __restrict__ out0, uint32_t* __restrict__ out1,
                                                    unsigned long long* __restrict__ counter,
                                                    const uint32_t* __restrict__ kin = nullptr,
                                                    uint32_t* __restrict__ out2 = nullptr) {
    constexpr int NW = US_B / WAVE;
    __shared__ uint32_t s_wtot[NW];
    __shared__ uint64_t s_base;
    const int w = wave_id(), l = lane_id();
    const uint64_t tile = (uint64_t)blockIdx.x * NW + (uint64_t)w;
    const uint64_t lt = lanemask_lt();
    const uint64_t base = tile * (STEPS * WAVE) + (uint64_t)l;
    uint64_t x[STEPS], y[TWO ? STEPS : 1];
    uint32_t kv[KEYS ? STEPS : 1];
#pragma unroll
    for (int j = 0; j < STEPS; j++) {
        const uint64_t i = base + (uint64_t)j * WAVE;
        x[j] = i < n ? __builtin_nontemporal_load(op.c1 + i) : 0;
        if (TWO) y[j] = i < n ? __builtin_nontemporal_load(op.c2 + i) : 0;
        // (build knob: every row's key loaded with the predicate columns -- neutral, 0.311-0.312 vs
        // 0.314-0.316 ms of filter_scan per C3 query, profiles/r06n_c3_bench.log)
        if (KEYS && QE_USCAN_KEYS_EARLY) kv[j] = i < n ? kin[i] : 0u;
    }
    uint32_t fb = 0, total = 0;
    uint32_t val[VALS ? STEPS : 1];
#pragma unroll
    for (int j = 0; j < STEPS; j++) {
        const uint64_t i = base + (uint64_t)j * WAVE;
        const bool f = i < n && cmp_rt(op.o1, x[j], op.v1) && cmp_rt(op.o2, TWO ? y[j] : x[j], op.v2);
        fb |= (uint32_t)f << j;
        total += (uint32_t)__popcll(__ballot(f));
        if (VALS) val[j] = (uint32_t)x[j];
    }
    if constexpr (KEYS && !QE_USCAN_KEYS_EARLY) {
#pragma unroll
        for (int j = 0; j < STEPS; j++) kv[j] = (fb >> j) & 1u ? kin[base + (uint64_t)j * WAVE] : 0u;
    }
    if (l == 0) s_wtot[w] = total;
    __syncthreads();
    if (w == 0) {   // the waves' exclusive offsets inside the workgroup's run; one atomic for the run
        const uint32_t c = l < NW ? s_wtot[l] : 0u;
        const uint32_t inc = wave_incl_scan_u32(c);
        const uint32_t sum = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        if (l < NW) s_wtot[l] = inc - c;
        if (l == 0) s_base = sum ? atomicAdd(counter, (unsigned long long)sum) : 0ull;
    }
    __syncthreads();
    uint64_t off = s_base + s_wtot[w];
    if (total == 0) return;
    const uint32_t row0 = (uint32_t)base + row_base;
#pragma unroll
    for (int j = 0; j < STEPS; j++) {
        const bool f = (fb >> j) & 1u;
        const uint64_t m = __ballot(f);
        if (f) {
            const uint64_t o = off + (uint64_t)__popcll(m & lt);
            out0[o] = row0 + (uint32_t)(j * WAVE);
            if (VALS) out1[o] = val[j];
            if constexpr (KEYS) out2[o] = kv[j];
        }
        off += (uint64_t)__popcll(m);
    }
}

uint64_t filter_scan2_unordered(qe_ctx* c, const uint64_t* c1, char op1, uint64_t v1, const uint64_t* c2, char op2,
                                uint64_t v2, uint64_t n, uint32_t row_base, uint32_t* out, uint32_t* outv,
                                const uint32_t* kin, uint32_t* outk) {
    if (n == 0) return 0;
    const FilterScan2Op op{c1, c2, v1, v2, op_code(op1), op_code(op2)};
    static const bool ordered = getenv("QE_PLAN_USCAN") && getenv("QE_PLAN_USCAN")[0] == '0';   // A/B knob
    if (ordered && row_base == 0 && !outk) return run_wscan(c, (c1 == c2 ? 8.0 : 16.0) * n, op, n, out, outv);
    const bool two = c2 != c1;
    constexpr uint64_t TILE = (uint64_t)US_STEPS * US_B;   // rows per workgroup
    const uint64_t nt = (n + TILE - 1) / TILE;
    if (nt >= (1ull << 31)) throw Error(QE_EINVAL, "input too large");
    unsigned long long* d_cnt = reinterpret_cast<unsigned long long*>(c->d_scratch);
    hipLaunchKernelGGL(zero_words_kernel, dim3(1), dim3(64), 0, c->stream, (uint64_t*)d_cnt, 1);
    QE_HIP(hipGetLastError());
    const unsigned grid = (unsigned)nt;
    {
        Timed t(c, "filter_scan", (two ? 16.0 : 8.0) * n);
#define QE_US_LAUNCH(TWO, VALS)                                                                                \
    hipLaunchKernelGGL((uscan_kernel<US_STEPS, TWO, VALS>), dim3(grid), dim3(US_B), 0, c->stream, op, n,       \
                       row_base, out, outv, d_cnt)
#define QE_USK_LAUNCH(TWO, VALS)                                                                               \
    hipLaunchKernelGGL((uscan_kernel<US_STEPS, TWO, VALS, true>), dim3(grid), dim3(US_B), 0, c->stream, op, n, \
                       row_base, out, outv, d_cnt, kin, outk)
        if (outk) {
            if (two && outv) QE_USK_LAUNCH(true, true);
            else if (two) QE_USK_LAUNCH(true, false);
            else if (outv) QE_USK_LAUNCH(false, true);
            else QE_USK_LAUNCH(false, false);
        } else if (two) {
            if (outv) QE_US_LAUNCH(true, true);
            else QE_US_LAUNCH(true, false);
        } else {
            if (outv) QE_US_LAUNCH(false, true);
            else QE_US_LAUNCH(false, false);
        }
#undef QE_US_LAUNCH
#undef QE_USK_LAUNCH
        QE_HIP(hipGetLastError());
    }
    const uint64_t m = read_u64(c, reinterpret_cast<uint64_t*>(d_cnt));
    add_bytes(c, "filter_scan", (4.0 + (outv ? 4.0 : 0.0) + (outk ? 8.0 : 0.0)) * m);   // (keys: 4 B read, 4 written)
    return m;
}

static bool cp_pipe_on() {
    static bool on = [] {   // tuning knob: QE_CP_PIPE=0 keeps one tile per workgroup
        const char* s = getenv("QE_CP_PIPE");
        return !(s && s[0] == '0');
    }();
    return on;
}

#ifdef QE_DIAG_STAMPS
extern "C" int qe_diag_stamps_cp(uint64_t* out, uint64_t n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(qe::g_cp_stamps), n * 8) == hipSuccess ? 0 : -2;
}
#endif

static uint32_t op_code(char op) {
    if (op == '=') return OP_EQ;
    if (op == '>') return OP_GT;
    if (op == '<') return OP_LT;
    throw Error(QE_EINVAL, "Wrong operator");
}

// `bytes` = algorithmic input bytes; 4 B per output list per survivor is added once the count
// is known (SURVEY.md §8(d) byte model).
template <int ITEMS, int NOUT, class Op>
static uint64_t run_compact(qe_ctx* c, const char* name, double bytes, const Op& op, uint64_t n, uint32_t* out0,
                            uint32_t* out1) {
    if (n == 0) return 0;
    constexpr int TILE = CB * ITEMS * Op::VEC;
    uint64_t nt = (n + TILE - 1) / TILE;
    if (nt >= (1ull << 31)) throw Error(QE_EINVAL, "input too large");
    LBSlot s = lb_acquire(c, nt);
    uint64_t* d_total = c->d_scratch;
    if (cp_pipe_on()) {
        static const uint32_t resident = [&] {
            int ncu = 0, per = 0;
            QE_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device));
            QE_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, compact_pipe_kernel<ITEMS, NOUT, Op>, CB, 0));
            return (uint32_t)(std::max(ncu, 1) * std::max(per, 1));
        }();
        const uint32_t grid = (uint32_t)std::min<uint64_t>(nt, resident);
        Timed t(c, name, bytes);
        hipLaunchKernelGGL((compact_pipe_kernel<ITEMS, NOUT, Op>), dim3(grid), dim3(CB), 0, c->stream, op, n,
                           (uint32_t)nt, s.status, s.ticket, s.epoch, out0, out1, d_total);
        QE_HIP(hipGetLastError());
    } else {
        Timed t(c, name, bytes);
        hipLaunchKernelGGL((compact_kernel<ITEMS, NOUT, Op>), dim3((unsigned)nt), dim3(CB), 0, c->stream, op, n,
                           (uint32_t)nt, s.status, s.ticket, s.epoch, out0, out1, d_total);
        QE_HIP(hipGetLastError());
    }
    uint64_t m = read_u64(c, d_total);
    add_bytes(c, name, 4.0 * NOUT * m);
    return m;
}

uint64_t filter_scan(qe_ctx* c, const uint64_t* col, uint64_t n, char op, uint64_t v, uint32_t* out) {
    // read 8 B/row; the 4 B/survivor write is added by the caller-visible count below
    double b = 8.0 * n;
    if (wscan_on()) {   // one predicate: the second is the same comparison of the same word
        const uint32_t o = op_code(op);
        return run_wscan(c, b, FilterScan2Op{col, col, v, v, o, o}, n, out, nullptr);
    }
    uint64_t m;
    switch (op) {
    case '=': m = run_compact<FS_ITEMS, 1>(c, "filter_scan", b, FilterScanOp<OP_EQ>{col, v}, n, out, nullptr); break;
    case '>': m = run_compact<FS_ITEMS, 1>(c, "filter_scan", b, FilterScanOp<OP_GT>{col, v}, n, out, nullptr); break;
    case '<': m = run_compact<FS_ITEMS, 1>(c, "filter_scan", b, FilterScanOp<OP_LT>{col, v}, n, out, nullptr); break;
    default: throw Error(QE_EINVAL, "Wrong operator");
    }
    return m;
}

uint64_t filter_scan2(qe_ctx* c, const uint64_t* c1, char op1, uint64_t v1, const uint64_t* c2, char op2, uint64_t v2,
                      uint64_t n, uint32_t* out) {
    // read 8 B/row per distinct column; 4 B/survivor added below
    const FilterScan2Op o{c1, c2, v1, v2, op_code(op1), op_code(op2)};
    if (wscan_on()) return run_wscan(c, (c1 == c2 ? 8.0 : 16.0) * n, o, n, out, nullptr);
    return run_compact<FS_ITEMS, 1>(c, "filter_scan", (c1 == c2 ? 8.0 : 16.0) * n, o, n, out, nullptr);
}

// the same, with the survivors' c1 values (u32) as a second output; half the tile (two staged
// outputs in the LDS of one)
#ifndef QE_FSV_ITEMS
#define QE_FSV_ITEMS (QE_FS_ITEMS / 2)
#endif
uint64_t filter_scan2_vals(qe_ctx* c, const uint64_t* c1, char op1, uint64_t v1, const uint64_t* c2, char op2,
                           uint64_t v2, uint64_t n, uint32_t* out, uint32_t* outv) {
    const FilterScan2Op o{c1, c2, v1, v2, op_code(op1), op_code(op2)};
    if (wscan_on()) return run_wscan(c, (c1 == c2 ? 8.0 : 16.0) * n, o, n, out, outv);
    return run_compact<QE_FSV_ITEMS, 2>(c, "filter_scan", (c1 == c2 ? 8.0 : 16.0) * n, o, n, out, outv);
}

uint64_t filter_refine(qe_ctx* c, const uint64_t* col, const uint32_t* in, uint64_t n, char op, uint64_t v,
                       uint32_t* out) {
    double b = 12.0 * n;
    switch (op) {
    case '=': return run_compact<RF_ITEMS, 1>(c, "filter_refine", b, FilterRefineOp<OP_EQ>{col, in, v}, n, out, nullptr);
    case '>': return run_compact<RF_ITEMS, 1>(c, "filter_refine", b, FilterRefineOp<OP_GT>{col, in, v}, n, out, nullptr);
    case '<': return run_compact<RF_ITEMS, 1>(c, "filter_refine", b, FilterRefineOp<OP_LT>{col, in, v}, n, out, nullptr);
    default: throw Error(QE_EINVAL, "Wrong operator");
    }
}

uint64_t scan_join_k(qe_ctx* c, const uint64_t* rk, const uint32_t* rv, const uint64_t* sk, const uint32_t* sv,
                     uint64_t n, uint32_t* outR, uint32_t* outS) {
    return run_compact<8, 2>(c, "scan_join", 24.0 * n, ScanJoinOp{rk, sk, rv, sv}, n, outR, outS);
}

uint64_t compact_nonzero_pairs(qe_ctx* c, const uint32_t* nz, uint64_t nzw, const uint32_t* last,
                               const uint32_t* edit, uint64_t n, uint32_t* out_last, uint32_t* out_edit) {
    return run_compact<NZ_ITEMS, 2>(c, "payload_prune", 8.0 * n, NonzeroPairsOp{nz, last, edit, nzw}, n, out_last,
                             out_edit);
}

uint64_t compact_prefix_max_hits(qe_ctx* c, const uint64_t* key, const uint64_t* pmax, uint64_t n, uint64_t limit,
                                 uint32_t* out) {
    return run_compact<4, 1>(c, "seq_merge", 16.0 * n, PrefixMaxHitOp{key, pmax, limit}, n, out, nullptr);
}

}  // namespace qe
