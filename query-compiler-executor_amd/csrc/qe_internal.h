// qe_internal.h -- shared internals of libqe (HIP C++ for gfx950).  Not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <map>
#include <stdexcept>
#include <string>
#include <unordered_set>
#include <unordered_map>
#include <vector>

#include "../../include/qe.h"

namespace qe {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define QE_HIP(call)                                                                           \
    do {                                                                                       \
        hipError_t e_ = (call);                                                                \
        if (e_ != hipSuccess)                                                                  \
            throw ::qe::Error(QE_EHIP, std::string(#call) + ": " + hipGetErrorString(e_));    \
    } while (0)

struct Relation {
    uint64_t rows = 0;
    bool owned = true;                 // false: another ctx's columns, shared (qe_workers)
    std::vector<uint64_t*> cols;
    std::vector<uint64_t> kor, kand;   // column statistics: OR / AND of all values (at load)
    // the same columns as u32 where every value fits (the OR below 2^32), else null: what the
    // sorts' first passes and histograms read -- half the bytes of the u64 column
    std::vector<uint32_t*> cols32;
};

struct PendingEvent {
    int kernel;
    hipEvent_t a, b;
    double bytes;
};

struct KStat {
    std::string name;
    uint64_t launches = 0;
    double ms = 0, bytes = 0;
};

// Status words of the decoupled-lookback scans: [epoch:16 | flag:2 | value:46].
constexpr uint64_t LB_FLAG_AGG = 1ull;
constexpr uint64_t LB_FLAG_INC = 2ull;
constexpr int LB_VAL_BITS = 46;
constexpr uint64_t LB_VAL_MASK = (1ull << LB_VAL_BITS) - 1;
constexpr int LB_MAX_COUNTERS = 65536;

// merge-join flags (one word per launch): R row with > 1 partner, S row with > 1 partner,
// internal error, 46-bit lookback sum overflow
enum : uint32_t { MJF_R_FANOUT = 1u, MJF_S_DUP = 2u, MJF_ERR = 4u, MJF_OVF = 8u };

// A two-level sort whose last step (the per-bucket LDS sort) has not run yet: the pairs' key /
// val buffers are allocated but unfilled, the bucket-partitioned packed words are kept.  An
// unordered join of two such sides with the same bucket geometry runs per bucket (bucket_join);
// anything else that reads the pairs first completes the sort (pairs_need_keys).
struct DeferredSort {
    uint64_t* words = nullptr;    // bucket-partitioned (field << 32 | rowid) words
    uint32_t* bstart = nullptr;   // bucket starts (+ end)
    uint64_t* d_max = nullptr;    // largest bucket (device word: > TL_CAP = skew, not yet checked)
    uint64_t* x = nullptr;        // carried payloads, in the words' order (qe_join_carry), or null
    uint32_t* x32 = nullptr;      // a 32-bit payload in the words' order (R's next join key), or null
    const uint64_t* v64 = nullptr;   // the words hold this column's low words, not row indices
    bool w32 = false;             // the words are u32 key fields only (no rows: bucket_join_sums' R)
    uint64_t* kout = nullptr;
    uint32_t* vout = nullptr;
    int lo = 0, L = 0;            // field = (key >> lo) & fmask; bucket = field >> L
    uint64_t fmask = 0, kconst = 0;
    int lr_n = 0, lr_bits[4] = {0, 0, 0, 0};
    bool shared = false;          // words / bstart / d_max belong to a batch's SortCache (not freed by drop)
};

// The two-level sort's histogram, computed while the keys were gathered (gather_with_hist): the
// sort of those keys skips its histogram read.  Kept by the pairs' key buffer.
// A batch's shared sorts of whole base columns (qe_sort_cache, qe_join.hip): one per (column,
// form), built by the first lane that needs it, read by every later join of the batch.
struct SortCache;

struct PreHist {
    uint32_t* tcnt = nullptr;   // per first-pass tile digit counts
    uint32_t* gcnt = nullptr;   // per (digit, group) segment digit counts
    int lo = 0, L = 0;
    uint64_t fmask = 0;
    // the keys as u32 (keys below 2^32, gathered for the plan's deferred sort): the u64 key buffer
    // was NOT written -- its sort's first pass reads these; anything else that reads the keys
    // calls keys_need_u64 first, which widens them into the buffer
    uint32_t* k32 = nullptr;
    uint64_t n = 0;
};

}  // namespace qe

// The per-stream working state queued work addresses: the stream, its lookback status words and
// tickets, scalar scratch and result words.  A ctx owns two: the main one (in the ctx's own fields)
// and a side one (qe_ctx::side) that SideFork (qe_join.hip) swaps in while one join side's sort is
// queued on the side stream, concurrently with the other side's.
struct StreamState {
    hipStream_t stream = nullptr;
    uint64_t* lb_status = nullptr;
    size_t lb_status_words = 0;
    uint32_t* lb_tickets = nullptr;
    uint32_t lb_epoch = 0;
    uint64_t* d_scratch = nullptr;
    uint32_t* d_zhist = nullptr;
    bool zhist_dirty = false;
    uint64_t* h_scratch = nullptr;
    hipEvent_t wait_ev = nullptr;
    uint64_t* h_ret = nullptr;
    uint64_t* d_ret = nullptr;
    uint64_t ret_seq = 0;
};

struct qe_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // the side stream's state (swapped with the fields above while a side is queued on it), and
    // the frees held back while two streams run: a block freed by one stream's queued work must
    // not be handed to the other stream's before they meet (released by SideFork::join)
    StreamState side;
    bool side_in = false;      // the side state is the one in the ctx's fields
    int hold_frees = 0;
    std::vector<void*> held;
    hipEvent_t fork_ev[2] = {nullptr, nullptr};
    std::string err;
    std::string late_err;   // an internal violation found where no throw is allowed (dfree), surfaced later

    // caching device allocator: exact size classes, stream-ordered reuse on the one stream
    std::multimap<size_t, void*> free_blocks;
    std::unordered_map<void*, size_t> live;
    std::unordered_map<void*, void*> pad_base;   // QE_ALLOC_PAD: offset block -> its hipMalloc base
    // qe_partition_columns: every base column's hash bucket `bparts_p` of `bparts_n`, by column
    std::unordered_map<const uint64_t*, qe_pairs> bparts;
    uint32_t bparts_n = 0, bparts_p = 0;
    uint64_t in_use = 0, cached = 0;

    std::vector<qe::Relation> rels;
    uint64_t last_result_rows = 0;
    // joins larger than this many pairs are not materialised (QE_ETOOBIG): the reference's
    // DArray holds at most INT32_MAX elements (src/DArray.h:14-15).  QE_MAT_LIMIT overrides.
    uint64_t mat_limit = 0x7FFFFFFFull;
    // Zipf sampling table (qe_set_zipf_table): CDF borrowed from the caller, guide owned
    const double* zipf_cdf = nullptr;
    uint64_t* zipf_guide = nullptr;
    double* zipf_owned = nullptr;     // the CDF when qe_set_zipf built it
    uint64_t zipf_domain = 0, zipf_perm_seed = 0;

    // decoupled-lookback state: status words + per-launch tile tickets, epoch-tagged so that
    // nothing is cleared between launches (cleared when the 16-bit epoch wraps)
    uint64_t* lb_status = nullptr;
    size_t lb_status_words = 0;
    uint32_t* lb_tickets = nullptr;
    uint32_t lb_epoch = 0;

    // small device scratch + pinned host mirror for scalar results
    uint64_t* d_scratch = nullptr;   // 64 words
    uint32_t* d_zhist = nullptr;     // the lookback-form sorts' histograms (32 K + 256 words), left zeroed by their scans
    bool zhist_dirty = false;        // set from a histogram launch until its scan is queued (a throw between: clear first)
    uint64_t* h_scratch = nullptr;   // pinned, 64 words
    hipEvent_t wait_ev = nullptr;    // polled for scalar results (read_u64 / read_words, QE_WAIT=event)
    // device blocks a batch's shared sort holds (qe_sort_cache): dfree of one of them is a bug
    // (a lane returning shared words to its allocator while other lanes read them -- the round-3
    // fault) and throws instead of recycling the block
    std::unordered_set<const void*> pinned;
    uint64_t* h_ret = nullptr;       // pinned coherent host words: [0] = sequence flag, [1..] = the result
    uint64_t* d_ret = nullptr;       // (h_ret as the device addresses it)
    uint64_t ret_seq = 0;            // the last sequence number published

    // loader (qe_load_relation): pinned staging ring for pageable host columns
    static constexpr int STAGE_SLOTS = 3;
    void* h_stage[STAGE_SLOTS] = {nullptr, nullptr, nullptr};
    hipEvent_t stage_ev[STAGE_SLOTS] = {nullptr, nullptr, nullptr};
    size_t stage_bytes = 0;
    double load_s = 0, load_bytes = 0;   // wall time / bytes of host -> HBM loads so far

    // two-level sorts awaiting their per-bucket step, by the pairs' key buffer
    std::unordered_map<const void*, qe::DeferredSort> deferred;
    std::unordered_map<const void*, qe::PreHist> prehist;

    // worker contexts on the same device (qe_workers): their own stream and allocator, this ctx's
    // relations shared -- the concurrent batch executor's lanes
    std::vector<qe_ctx*> workers;
    // the batch's shared base-column sorts (qe_sort_cache; null: off), this ctx's and its workers'
    qe::SortCache* scache = nullptr;
    uint64_t scache_hits = 0, scache_builds = 0;   // over this ctx's finished batches

    // profiling
    bool prof = false;
    std::string prof_only;           // non-empty: only this stage is timed (qe_set_profiling_only)
    // a payload for the next deferred lookback-free two-level sort to carry (join_pairs_carry)
    const uint32_t* carry_xa = nullptr;
    const uint32_t* carry_xb = nullptr;
    // ... or one 32-bit payload: a u32 array, or a u64 column's low words (row i = input element i)
    const uint32_t* carry_x32 = nullptr;
    const uint64_t* carry_c64 = nullptr;
    // ... and for a sort without vals: pack this u64 column's low words instead of the row index
    const uint64_t* sort_v64 = nullptr;
    // ... or keep the key fields only (u32 words): the next deferred sort's rows are never read
    bool sort_keys_only = false;
    bool gather_k32 = false;   // (set by the plan engine around its key gathers: see PreHist::k32)
    std::vector<qe::PendingEvent> pending;
    std::vector<hipEvent_t> event_pool;
    std::vector<qe::KStat> kstats;
    std::map<std::string, int> kindex;
};

namespace qe {

// the u32 copy of a loaded relation's column (by its u64 pointer and length), or null
inline const uint32_t* narrow_of(const qe_ctx* c, const void* col, uint64_t n) {
    if (!col) return nullptr;
    for (const auto& r : c->rels)
        if (r.rows == n)
            for (size_t j = 0; j < r.cols.size() && j < r.cols32.size(); j++)
                if (r.cols[j] == col) return r.cols32[j];
    return nullptr;
}

// every data buffer a kernel reads through the soffset-strided buffer loads (qe_device.h) is
// libqe's own -- a dalloc block, a relation column or its u32 copy (no entry point takes a caller's
// device pointer) -- and each is followed by DALLOC_SLACK allocated bytes: such a load may read up
// to a tile's stride past a buffer's end, never past its allocation (the strides are checked
// against it by a static_assert in qe_sort.hip).  The few fixed-size control words allocated with
// a plain hipMalloc (lookback status, tickets, scratch, the zero histogram, the comm's reduction
// words) are read only by ordinary indexed loads within their sizes
constexpr size_t DALLOC_SLACK = 64u << 10;
void* dalloc(qe_ctx* c, size_t bytes);
bool alloc_log_on();   // QE_ALLOC_LOG=1 (placement A/Bs)
void drop_partitions(qe_ctx* c);   // qe_partition_columns' buckets freed
void dfree(qe_ctx* c, void* p);
template <class T>
T* dalloc_t(qe_ctx* c, size_t n) { return static_cast<T*>(dalloc(c, n * sizeof(T))); }

// one epoch per lookback launch: returns (status base, ticket counter, epoch tag)
struct LBSlot {
    uint64_t* status;
    uint32_t* ticket;
    uint32_t epoch;
};
LBSlot lb_acquire(qe_ctx* c, size_t words);

// One join side's sort queued on the ctx's side stream while the other side's sort is queued on the
// ctx stream, so the two run concurrently (a histogram's LDS atomics, a gather's latency and the
// small scan launches of one side beside the other's streaming passes).
//   SideFork f(c, big);  f.enter(); <queue side A>  f.leave();  <queue side B>  f.join();  <consumer>
// The side stream waits for the ctx stream's work queued before the fork; join() makes the ctx
// stream wait for the side stream's; frees in between are held and recycled at join() (a block one
// stream frees must not be reused by the other's queued work).  The side state (stream, lookback
// words, scratch, result words) is swapped into the ctx's fields between enter() and leave(), so
// everything queued there addresses it unchanged.  The destructor joins.  QE_SIDE_STREAM=1: on
// (off by default: see side_stream_on).
struct SideFork {
    qe_ctx* c;
    bool on = false;
    SideFork(qe_ctx* c, bool want);
    ~SideFork();
    void enter();
    void leave();
    void join();
    SideFork(const SideFork&) = delete;
    SideFork& operator=(const SideFork&) = delete;
};
bool side_stream_on();

// profiling-aware launch bracket
void add_bytes(qe_ctx* c, const char* stage, double bytes);

struct Timed {
    qe_ctx* c;
    int k = -1;
    hipEvent_t a = nullptr, b = nullptr;
    double bytes;
    Timed(qe_ctx* c_, const char* name, double alg_bytes);
    ~Timed();
};

// (the call site is recorded with each host round trip when QE_RT_SITES=1 and profiling is on)
void sync(qe_ctx* c, const char* file = __builtin_FILE(), int line = __builtin_LINE());
uint64_t read_u64(qe_ctx* c, const uint64_t* d, const char* file = __builtin_FILE(), int line = __builtin_LINE());
void read_words(qe_ctx* c, const uint64_t* d, uint64_t* h, int n, const char* file = __builtin_FILE(),
                int line = __builtin_LINE());

inline unsigned grid_for(uint64_t n, unsigned per_block, unsigned cap = 0x7fffffffu) {
    uint64_t g = (n + per_block - 1) / per_block;
    if (g == 0) g = 1;
    return (unsigned)(g < cap ? g : cap);
}

// ---- primitives shared between translation units ------------------------------------------
// compaction family (qe_scan.hip)
uint64_t filter_scan(qe_ctx* c, const uint64_t* col, uint64_t n, char op, uint64_t v, uint32_t* out);
uint64_t filter_scan2(qe_ctx* c, const uint64_t* c1, char op1, uint64_t v1, const uint64_t* c2, char op2, uint64_t v2,
                      uint64_t n, uint32_t* out);
uint64_t filter_scan2_vals(qe_ctx* c, const uint64_t* c1, char op1, uint64_t v1, const uint64_t* c2, char op2,
                           uint64_t v2, uint64_t n, uint32_t* out, uint32_t* outv);
// the partitioned plan's scans: the same rows, in no particular order (one atomic per wave tile
// instead of a lookback); rowids numbered from row_base; outv (nullable): c1's low words, aligned;
// kin / outk (nullable): the survivors' values of the u32 column kin (row i = element i), aligned
uint64_t filter_scan2_unordered(qe_ctx* c, const uint64_t* c1, char op1, uint64_t v1, const uint64_t* c2, char op2,
                                uint64_t v2, uint64_t n, uint32_t row_base, uint32_t* out, uint32_t* outv,
                                const uint32_t* kin = nullptr, uint32_t* outk = nullptr);
uint64_t filter_refine(qe_ctx* c, const uint64_t* col, const uint32_t* in, uint64_t n, char op, uint64_t v,
                       uint32_t* out);
uint64_t scan_join_k(qe_ctx* c, const uint64_t* rk, const uint32_t* rv, const uint64_t* sk, const uint32_t* sv,
                     uint64_t n, uint32_t* outR, uint32_t* outS);
// indices i (ascending) with key[i] == pmax[i] <= limit (pmax = inclusive prefix max of key)
uint64_t compact_prefix_max_hits(qe_ctx* c, const uint64_t* key, const uint64_t* pmax, uint64_t n, uint64_t limit,
                                 uint32_t* out);
uint64_t compact_nonzero_pairs(qe_ctx* c, const uint32_t* nz, uint64_t nzw, const uint32_t* last, const uint32_t* edit,
                               uint64_t n, uint32_t* out_last, uint32_t* out_edit);

// sort (qe_sort.hip): stable LSD radix; returns buffers (may alias inputs when 0 passes needed)
struct SortOut {
    void* keys;
    uint32_t* vals;
    bool keys_new, vals_new;
};
// bits (nullable): host {OR, AND} of the keys when already known; otherwise one reduction pass
// defer = true (qe_join_pairs only): a two-level sort may stop before its per-bucket step (see
// DeferredSort); the returned buffers are then filled by pairs_need_keys, or never (bucket_join)
SortOut radix_sort_u64(qe_ctx* c, const uint64_t* keys, const uint32_t* vals /*nullable: iota*/, uint64_t n,
                       bool with_vals, const uint64_t* bits = nullptr, bool defer = false);
// deferred two-level sorts (qe_sort.hip): complete one before its keys (or vals) are read;
// drop one whose pairs are freed; the unordered per-bucket join of two deferred sides (false:
// not applicable -- the caller completes both sorts and merges as usual)
void pairs_need_keys(qe_ctx* c, const qe_pairs* p);
void pairs_need_vals(qe_ctx* c, const qe_pairs* p);
// (also drops a gathered histogram; keep_k32: a key buffer the pairs only borrow keeps its u32
// keys, PreHist::k32, for another sort of it -- its owner's release frees them)
void pairs_drop_deferred(qe_ctx* c, const qe_pairs* p, bool keep_k32 = false);
// keys = col[rows] for a list whose sort will be the lookback-free two-level one: the sort's
// histogram is built in the same pass (false: not that sort -- the caller gathers plainly)
bool gather_with_hist(qe_ctx* c, const uint64_t* col, const uint32_t* rows, uint64_t n, uint64_t kor, uint64_t kand,
                      uint64_t* keys, uint64_t col_rows = 0);   // col_rows: the column's length (its u32 copy)
bool bucket_join(qe_ctx* c, const qe_pairs* R, const qe_pairs* S, qe_list* outR, qe_list* outS,
                 qe_list* outX0 = nullptr, qe_list* outX1 = nullptr, qe_list* outRX = nullptr);
// the payload carry of join_pairs_carry applies: both sides' sorts will be deferred two-level
// ones with one bucket geometry, S's in the lookback-free form
// (rpay: R carries a payload too -- its sort must be the lookback-free form as well)
bool carry_eligible(const qe_pairs* R, const qe_pairs* S, bool rpay = false);
// both sides' key bounds widened to their union when that gives both the deferred two-level sort
// with one bucket geometry (the bucket join instead of complete sorts + the merge)
void unify_geometry(qe_pairs* R, qe_pairs* S);
// qe_join_pairs with S carrying one or two u32 payload columns (xa, xb nullable) through its sort
// and the bucket join: outX0 / outX1 aligned with the pairs; and/or R carrying one 32-bit payload,
// a u32 array (rx32) or a u64 column's low words (rc64), both in R's input order: outRX.  False:
// nothing was produced and the inputs are as they were (ineligible, or a bucket beyond LDS) --
// the caller joins without it.
// rv64 (R without vals only): outR holds this u64 column's low words at R's rows instead of the
// row indices (R's binding read later only through that column).
bool join_pairs_carry(qe_ctx* c, qe_pairs* R, qe_pairs* S, const uint32_t* xa, const uint32_t* xb, qe_list* outR,
                      qe_list* outS, qe_list* outX0, qe_list* outX1, const uint32_t* rx32 = nullptr,
                      const uint64_t* rc64 = nullptr, qe_list* outRX = nullptr, const uint64_t* rv64 = nullptr);
// keys = (u64) vals for a list whose sort will be the lookback-free two-level one, with that
// sort's histogram (gather_with_hist without the gather); false: not that sort
// adopted (nullable): vals is a dalloc block of the keys as u32 that the caller gives up if the sort
// keeps its keys as u32 (PreHist::k32 = vals, no copy); *adopted = whether it did
bool widen_with_hist(qe_ctx* c, const uint32_t* vals, uint64_t n, uint64_t kor, uint64_t kand, uint64_t* keys,
                     bool* adopted = nullptr);
// a key buffer gathered as u32 only (PreHist::k32): widen it into the buffer now (no-op otherwise)
void keys_need_u64(qe_ctx* c, const void* keys);
// the join's checksums without its pairs (the plan's last join): sums[k] = sum over pairs of
// col_k[S-side rowid], the rowid being S's val (src 0) or the low / high half of its carried
// payload (src 1 / 2); *pairs = the pair count.  False: not applicable (geometry, a bucket
// beyond LDS) -- nothing was produced.
constexpr int HJ_SUMS = 4;
struct HjSums {
    const uint64_t* col[HJ_SUMS];
    int src[HJ_SUMS];
    int n;
};
bool bucket_join_sums(qe_ctx* c, const qe_pairs* R, const qe_pairs* S, const HjSums& sc, uint64_t* pairs,
                      uint64_t* sums);
// join_pairs_carry's sort + bucket_join_sums (xa null: S carries no payload); false: as there
bool join_pairs_sums(qe_ctx* c, qe_pairs* R, qe_pairs* S, const uint32_t* xa, const uint32_t* xb, const HjSums& sc,
                     uint64_t* pairs, uint64_t* sums);
SortOut radix_sort_u32(qe_ctx* c, const uint32_t* keys, const uint32_t* vals, uint64_t n,
                       const uint64_t* bits = nullptr);
// multi-GPU (qe_dist.hip): hash-partition rows into per-destination segments of out_keys /
// out_cols; d_cnt (2 x 64 words, device) receives the per-destination counts (then the cursors).
// Queued on the ctx stream, no host synchronisation.  keys32 (nullable): read these u32 keys instead
// of `keys`; out32: write the keys as u32 into out_keys (every key below 2^32).  A key's destination
// is its value's, whatever the width.
void partition_dev(qe_ctx* c, const uint64_t* keys, uint64_t n, const uint32_t* const* cols, int ncols,
                   uint32_t nparts, unsigned long long* d_cnt, uint64_t* out_keys, uint32_t* const* out_cols,
                   const uint32_t* keys32 = nullptr, bool out32 = false);
// the keys' pending u32 copy (PreHist::k32: gathered as u32, the u64 buffer not yet written), or null
const uint32_t* keys_pending_u32(qe_ctx* c, const void* keys);
// OR / AND of n keys -> host out[2] (synchronises)
void key_bits_u64(qe_ctx* c, const uint64_t* keys, uint64_t n, uint64_t* out);
// (key field << 32 | (uint32_t) val) words of a base column, stable-sorted by the field
// (key >> lo) & (2^nb - 1), nb <= 32 (qe_join_aggregate); vals == null packs the row index
uint64_t* sort_words_kv64(qe_ctx* c, const uint64_t* keys, const uint64_t* vals, uint64_t n, int lo, int nb,
                          const uint32_t* vals32 = nullptr);
// the aggregate join (qe_agg.hip) over two sides given as arrays: keys with bounds kb = {OR, AND}
// (a superset's are fine), values as a u64 column's low words (v64) or u32 (v32), or none (v64 =
// v32 = null: that sum is 0).  out = {pairs, sum over pairs of R's value, of S's value} mod 2^64.
// Sides of 2^32 rows or more, or keys varying in more than 32 bits: QE_ENOTSUP.
struct AggSide {
    const uint64_t* keys;
    const uint64_t* v64;
    const uint32_t* v32;
    uint64_t n;
    uint64_t kb[2];
};
void join_aggregate_sides(qe_ctx* c, const AggSide& R, const AggSide& S, uint64_t out[3]);
// (qe_sort.hip) the two-level sort's two global passes alone over (key field << 32 | value) words:
// *words (n) partitioned into 2^15 buckets of the field's top 15 bits, *bstart the 2^15 + 1 bucket
// starts -- no order inside a bucket.  nb (the field's width, from bit lo) in 16..31.
void partition_words_kv(qe_ctx* c, const uint64_t* keys, const uint64_t* v64, const uint32_t* v32, uint64_t n, int lo,
                        int nb, uint64_t** words, uint32_t** bstart);
constexpr int AGG_BUCKET_BITS = 15;
// (qe_dist.hip) a replicated base column's bucket `part` of `nparts` without the sorted heavy
// keys (qe_bucket_select), with a value column's low words beside each key instead of the rowid
// (vals null: the rowid); out->val holds them
void bucket_select_dev(qe_ctx* c, qe_col col, uint32_t nparts, uint32_t part, const uint64_t* heavy, uint32_t nheavy,
                       const uint64_t* vals, qe_pairs* out);
// (qe_dist.hip) the skew path's heavy keys: over the first `sample` rows of each column, the keys
// whose run in the sorted sample is longer than sample / div -- at most maxk of them, the most
// frequent, returned sorted.  Deterministic: every rank of replicated columns gets the same list.
std::vector<uint64_t> heavy_keys_dev(qe_ctx* c, const qe_col* cols, int ncols, uint64_t sample, uint64_t div,
                                     uint32_t maxk);

}  // namespace qe

#define QE_API_BEGIN(ctx) \
    try {
#define QE_API_END(ctx)                                                                         \
    }                                                                                           \
    catch (const ::qe::Error& e) {                                                              \
        if (ctx) (ctx)->err = e.what();                                                         \
        return e.code;                                                                          \
    }                                                                                           \
    catch (const std::exception& e) {                                                           \
        if (ctx) (ctx)->err = e.what();                                                         \
        return QE_EINVAL;                                                                       \
    }
