/*
 * qe.h -- C ABI of libqe, the MI355X-native sort-merge-join executor.
 *
 * The reference (giorgosLiako/Query-Compiler-Executor) has no FFI: its operator seam is two
 * C functions called by execute_query (src/utilities.c:262-269) plus the static print_sums
 * (src/utilities.c:197).  libqe replaces that seam at two levels:
 *
 *   1. the executor level -- qe_run_queries() runs a whole query batch with the reference's
 *      stdin/stdout semantics (main/queries_main.c:24-68, src/utilities.c:258-300): the host-C
 *      restatement of parsing.c / pred_arrange.c / the mid_result state machine drives the
 *      device primitives below, and `queries` (host/qe_main.c) is the drop-in binary;
 *   2. the primitive level -- one entry point per hot-path step,
 *      each citing the reference function it replaces.
 *
 * Conventions: every call returns 0 on success and a negative QE_E* code on
 * failure (qe_last_error() has the message); no exceptions cross the ABI; device buffers are
 * plain pointers owned by the qe_ctx that allocated them (release with qe_list_free /
 * qe_pairs_free); one host thread drives one ctx; work is ordered on the ctx's HIP stream and
 * every call that returns a host-visible size or value synchronises that stream.
 * Rowids are uint32 (relations below 2^32 rows), keys/values uint64, sums wrap mod 2^64.
 */
#ifndef QE_H
#define QE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QE_ABI_VERSION 1

enum {
    QE_OK = 0,
    QE_EINVAL = -1,      /* bad argument / reference-undefined input */
    QE_EHIP = -2,        /* HIP runtime error */
    QE_ENOMEM = -3,      /* device allocation failed */
    QE_EEXIT = -4,       /* the reference would have called exit(EXIT_FAILURE) here */
    QE_ETOOBIG = -5,     /* a join result beyond the materialisation limit (qe_set_materialize_limit) */
    QE_ENOTSUP = -6,     /* outside the partitioned plan's domain (include/qe_plan.h): run it faithfully */
};

typedef struct qe_ctx qe_ctx;

/* A device column: `n` uint64 values (one column of a relation in HBM). */
typedef struct { const uint64_t* d; uint64_t n; } qe_col;

/* A device rowid list -- the reference's payload DArray (src/DArray.h, src/structs.h:44-49).
 * flags bit 0 (QE_LIST_DISTINCT): no rowid occurs twice. */
typedef struct { uint32_t* d; uint64_t n; uint64_t cap; uint32_t flags; } qe_list;
#define QE_LIST_DISTINCT 1u

/* Join input: (key, rowid) pairs in SoA -- the reference's `relation` of `tuple`s
 * (src/structs.h:7-15).  `val == NULL` means rowid i for every i (a base column).
 * match: per-row count of partner rows, filled by qe_merge_join on its sorted path (NULL
 * before), used by qe_driver_counts.  kor/kand: key bounds when QE_PAIRS_BITS is set -- every
 * key k satisfies (k & ~kor) == 0 and (k & kand) == kand (the OR / AND of all keys, or of a
 * superset such as the column the keys were gathered from); the sort then needs no reduction.
 * flags: QE_PAIRS_DISTINCT (no rowid twice), QE_PAIRS_SORTED (ascending by key), QE_PAIRS_BITS.
 * owns: bit 0 key, bit 1 val, bit 2 match buffer belong to the pairs (qe_pairs_free). */
typedef struct {
    uint64_t* key;
    uint32_t* val;
    uint32_t* match;
    uint64_t n;
    uint64_t kor, kand;
    uint32_t flags;
    uint32_t owns;
} qe_pairs;
#define QE_PAIRS_DISTINCT 1u
#define QE_PAIRS_SORTED 2u
#define QE_PAIRS_BITS 4u
/* match holds this side's partner counts for the join it last took part in (set by
 * qe_merge_join on R and by qe_merge_join_counts on both sides, cleared by qe_sort_pairs) */
#define QE_PAIRS_MATCHED 8u

/* Per-kernel statistics (profiling, qe_set_profiling). */
typedef struct {
    char     name[48];
    uint64_t launches;
    double   total_ms;        /* sum of HIP-event durations on the ctx stream */
    double   alg_bytes;       /* algorithmic bytes summed over launches */
} qe_kstat;

/* ---- lifecycle --------------------------------------------------------------------------- */
qe_ctx*     qe_init(int device);
void        qe_fini(qe_ctx*);
const char* qe_last_error(qe_ctx*);
int         qe_abi_version(void);
int         qe_device_name(qe_ctx*, char* out, size_t cap);
int         qe_sync(qe_ctx*);

/* ---- relations (loader: src/utilities.c:105-162) ------------------------------------------ */
/* Copy a column-major host relation into HBM; returns the relation id (= load order) or <0. */
int qe_load_relation(qe_ctx*, uint64_t rows, uint64_t ncols, const uint64_t* const* host_cols);
/* Generate a relation on the device with the splitmix64 generator of SURVEY.md §9.1.
 * kinds[c]: 0 = v % mod[c], 1 = v >> 32, 2 = Zipf key over [0, mod[c]) drawn through the table
 * of qe_set_zipf_table (mod[c] must equal its domain).  Returns the relation id or <0. */
int qe_gen_relation(qe_ctx*, uint64_t rows, uint64_t ncols, const int* kinds, const uint64_t* mods,
                    uint64_t seed, uint32_t gen_rel, uint64_t row_start);
/* Zipf sampling table for kind 2 (the C5 skew workload): d_cdf holds `domain`
 * nondecreasing doubles in device memory, the last one 1.0 (borrowed until the next call or
 * qe_fini).  A draw takes the 53-bit uniform u = (v >> 11) * 2^-53, rank = #{r : cdf[r] <= u}
 * capped at domain-1, and returns the seeded Feistel permutation of rank (qe/datagen.py
 * feistel_perm).  d_cdf = NULL drops the table. */
int qe_set_zipf_table(qe_ctx*, const double* d_cdf, uint64_t domain, uint64_t perm_seed);
/* The same with a table libqe builds and owns: cdf[r] = sum_{q<=r} (q+1)^-theta / total, summed
 * in a fixed order so every run on the device draws the same keys (C5 bench data). */
int qe_set_zipf(qe_ctx*, uint64_t domain, double theta, uint64_t perm_seed);
int qe_relation_count(qe_ctx*);
int qe_relation_column(qe_ctx*, int rel, int col, qe_col* out);
/* Column statistics computed once when the relation is loaded/generated (OR and AND of every
 * value: the bits that vary, which is all an LSD radix sort needs to plan its passes). */
int qe_relation_column_bits(qe_ctx*, int rel, int col, uint64_t* kor, uint64_t* kand);
int qe_relation_rows(qe_ctx*, int rel, uint64_t* rows);
int qe_drop_relations(qe_ctx*);

/* ---- executor (src/utilities.c:258-300 + main/queries_main.c) ------------------------------ */
/* Run every query line of `text` (relation ids = load order) and return the exact stdout bytes
 * the reference would print in a malloc'd buffer (free with qe_free_host).  Returns 0, QE_EEXIT
 * when the reference would have exited with status 1 (output up to that point is returned), or
 * another negative code. */
int  qe_run_queries(qe_ctx*, const char* text, char** out, size_t* outlen);
void qe_free_host(void*);
/* The same batch with its queries run concurrently: `workers` (1..16) contexts on this ctx's GPU --
 * each its own HIP stream and allocator, this ctx's relations shared -- take queries in turn from
 * host threads; the outputs are joined in input order and cut after the first query where the
 * reference exits (QE_EEXIT), so the bytes and the status are qe_run_queries'.  The reference runs
 * its queries one after another with no state between them but rand() (src/utilities.c:289-300;
 * the gate excludes rand-dependent outputs), so the order of execution is not observable. */
int  qe_run_queries_parallel(qe_ctx*, int workers, const char* text, char** out, size_t* outlen);
/* The concurrent batch with a choice of executor per query: QE_EXEC_FAITHFUL (qe_run_queries'
 * state machine; = qe_run_queries_parallel) or QE_EXEC_PLAN (each query through the partitioned
 * plan on its lane's ctx as one rank, the faithful executor for the queries the plan refuses --
 * qe_run_queries_dist's bytes).  workers <= 1 runs the batch on this ctx. */
#define QE_EXEC_FAITHFUL 0
#define QE_EXEC_PLAN 1
int  qe_run_queries_lanes(qe_ctx*, int workers, int executor, const char* text, char** out, size_t* outlen);
/* A batch's shared sorts of whole base columns (no reference counterpart: the reference sorts a
 * base relation again for every join, src/join.c:122-142 + :5-94).  on = 1: from now on the first
 * join of a column sorts it once, on whichever lane or ctx of this ctx's family needs it first, and
 * every later join on that column reads that sort (payload-carrying sorts excepted); on = 0: waits
 * for every stream of the family and frees them.  qe_run_queries_lanes brackets its batch with
 * it; QE_SORT_CACHE=0 turns it off.  Stats: cached sorts reused / built over finished batches. */
int  qe_sort_cache(qe_ctx*, int on);
int  qe_sort_cache_stats(qe_ctx*, uint64_t* hits, uint64_t* builds);
/* The worker contexts behind qe_run_queries_parallel (made on first use, freed by qe_fini; the
 * relations re-shared at every call); qe_bind_thread makes the ctx's GPU the calling thread's. */
int  qe_workers(qe_ctx*, int n, qe_ctx** out);
int  qe_bind_thread(qe_ctx*);
/* Row count of the first selected binding's list in the last query that printed sums (the
 * join's output cardinality for the relational shapes; bench "joined tuples"). */
int  qe_last_result_rows(qe_ctx*, uint64_t* rows);
int  qe_set_last_result_rows(qe_ctx*, uint64_t rows);

/* ---- device primitives ---------------------------------------------------- */
/* a1: exec_filter_rel_no_exists (src/filter.c:37-64): rowids i with col[i] op v, ascending. */
int qe_filter_scan(qe_ctx*, qe_col col, char op, uint64_t v, qe_list* out);
/* a2: exec_filter_rel_exists (src/filter.c:3-35): keep rowids r of `in` with col[r] op v, in
 * order (the count is the stray stdout line of src/filter.c:32; printing is the caller's). */
int qe_filter_refine(qe_ctx*, qe_col col, char op, uint64_t v, qe_list* inout);
/* a3/a4: allocate_relation / allocate_relation_mid_results (src/join.c:96-142):
 * (key = col[rowid], rowid) for rows == NULL (every row) or for each rowid of *rows in order. */
int qe_gather_pairs(qe_ctx*, qe_col col, const qe_list* rows, qe_pairs* out);
/* a5-a7: iterative_sort + quicksort (src/join.c:5-94, src/quicksort.c): ascending by key,
 * stable (LSD radix over the key bits that vary). */
int qe_sort_pairs(qe_ctx*, qe_pairs* inout);
int qe_is_sorted(qe_ctx*, const qe_pairs*, int* sorted);
/* a8: join_relations (src/join.c:325-392): aligned payload lists in key, R, S order.  Runs the
 * merge-path kernel when both inputs are sorted and the exact two-pointer semantics otherwise.
 * A sorted join of more pairs than the materialisation limit returns QE_ETOOBIG with
 * outR->n = outS->n = the exact pair count, no lists, and R->match filled (the reference's
 * DArray cannot hold such a result either: src/DArray.h:14-15, src/DArray.c:62-65). */
int qe_merge_join(qe_ctx*, qe_pairs* R, const qe_pairs* S, qe_list* outR, qe_list* outS);
/* a8 without the order: every (R.val[i], S.val[j]) with equal keys (row i / j when val is NULL),
 * aligned in outR / outS in NO particular order -- the partitioned plan's join (include/qe_plan.h),
 * whose pairs feed only order-free consumers.  Both sides are sorted by their two global radix
 * passes only; when the two bucket geometries agree, each 15-bit bucket joins in LDS (a counting
 * sort of R's bucket by its remaining key bits, one bound lookup per S row), else the sorts
 * complete and the merge runs.  QE_ETOOBIG beyond the materialisation limit. */
int qe_join_pairs(qe_ctx*, qe_pairs* R, qe_pairs* S, qe_list* outR, qe_list* outS);
/* Pairs above which qe_merge_join returns QE_ETOOBIG (default INT32_MAX; env QE_MAT_LIMIT). */
int qe_set_materialize_limit(qe_ctx*, uint64_t pairs);
/* a8, aggregate form (C5, SURVEY.md §0.7 / §8(e) "aggregate push-down"): for sorted R and S,
 * R->match[i] = #S rows with R's key, S->match[j] = #R rows with S's key, *pairs = the join's
 * exact pair count.  No pair is materialised.  An R already carrying QE_PAIRS_MATCHED (what
 * qe_merge_join leaves on R, e.g. after QE_ETOOBIG) is taken as counted against this S. */
int qe_merge_join_counts(qe_ctx*, qe_pairs* R, qe_pairs* S, uint64_t* pairs);
/* a9: scan_join (src/join.c:395-423). */
int qe_scan_join(qe_ctx*, const qe_pairs* R, const qe_pairs* S, qe_list* outR, qe_list* outS);
/* a8 dedup: the multiset non_duplicates[mode] of a join (src/join.c:358-367) as a dense count
 * array over rowids [0, rows): counts[x] = #distinct (pR,pS) pairs whose mode-side rowid is x.
 * R/S (nullable) are the join's inputs: when both are QE_PAIRS_SORTED and the other side is
 * QE_PAIRS_DISTINCT the counts come from the merge's per-row match counts (mode 0) or one
 * annotated merge pass (mode 1); otherwise from an exact sort + unique of the packed pairs
 * (outR[i], outS[i]).  join_payloads only ever uses the driver as a sorted multiset
 * (src/join.c:436-445), so counts are all it needs. */
int qe_driver_counts(qe_ctx*, const qe_pairs* R, const qe_pairs* S, const qe_list* outR, const qe_list* outS,
                     int mode, uint64_t rows, uint32_t** d_counts);
/* a10: join_payloads (src/join.c:426-484): edit[i] repeated counts[last[i]] times, ordered by
 * last[i] (stable).  |edit| < |last| is undefined in the reference -> QE_EINVAL. */
int qe_join_payloads(qe_ctx*, const uint32_t* d_counts, uint64_t rows, const qe_list* last,
                     const qe_list* edit, qe_list* out);
/* The same for every entry fix_all_mid_results updates with one (driver, last) pair
 * (src/join.c:493-500): the pruning, the sort by `last` and the counts are shared, only the
 * expansion runs per edit list.  outs[k] receives join_payloads(driver, last, edits[k]). */
int qe_join_payloads_multi(qe_ctx*, const uint32_t* d_counts, uint64_t rows, const qe_list* last,
                           const qe_list* const* edits, int nedits, qe_list* outs);
/* a12: print_sums' inner loop (src/utilities.c:216-219): sum of col[rowid] mod 2^64. */
int qe_checksum(qe_ctx*, qe_col col, const qe_list* rows, uint64_t* sum);
/* print_sums' whole select loop (src/utilities.c:199-221) for n (column, list) pairs: every sum
 * is computed before one host round trip; sums[k] = qe_checksum(cols[k], rows[k]). */
int qe_checksums(qe_ctx*, int n, const qe_col* cols, const qe_list* const* rows, uint64_t* sums);
/* a12 over an unmaterialised join side: sum of col[p->val[i]] * p->match[i] mod 2^64, which is
 * qe_checksum over the list qe_merge_join would have produced for that side
 * (sum_pairs col(pR) = sum_k (sum_{r in R_k} col(r)) * |S_k|). */
int qe_checksum_weighted(qe_ctx*, qe_col col, const qe_pairs* p, uint64_t* sum);
/* a8 + print_sums, aggregate form for two BASE columns (C5: the query's last join, each side's
 * selects on at most one column): with c_i = #S rows whose key equals R.key[i] (and symmetric),
 * out[0] = sum_i c_i = the join's pair count P, out[1] = sum_i valR[i] * c_i and out[2] =
 * sum_j valS[j] * c_j (mod 2^64) -- the checksums qe_checksum computes over the two P-row lists
 * the reference would build (src/join.c:325-392, src/utilities.c:197-224).  Each side is sorted
 * once with its value column in the word, then one merge-path pass counts both sides: no rowid,
 * no gather, no pair.  valR.d / valS.d may be NULL (that sum is 0).  QE_ENOTSUP when a value
 * column holds values >= 2^32, the keys vary in more than 32 bits or a side has >= 2^32 rows. */
int qe_join_aggregate(qe_ctx*, qe_col keyR, qe_col valR, qe_col keyS, qe_col valS, uint64_t* out);

/* ---- multi-GPU plan; the exchange itself is an RCCL all-to-all -------------- */
/* Hash-partition n rows on their key: dest = (hi32((key ^ key >> 29) * 0xbf58476d1ce4e5b9) * nparts) >> 32.  Rows go
 * to contiguous per-destination segments (dest order; order inside a segment unspecified) of the
 * caller's device buffers out_keys / out_cols[c] (capacity n each); counts[p] (host) = rows for
 * destination p.  ncols <= 4 uint32 rowid columns travel with each key. */
int qe_partition(qe_ctx*, const uint64_t* keys, uint64_t n, const uint32_t* const* cols, int ncols,
                 uint32_t nparts, uint64_t* counts, uint64_t* out_keys, uint32_t* const* out_cols);
/* a1 on a row range [start, end) of a column, rowids numbered globally (a rank's slice). */
int qe_filter_scan_range(qe_ctx*, qe_col col, uint64_t start, uint64_t end, char op, uint64_t v, qe_list* out);
/* a1 + a2 fused: rowids r in [start, end) with col1[r] op1 v1 AND col2[r] op2 v2, ascending --
 * exec_filter_rel_no_exists followed by exec_filter_rel_exists on the same binding
 * (src/filter.c:37-64, 3-35); the refine's list is never built.  col1 and col2 may be the same
 * column (read once). */
int qe_filter_scan2_range(qe_ctx*, qe_col col1, char op1, uint64_t v1, qe_col col2, char op2, uint64_t v2,
                          uint64_t start, uint64_t end, qe_list* out);
/* rowids start .. start+n-1 (an unfiltered slice). */
int qe_iota(qe_ctx*, uint64_t start, uint64_t n, qe_list* out);
/* out[i] = src[idx[i]] (carry a rowid column through a join's index lists). */
int qe_take_u32(qe_ctx*, const uint32_t* src, const qe_list* idx, qe_list* out);
/* Equi-join of two key arrays (a rank's bucket): sort both, merge, return aligned row indices. */
int qe_join_indices(qe_ctx*, const uint64_t* keysA, uint64_t nA, const uint64_t* keysB, uint64_t nB, qe_list* ia,
                    qe_list* ib);
/* Local bucket of a replicated base column: the rows whose qe_partition dest is `part`, as
 * (key, rowid) pairs in no particular order (out owns both arrays).  Keys in the sorted list
 * heavy[0..nheavy) (host memory, <= 1024, the skew path) are left out.  Replaces the exchange
 * of a join side that is a whole base relation: every rank holds the column. */
int qe_bucket_select(qe_ctx*, qe_col col, uint32_t nparts, uint32_t part, const uint64_t* heavy, uint32_t nheavy,
                     qe_pairs* out);
/* Hash-partitioned layout of the base relations (north star "relations
 * hash-partition across the GPUs"): from this call on, the partitioned plan at nparts ranks keeps,
 * per base column it joins as a whole base side, this rank's hash bucket (part of nparts) as
 * qe_bucket_select leaves it -- selected the first time a join reads that column, kept in the ctx
 * until the relations are dropped -- instead of scanning the replicated column once per join
 * (~0.18 ms per 1e8-row side on every rank, at any rank count).  Columns never read that way (payload
 * columns, broadcast joins' base sides) hold no bucket.  Columns stay replicated (the faithful
 * fallback runs on rank 0).  Fails only on bad arguments.  Replaces nothing in the reference (it has
 * no multi-GPU path); the row set per bucket is qe_bucket_select's. */
int qe_partition_columns(qe_ctx*, uint32_t nparts, uint32_t part);
/* Skew path (C5): over rows [start, end) of `keys`, counts[h] = #rows whose key is heavy[h]
 * (host arrays, heavy sorted, <= 1024) and, when weights != NULL,
 * wsum = sum of vals[row] * weights[h] over those rows mod 2^64.  counts/wsum nullable. */
int qe_heavy_stats(qe_ctx*, qe_col keys, uint64_t start, uint64_t end, const uint64_t* heavy, uint32_t nheavy,
                   qe_col vals, const uint64_t* weights, uint64_t* counts, uint64_t* wsum);
/* ---- multi-GPU: RCCL communicator, exchange, all-reduce, the partitioned executor ------------ */
/* One rank per GPU (one process each); rank 0 makes the bootstrap id and hands it to every rank
 * out of band (bench.py: torch.distributed gloo; `queries`: a pipe). */
typedef struct qe_comm qe_comm;
/* ncclGetUniqueId: 128 bytes */
int  qe_comm_unique_id(uint8_t* id);
/* ncclCommInitRank on the ctx's device; exchanges run on the communicator's own stream */
int  qe_comm_init(qe_ctx*, int nranks, int rank, const uint8_t* id, qe_comm** out);
void qe_comm_fini(qe_comm*);
/* vals[i] = sum over ranks of vals[i] mod 2^64 (host array, n <= 64): ncclAllReduce(ncclUint64,
 * ncclSum) -- print_sums' checksums (src/utilities.c:216-219) and list lengths across ranks */
int  qe_allreduce_u64(qe_ctx*, qe_comm*, uint64_t* vals, int n);
/* Hash-partition n rows (keys + ncols uint32 rowid columns) on the key (qe_partition's dest) and
 * exchange them: every rank receives its bucket from every rank, one grouped ncclSend/ncclRecv.
 * Outputs are ctx device buffers (qe_buffer_free); inputs are left untouched. */
int  qe_shuffle_pairs(qe_ctx*, qe_comm*, const uint64_t* keys, uint64_t n, const uint32_t* const* cols, int ncols,
                      uint64_t** out_keys, uint32_t** out_cols, uint64_t* out_n);
void qe_buffer_free(qe_ctx*, void*);
int  qe_comm_stats(qe_comm*, uint64_t* exchanges, uint64_t* bytes_sent);
/* execute_queries (src/utilities.c:289-300) on every rank of `comm` (NULL: one rank): each query
 * whose output is the relational answer (qe_plan.h's replay of the reference's state machine) runs
 * key-partitioned -- rank slices filtered, derived join sides exchanged, local sort-merge joins,
 * sums all-reduced; the others run on the faithful executor on rank 0 (relations are replicated on
 * every rank).  Every rank passes the same text and relations; *out (rank 0) is the reference's
 * stdout; *refused = queries run the faithful way.  Returns 0, QE_EEXIT or an error. */
int  qe_run_queries_dist(qe_ctx*, qe_comm*, const char* text, char** out, size_t* outlen, uint64_t* refused);
/* The in-process transport: nranks communicators over ctxs[0..nranks) (contexts of this process --
 * typically qe_workers of one ctx on ONE GPU, where RCCL refuses a second rank), each rank driven by
 * its own host thread.  Only the transport differs from qe_comm_init's: the counts all-to-all and the
 * grouped send/recv become host barriers + device-to-device copies pulled by each receiver, the
 * all-reduce a host sum; the partitioning, the plan and every kernel are the same code.  A rank that
 * fails outside a collective breaks the group (its peers return QE_EHIP instead of waiting); a peer
 * that never arrives times out after QE_LOCAL_TIMEOUT_S seconds (default 600).  Release each with
 * qe_comm_fini. */
int  qe_comm_init_local(qe_ctx* const* ctxs, int nranks, qe_comm** out);
/* qe_run_queries_dist on nranks (1..16) in-process ranks over qe_workers(ctx, nranks) and
 * qe_comm_init_local, one host thread each: rank 0's bytes and status, *refused = rank 0's
 * fallback count, *bytes_sent (nullable) = every rank's exchanged bytes (key + carried columns
 * sent to other ranks).  `queries` runs it with QE_LOCAL_RANKS=N. */
int  qe_run_queries_local(qe_ctx*, int nranks, const char* text, char** out, size_t* outlen, uint64_t* refused,
                          uint64_t* bytes_sent);

/* The ctx's HIP stream (hipStream_t), for callers that order their own work against it. */
int qe_sync_stream_ptr(qe_ctx*, void** stream);

/* ---- buffers ------------------------------------------------------------------------------- */
int  qe_list_alloc(qe_ctx*, uint64_t n, qe_list* out);
int  qe_list_from_host(qe_ctx*, const uint32_t* h, uint64_t n, uint32_t flags, qe_list* out);
int  qe_list_to_host(qe_ctx*, const qe_list*, uint32_t* h);
void qe_list_free(qe_ctx*, qe_list*);
int  qe_pairs_from_host(qe_ctx*, const uint64_t* key, const uint32_t* val, uint64_t n, qe_pairs* out);
int  qe_pairs_to_host(qe_ctx*, const qe_pairs*, uint64_t* key, uint32_t* val);
void qe_pairs_free(qe_ctx*, qe_pairs*);
void qe_counts_free(qe_ctx*, uint32_t*);
int  qe_counts_to_host(qe_ctx*, const uint32_t* d, uint64_t n, uint32_t* h);
/* device memory in use / cached by the ctx allocator (bytes) */
int  qe_mem_stats(qe_ctx*, uint64_t* in_use, uint64_t* cached);
/* host -> HBM loads so far (qe_load_relation): wall seconds and bytes, PCIe and the pinned
 * staging included, and the load-time layout work too (the column OR/AND read and the u32 copies
 * of narrow columns) -- the loader of the reference, read_relations (src/utilities.c:124-162) */
int  qe_load_stats(qe_ctx*, double* seconds, double* bytes);
int  qe_mem_trim(qe_ctx*);

/* ---- profiling ----------------------------------------------------------------------------- */
int qe_set_profiling(qe_ctx*, int on);
/* time only the launches of one stage (NULL or "": all): two HIP events per launch cost host
 * time, so the bench's timed region measures its roofline kernel alone (bench.py) */
int qe_set_profiling_only(qe_ctx*, const char* stage);
int qe_reset_stats(qe_ctx*);
/* fills up to `max` entries, returns the number of kernels with statistics */
int qe_kernel_stats(qe_ctx*, qe_kstat* out, int max);

#ifdef __cplusplus
}
#endif
#endif /* QE_H */
