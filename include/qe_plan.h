/*
 * qe_plan.h -- the key-partitioned multi-GPU plan as host C over an engine.
 *
 * The reference is single-threaded (main/queries_main.c:37 -> execute_queries,
 * src/utilities.c:289-300).  Its join path shards by key: R ⋈ S = ⋃_g R_g ⋈ S_g with
 * g = part(key), and every printed number is a sum mod 2^64 (src/utilities.c:216-219), so a query
 * whose output is the relational answer can run on N ranks -- each rank filters its rowid slice,
 * exchanges the derived join sides by key (an RCCL all-to-all), joins its bucket locally and
 * all-reduces the sums.
 *
 * Not every query's output IS the relational answer: the reference's mid_result state machine
 * (src/join.c:152-628) prints positional garbage for some shapes (scan_join of unrelated lists,
 * join_payloads zipping misaligned lists, merges of stale "sorted" lists, stale entries of a
 * relation used twice).  qe_plan_check replays that state machine on the bindings alone (no data)
 * and accepts a query only when every list a later predicate or select reads is provably the
 * relational projection of its binding; a refused query (QE_ENOTSUP) is run by the engine's
 * fallback -- libqe's faithful executor on one rank, relations being replicated.
 *
 * The plan is engine-agnostic: libqe supplies the device + RCCL engine (qe_run_queries_dist in
 * qe.h), the tests supply a numpy + gloo engine through ctypes (tests/plan_engine.py), so one
 * implementation is exercised both ways.
 */
#ifndef QE_PLAN_H
#define QE_PLAN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* An engine array: a rowid list (uint32) or a key array (uint64), owned by the engine; 0 = none.
 * Handles given to the plan are released by it (release) unless noted. */
typedef uint64_t qe_h;

#define QE_PLAN_VALUES 0xFFFFFFFFu   /* checksums: rows_k holds the values themselves */
#define QE_PLAN_VALUES_SRC 4        /* join_sums: src[s] | this -- the carried list holds values */

typedef struct qe_engine {
    void* u;                    /* the engine's state, passed back to every call */
    uint32_t rank, world;
    /* relation metadata (replicated on every rank) */
    int (*rel_count)(void* u, uint32_t* n);
    int (*rel_shape)(void* u, uint32_t rel, uint64_t* rows, uint32_t* ncols);
    /* a1 on rows [start, end): rowids (global numbering) with col[r] op v, in no particular order
     * (the plan's lists feed only order-free consumers: its accepted queries are relational) */
    int (*scan)(void* u, uint32_t rel, uint32_t col, uint64_t start, uint64_t end, char op, uint64_t v, qe_h* out);
    /* rowids start .. start + n - 1 */
    int (*iota)(void* u, uint64_t start, uint64_t n, qe_h* out);
    /* a2: the rowids r of `rows` with col[r] op v, in their order (`rows` is consumed) */
    int (*refine)(void* u, uint32_t rel, uint32_t col, qe_h rows, char op, uint64_t v, qe_h* out);
    /* a4: keys col[rows[i]] (`rows` is borrowed) */
    int (*keys)(void* u, uint32_t rel, uint32_t col, qe_h rows, qe_h* out);
    /* a whole base relation as a join side: one rank -- the column itself, *rowids = 0 (row i);
     * N ranks -- this rank's hash bucket of the replicated column, as keys + rowids */
    int (*base_side)(void* u, uint32_t rel, uint32_t col, qe_h* keys, qe_h* rowids);
    /* hash-partition (keys, cols[0..ncols)) on the key and all-to-all them; the inputs are
     * consumed.  start queues the exchange (the plan works on the other join side meanwhile),
     * finish returns this rank's bucket */
    int (*exchange_start)(void* u, qe_h keys, const qe_h* cols, int ncols, qe_h* ticket);
    int (*exchange_finish)(void* u, qe_h ticket, qe_h* keys, qe_h* cols);
    /* a5-a8 on a rank's bucket: sort both sides by key, merge; oa[i] = va[ia[i]] (or ia[i] when
     * va == 0), likewise ob -- aligned, every matching pair once.  Inputs are borrowed. */
    int (*join)(void* u, qe_h ka, qe_h va, qe_h kb, qe_h vb, qe_h* oa, qe_h* ob);
    /* out[i] = src[idx[i]] (both borrowed) */
    int (*take)(void* u, qe_h src, qe_h idx, qe_h* out);
    int (*length)(void* u, qe_h h, uint64_t* n);
    /* a12, local: sums[k] = sum of col_k[rows_k[i]] mod 2^64 (rows borrowed) */
    int (*checksums)(void* u, int n, const uint32_t* rels, const uint32_t* cols, const qe_h* rows, uint64_t* sums);
    /* in place: v[i] = sum over ranks mod 2^64 */
    int (*allreduce)(void* u, uint64_t* v, int n);
    void (*release)(void* u, qe_h h);
    /* a query outside the plan's domain (nullable): `query` is a parsed, arranged query_t of
     * host/qe_query.h, `out` the FILE* the batch prints to (rank 0's matters); returns 0 or the
     * reference's exit code path (QE_EEXIT) -- identical on every rank */
    int (*fallback)(void* u, void* query, void* out);
    /* a1 then a2 on the same binding, fused (nullable): rowids r in [start, end) with
     * col1[r] op1 v1 and col2[r] op2 v2, in no particular order -- one pass over the column(s) instead of a
     * scan and a refine gathering through its list.  values bit 0: the plan expects to ask for col1's
     * values of this list later (`values` below) -- the engine may emit them from the same pass;
     * bits 8..15 (nonzero): 1 + the column every join of this binding keys on -- the engine may
     * emit those values too and take them for the binding's key side (`keys`) without a gather */
    int (*scan2)(void* u, uint32_t rel, uint32_t col1, char op1, uint64_t v1, uint32_t col2, char op2, uint64_t v2,
                 uint64_t start, uint64_t end, int values, qe_h* out);
    /* join, with side b's carried rowid columns cb[0..nb) delivered beside the pairs (nullable):
     * outb[k][i] = cb[k][ib] for pair i's b row.  xa (0: none): a column handle of `column` below,
     * side a being that column's base relation (ka its key column or bucket, va its rowids or 0):
     * *outxa[i] = the column's value at pair i's a row -- its next join's key, which then needs no
     * gather through the rowids.  The engine may carry them through its sorts and join instead of
     * taking them through the pairs afterwards.  Inputs are borrowed. */
    int (*join_carry)(void* u, qe_h ka, qe_h va, qe_h kb, qe_h vb, int nb, const qe_h* cb, qe_h xa, qe_h* oa, qe_h* ob,
                      qe_h* outb, qe_h* outxa);
    /* the last join of a query when only the checksums read its lists and side a carries no
     * binding (nullable): *pairs = the local pair count, sums[s] = the local sum mod 2^64 of
     * col_s (relation rels[s], column cols[s]) over the pairs' b rows, through b's vals (src[s]
     * = 0; its positions when vb == 0) or cb[src[s] - 1] -- the numbers print_sums would
     * compute from the materialised lists (src/utilities.c:197-224); the engine may skip
     * materialising them.  Inputs are borrowed. */
    int (*join_sums)(void* u, qe_h ka, qe_h va, qe_h kb, qe_h vb, int nb, const qe_h* cb, int nsel, const int* src,
                     const uint32_t* rels, const uint32_t* cols, uint64_t* pairs, uint64_t* sums);
    /* a binding read later only by selects of one column (nullable): out[i] = col[rows[i]] as
     * uint32 when every value of the column is below 2^32, QE_ENOTSUP otherwise (`rows` is
     * borrowed).  The plan then carries the values instead of the rowids: a list of values is
     * passed to checksums with rels[k] = QE_PLAN_VALUES (its own sum) and to join_sums with
     * src[s] | QE_PLAN_VALUES_SRC (summed, not gathered). */
    int (*values)(void* u, uint32_t rel, uint32_t col, qe_h rows, qe_h* out);
    /* the materialisation limit (nullable: none): a join whose pair count summed over every rank
     * exceeds *mat_limit ends the query with QE_ETOOBIG on every rank (then e->fallback) -- the
     * reference's DArray bound is on the whole result (src/DArray.h:14-15), so the same query
     * takes the same branch at any rank count.  (An engine may also refuse a join whose LOCAL
     * share exceeds it: that share is a lower bound of the global count.) */
    const uint64_t* mat_limit;
    /* the query's last join when both sides are whole base relations and every select reads one of
     * its two bindings (nullable): the join in aggregate form -- *pairs = this rank's share of the
     * pair count, sums[s] = its share of the sum mod 2^64 of column cols[s] of side side[s] (0: a,
     * 1: b) over the pairs -- the numbers print_sums computes from the lists (src/join.c:325-392,
     * src/utilities.c:197-224), no pair materialised, any key skew (C5).  Shares add up over the
     * ranks (the plan all-reduces them).  QE_ENOTSUP: not applicable (the plan then joins as
     * usual).  No materialisation limit applies: nothing is materialised. */
    int (*join_agg)(void* u, uint32_t rel_a, uint32_t col_a, uint32_t rel_b, uint32_t col_b, int nsel, const int* side,
                    const uint32_t* cols, uint64_t* pairs, uint64_t* sums);
    /* a base column as join_carry's xa (nullable): QE_ENOTSUP when its values do not all fit 32
     * bits.  Released like any handle (the column itself stays). */
    int (*column)(void* u, uint32_t rel, uint32_t col, qe_h* out);
    /* keys from a list of the key column's values (nullable; join_carry's outxa): the keys `keys`
     * would gather through the rowids, without the gather (`vals` borrowed) */
    int (*keys_of)(void* u, uint32_t rel, uint32_t col, qe_h vals, qe_h* out);
    /* a WHOLE base relation as a join side at any rank count (nullable): the column itself,
     * *rowids = 0 (row i), as base_side gives it at one rank.  The plan's broadcast joins use it:
     * at N ranks a join of a derived side with a whole (replicated) base relation may leave the
     * derived side where it lies and join it against the whole column on every rank -- each pair
     * is still made on exactly one rank -- instead of exchanging the derived side and joining
     * bucket against bucket; the plan picks the cheaper by its cost model (QE_PLAN_BCAST). */
    int (*base_side_all)(void* u, uint32_t rel, uint32_t col, qe_h* keys, qe_h* rowids);
} qe_engine;

/* Replay the reference's variant choice and list bookkeeping for every query of `text` on the
 * bindings alone; accepted[i] = 1 when query i's output is the relational answer (nullable).
 * Returns the number of queries. */
int qe_plan_check_text(const qe_engine* e, const char* text, uint8_t* accepted, size_t cap);
/* The first refusal reason of the last qe_plan_check_text / qe_plan_run_text call on this thread. */
const char* qe_plan_why(void);

/* Run every query of `text` (the reference's protocol: F lines skipped, every query parsed before
 * any runs) with the partitioned plan, refused queries through e->fallback (QE_ENOTSUP when there
 * is none).  Every rank calls it with the same text; *out (malloc'd, free with free()) is the
 * stdout the reference would print (meaningful on rank 0).  *rows (nullable): the global row count
 * of the last printed query's first select.  *nrefused (nullable): queries sent to the fallback. */
int qe_plan_run_text(const qe_engine* e, const char* text, char** out, size_t* outlen, uint64_t* rows,
                     uint64_t* nrefused);
/* One parsed, arranged query (a host/qe_query.h query_t) the same way, printing to the FILE* `out`:
 * planned when accepted, else (or on QE_ETOOBIG) through e->fallback; *refused = 1 then.  *rows
 * (nullable) as above.  (The concurrent batch runs its lanes' queries through this.) */
int qe_plan_run_query(const qe_engine* e, void* query, void* out, uint64_t* rows, int* refused);

#ifdef __cplusplus
}
#endif
#endif /* QE_PLAN_H */
