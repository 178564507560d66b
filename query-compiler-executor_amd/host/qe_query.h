/*
 * qe_query.h -- the reference's query frontend, restated in C (host side of libqe; shared by the
 * faithful executor host/qe_exec.c and the partitioned plan host/qe_plan.c).  Not part of the ABI.
 */
#ifndef QE_QUERY_H
#define QE_QUERY_H

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {                 /* predicate (src/structs.h:29-34) */
    int type;                    /* 0 join, 1 filter, -1 unparsed */
    uint64_t frel, fcol, srel, scol;   /* filter: srel = constant, scol = 0 (what is_match reads) */
    char op;
    uint64_t cval;               /* uint32 constant, zero-extended (src/filter.c:70) */
} pred_t;

typedef struct {
    uint32_t* rels; size_t nrels;
    pred_t* preds; size_t npreds;
    uint64_t* sel; size_t nsel;
} query_t;

/* parser() (src/parsing.c:118-148): every line of `text` until its end, 'F' lines skipped; the
 * three scan buffers persist across lines as the reference's stack arrays do.  Returns a malloc'd
 * array of *nq queries (qe_free_queries). */
query_t* qe_parse_text(const char* text, size_t* nq);
void qe_free_queries(query_t* qs, size_t nq);
/* arrange_predicates (src/pred_arrange.c:50-93), index-lag quirk included */
void qe_arrange_predicates(query_t* q);

/* ---- the mid_result bookkeeping both executors share ------------------------------------------
 * A mid_result (src/structs.h:44-49) without its list: the faithful executor keeps a device list
 * beside it, the plan's replay a symbolic one.  Both see mid_results_array through a view, and the
 * variant choice of build_relations is written once, here. */
typedef struct { uint64_t relation, pid; int32_t lcs; } qe_mid_t;

typedef struct {
    void* u;
    size_t (*count)(void* u);                            /* entities, oldest first */
    size_t (*size)(void* u, size_t ent);                 /* entries of one entity */
    qe_mid_t* (*at)(void* u, size_t ent, size_t idx);
    void (*push_entity)(void* u);                        /* create_entity_mid_results (src/join.c:145-150) */
} qe_mids;

typedef struct { ptrdiff_t ent, idx; } qe_where_t;       /* ent = -1: none */

/* relation_exists (src/utilities.c:164-181): newest entity first, first match */
qe_where_t qe_mid_exists(const qe_mids* M, uint64_t relation, uint64_t pid);
/* relation_exists_current (src/utilities.c:183-194): last match in one entity, -1 none */
ptrdiff_t qe_mid_exists_current(const qe_mids* M, size_t ent, uint64_t relation, uint64_t pid);

enum { QE_CLASSIC_JOIN = 1, QE_JOIN_SORT_LHS = 2, QE_JOIN_SORT_RHS = 3, QE_SCAN_JOIN = 4, QE_DO_NOTHING = 5 };

/* build_relations (src/join.c:152-292) without the gathers: the join variant, and the entry each
 * side is gathered from (ent = -1: the whole base relation), with the reference's side effects on
 * the entities (a first / a new entity, last_column_sorted updates) and its quirks
 * (src/join.c:258-262 compare the wrong side's column). */
typedef struct { int variant; qe_where_t lhs, rhs; } qe_join_choice_t;
qe_join_choice_t qe_build_relations(const qe_mids* M, const query_t* q, const pred_t* p);

struct qe_ctx;
/* host/qe_exec.c: one parsed, arranged query through the faithful executor (0, QE_EEXIT, <0) */
int qe_exec_query(struct qe_ctx* ctx, query_t* q, FILE* out);
/* csrc/qe_comm.hip: one parsed, arranged query through the partitioned plan on this ctx alone
 * (one rank), the faithful executor for what the plan refuses -- the same bytes */
int qe_plan_exec_query(struct qe_ctx* ctx, query_t* q, FILE* out);

#ifdef __cplusplus
}
#endif

#endif
