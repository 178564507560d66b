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

struct qe_ctx;
/* host/qe_exec.c: one parsed, arranged query through the faithful executor (0, QE_EEXIT, <0) */
int qe_exec_query(struct qe_ctx* ctx, query_t* q, FILE* out);

#ifdef __cplusplus
}
#endif

#endif
