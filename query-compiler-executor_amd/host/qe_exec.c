/*
 * qe_exec.c -- the host side of libqe: the reference's query frontend and executor, restated
 * in C over the device primitives of include/qe.h.  This is the drop-in for the reference's
 * execute_queries / execute_query / execute_filter / execute_join / print_sums seam
 * (src/utilities.c:258-300, src/filter.c:66-100, src/join.c:630-679, src/utilities.c:197-224).
 *
 * Host work only: parsing (src/parsing.c), predicate arrangement with its quirks
 * (src/pred_arrange.c), and the mid_result state machine (src/join.c:152-292, 486-628).  Every
 * row-sized step (scan, refine, gather, sort, merge, payload propagation, checksum) runs on the
 * GPU through qe_* calls; rowid lists stay in HBM as qe_list and never visit the host.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <setjmp.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/qe.h"
#include "qe_query.h"

/* ------------------------------------------------------------------------------------------ */
/* model                                                                                        */
/* ------------------------------------------------------------------------------------------ */

typedef struct {                 /* mid_result (src/structs.h:44-49), list in HBM */
    qe_mid_t h;                  /* relation, predicate id (binding), last_column_sorted */
    qe_list* list;
} mid_t;

typedef struct { mid_t* e; size_t n, cap; } entity_t;
typedef struct { entity_t** v; size_t n, cap; } mra_t;

typedef qe_where_t exists_t;

enum {
    CLASSIC_JOIN = QE_CLASSIC_JOIN,
    JOIN_SORT_LHS = QE_JOIN_SORT_LHS,
    JOIN_SORT_RHS = QE_JOIN_SORT_RHS,
    SCAN_JOIN = QE_SCAN_JOIN,
    DO_NOTHING = QE_DO_NOTHING
};

typedef struct {
    qe_ctx* q;
    FILE* out;
    jmp_buf jb;                  /* reference exit(EXIT_FAILURE) or a device error */
    int jb_code;
    qe_list** lists;             /* every list made for the current query (freed at its end) */
    size_t nlists, caplists;
    int dle;                     /* dead-list elimination on (QE_DLE=0 turns it off) */
    const uint8_t* live;         /* live[b]: binding b is read by a later predicate or a select */
    const uint8_t* pred_live;    /* pred_live[b]: binding b is read by a later predicate */
    struct agg_side { const qe_list* l; qe_pairs p; } *aggs;   /* unmaterialised join sides */
    size_t naggs, capaggs;
    int last_pred;               /* the predicate running is the query's last */
    struct agg_sum { const qe_list* l; uint64_t col; uint64_t sum; } sums[2];   /* qe_join_aggregate */
    size_t nsums;
} exec_t;

/* Dead-list elimination.  fix_all re-materialises every other entry of the entity
 * (join_payloads, src/join.c:486-505), but an entry whose binding no later predicate and no select
 * reads is never observed again: its CONTENT is skipped, its LENGTH -- the only thing a later
 * join_payloads looks at (the |edit| < |last| guard) -- is kept exactly.  Such a list carries
 * QE_LIST_DEAD (host-only) and no data; reading one is an internal error, not a fallback. */
#define QE_LIST_DEAD 0x40000000u

/* Aggregate join results.  A sorted merge join of more pairs than the materialisation limit
 * (QE_ETOOBIG; the reference's DArray cannot hold them, src/DArray.h:14-15) whose lists only
 * print_sums reads afterwards keeps its sorted inputs with per-row partner counts instead: the
 * list of a side has length P and checksum sum_i col[val[i]] * match[i] (aggregate push-down,
 * SURVEY.md §0.7).  Such a list carries QE_LIST_AGG and no data. */
#define QE_LIST_AGG 0x20000000u

static void need_data(exec_t* x, const qe_list* l);

static void fail(exec_t* x, int code, const char* msg) {
    if (msg) fprintf(stderr, "[ERROR] %s\n", msg);
    x->jb_code = code;
    longjmp(x->jb, 1);
}

static void chk(exec_t* x, int rc) {
    if (rc != 0) {
        fprintf(stderr, "[ERROR] libqe: %s\n", qe_last_error(x->q));
        fail(x, rc, NULL);
    }
}

static void need_data(exec_t* x, const qe_list* l) {
    if (l && (l->flags & QE_LIST_DEAD)) fail(x, QE_EINVAL, "internal: a dead-eliminated list was read");
    if (l && (l->flags & QE_LIST_AGG)) fail(x, QE_EINVAL, "internal: an aggregate join list was read");
}

static qe_list* new_list(exec_t* x) {
    qe_list* l = (qe_list*)calloc(1, sizeof(qe_list));
    if (x->nlists == x->caplists) {
        x->caplists = x->caplists ? 2 * x->caplists : 64;
        x->lists = (qe_list**)realloc(x->lists, x->caplists * sizeof(qe_list*));
    }
    x->lists[x->nlists++] = l;
    return l;
}

static void free_lists(exec_t* x) {
    for (size_t i = 0; i < x->naggs; i++) qe_pairs_free(x->q, &x->aggs[i].p);
    x->naggs = 0;
    x->nsums = 0;
    for (size_t i = 0; i < x->nlists; i++) {
        qe_list_free(x->q, x->lists[i]);
        free(x->lists[i]);
    }
    x->nlists = 0;
}

static void entity_push(entity_t* E, mid_t m) {
    if (E->n == E->cap) {
        E->cap = E->cap ? 2 * E->cap : 4;
        E->e = (mid_t*)realloc(E->e, E->cap * sizeof(mid_t));
    }
    E->e[E->n++] = m;
}

static entity_t* new_entity(mra_t* M) {          /* create_entity_mid_results, src/join.c:145-150 */
    if (M->n == M->cap) {
        M->cap = M->cap ? 2 * M->cap : 4;
        M->v = (entity_t**)realloc(M->v, M->cap * sizeof(entity_t*));
    }
    entity_t* E = (entity_t*)calloc(1, sizeof(entity_t));
    M->v[M->n++] = E;
    return E;
}

static void mra_free(mra_t* M) {
    for (size_t i = 0; i < M->n; i++) {
        free(M->v[i]->e);
        free(M->v[i]);
    }
    free(M->v);
    memset(M, 0, sizeof(*M));
}

/* mid_results_array as the shared view (host/qe_query.h) */
static size_t v_count(void* u) { return ((mra_t*)u)->n; }
static size_t v_size(void* u, size_t ent) { return ((mra_t*)u)->v[ent]->n; }
static qe_mid_t* v_at(void* u, size_t ent, size_t idx) { return &((mra_t*)u)->v[ent]->e[idx].h; }
static void v_push_entity(void* u) { (void)new_entity((mra_t*)u); }

static qe_mids view(const mra_t* M) {
    qe_mids v = {(void*)M, v_count, v_size, v_at, v_push_entity};
    return v;
}

/* relation_exists (src/utilities.c:164-181) */
static exists_t relation_exists(const mra_t* M, uint64_t relation, uint64_t pid) {
    const qe_mids v = view(M);
    return qe_mid_exists(&v, relation, pid);
}

static qe_col column(exec_t* x, uint64_t relation, uint64_t col) {
    qe_col c;
    if (qe_relation_column(x->q, (int)relation, (int)col, &c) != 0) fail(x, QE_EINVAL, "no such relation/column");
    return c;
}

static uint64_t rows_of(exec_t* x, uint64_t relation) {
    uint64_t r = 0;
    if (qe_relation_rows(x->q, (int)relation, &r) != 0) fail(x, QE_EINVAL, "no such relation");
    return r;
}

/* ------------------------------------------------------------------------------------------ */
/* joins                                                                                         */
/* ------------------------------------------------------------------------------------------ */

typedef struct {
    qe_list* res[2];             /* join_result.results[0/1] */
    qe_pairs* R;                 /* the join inputs, kept for the driver-count fast path */
    qe_pairs* S;
    const qe_list* src[2];       /* the lists R / S were gathered from (NULL: a base column) */
} jres_t;

/* allocate_relation (src/join.c:122-142) / allocate_relation_mid_results (src/join.c:96-120) */
static void gather(exec_t* x, qe_pairs* out, uint64_t relation, uint64_t col, const qe_list* rows) {
    if (rows) need_data(x, rows);
    chk(x, qe_gather_pairs(x->q, column(x, relation, col), rows, out));
}

static void ensure_sorted_flag(exec_t* x, qe_pairs* p) {
    if (p->flags & QE_PAIRS_SORTED) return;
    int s = 0;
    chk(x, qe_is_sorted(x->q, p, &s));
    if (s) p->flags |= QE_PAIRS_SORTED;
}

/* non_duplicates[mode] as driver counts, then join_payloads for every other entry of the
 * entity (fix_all_mid_results, src/join.c:486-505) */
static void fix_all(exec_t* x, const jres_t* jr, exists_t ex, mra_t* M, uint32_t relR, uint32_t relS, mid_t tmp,
                    int mode) {
    entity_t* E = M->v[ex.ent];
    qe_list* update = E->e[ex.idx].list;
    /* which entries get join_payloads: every other one; with DLE only those still read later */
    uint8_t* pick = (uint8_t*)calloc(E->n ? E->n : 1, 1);
    size_t nedit = 0, npick = 0;
    ptrdiff_t first_edit = -1;
    for (size_t i = 0; i < E->n; i++)
        if (E->e[i].h.relation != relR && E->e[i].h.relation != relS) {
            nedit++;
            if (first_edit < 0) first_edit = (ptrdiff_t)i;
            if (!x->dle || x->live[E->e[i].h.pid]) {
                pick[i] = 1;
                npick++;
            }
        }
    if (nedit) {
        for (size_t i = 0; i < E->n; i++)   /* join_payloads' guard, on every entry, dead or not */
            if (E->e[i].h.relation != relR && E->e[i].h.relation != relS && E->e[i].list->n < update->n) {
                free(pick);
                fail(x, QE_EINVAL, "join_payloads on lists of different lengths (reference-undefined)");
            }
        /* join_payloads' output length is the sum over `update` of the driver count.  When the
         * counts come from the sorted fast path (the other side's rowids distinct) and `update` is
         * the list this side was gathered from, that sum IS the join's pair count. */
        const qe_pairs* me = mode == 0 ? jr->R : jr->S;
        const qe_pairs* other = mode == 0 ? jr->S : jr->R;
        const int p_known = (me->flags & QE_PAIRS_SORTED) && (other->flags & QE_PAIRS_SORTED) &&
                            (other->flags & QE_PAIRS_DISTINCT) && jr->src[mode] == update;
        if (npick == 0 && !p_known) {       /* materialise one entry to learn the length */
            pick[first_edit] = 1;
            npick = 1;
        }
        uint64_t P = jr->res[0]->n;
        qe_list* outs = NULL;
        if (npick) {
            need_data(x, update);
            uint64_t rows = rows_of(x, E->e[ex.idx].h.relation);
            uint32_t* counts = NULL;
            chk(x, qe_driver_counts(x->q, jr->R, jr->S, jr->res[0], jr->res[1], mode, rows, &counts));
            const qe_list** edits = (const qe_list**)malloc(npick * sizeof(qe_list*));
            outs = (qe_list*)calloc(npick, sizeof(qe_list));
            size_t k = 0;
            for (size_t i = 0; i < E->n; i++)
                if (pick[i]) {
                    need_data(x, E->e[i].list);
                    edits[k++] = E->e[i].list;
                }
            int rc = qe_join_payloads_multi(x->q, counts, rows, update, edits, (int)npick, outs);
            qe_counts_free(x->q, counts);
            free(edits);
            if (rc != 0) {
                free(outs);
                free(pick);
                if (rc == QE_EINVAL) fail(x, QE_EINVAL, "join_payloads on lists of different lengths (reference-undefined)");
                chk(x, rc);
            }
            P = outs[0].n;
        }
        size_t k = 0;
        for (size_t i = 0; i < E->n; i++) {
            mid_t* ed = &E->e[i];
            if (ed->h.relation == relR || ed->h.relation == relS) continue;
            qe_list* nl = new_list(x);
            if (pick[i]) {
                *nl = outs[k++];
            } else {
                nl->n = P;
                nl->flags = QE_LIST_DEAD;
            }
            ed->list = nl;
        }
        free(outs);
    }
    free(pick);
    E->e[ex.idx] = tmp;
}

/* update_mid_results (src/join.c:507-628) */
static void update_mid_results(exec_t* x, const jres_t* jr, mra_t* M, uint64_t relR, uint64_t predR, uint64_t colR,
                               uint64_t relS, uint64_t predS, uint64_t colS, int join_id) {
    mid_t tR = {{relR, predR, (int32_t)colR}, jr->res[0]};
    mid_t tS = {{relS, predS, (int32_t)colS}, jr->res[1]};
    exists_t ex;
    switch (join_id) {
    case CLASSIC_JOIN:
        ex = relation_exists(M, relR, predR);
        if (ex.idx == -1) entity_push(M->v[M->n - 1], tR);
        else fix_all(x, jr, ex, M, (uint32_t)relR, (uint32_t)relS, tR, 0);
        ex = relation_exists(M, relS, predS);
        if (ex.idx == -1) entity_push(M->v[M->n - 1], tS);
        else fix_all(x, jr, ex, M, (uint32_t)relR, (uint32_t)relS, tS, 1);
        break;
    case JOIN_SORT_LHS:
        ex = relation_exists(M, relR, predR);
        if (ex.idx == -1) entity_push(M->v[M->n - 1], tR);
        else M->v[ex.ent]->e[ex.idx] = tR;
        ex = relation_exists(M, relS, predS);
        if (ex.idx == -1) fail(x, QE_EEXIT, "Something went really wrong");
        fix_all(x, jr, ex, M, (uint32_t)relR, (uint32_t)relS, tS, 1);
        break;
    case JOIN_SORT_RHS:
        ex = relation_exists(M, relS, predS);
        if (ex.idx == -1) entity_push(M->v[M->n - 1], tS);
        else M->v[ex.ent]->e[ex.idx] = tS;
        ex = relation_exists(M, relR, predR);
        if (ex.idx == -1) fail(x, QE_EEXIT, "Something went really wrong");
        fix_all(x, jr, ex, M, (uint32_t)relR, (uint32_t)relS, tR, 0);
        break;
    case SCAN_JOIN:
        ex = relation_exists(M, relR, predR);
        if (ex.idx == -1) fail(x, QE_EEXIT, "Something went really wrong");
        M->v[ex.ent]->e[ex.idx].list = jr->res[0];
        ex = relation_exists(M, relS, predS);
        if (ex.idx == -1) fail(x, QE_EEXIT, "Something went really wrong");
        M->v[ex.ent]->e[ex.idx].list = jr->res[1];
        break;
    }
}

/* build_relations (src/join.c:152-292): the variant (host/qe_query.c, shared with the plan's
 * replay), then both inputs gathered from the entries it names (NULL: the whole base relation) */
static int build_relations(exec_t* x, const query_t* q, const pred_t* p, mra_t* M, qe_pairs rel[2],
                           const qe_list* src[2]) {
    const qe_mids v = view(M);
    const qe_join_choice_t j = qe_build_relations(&v, q, p);
    if (j.variant == DO_NOTHING) return DO_NOTHING;
    src[0] = j.lhs.ent >= 0 ? M->v[j.lhs.ent]->e[j.lhs.idx].list : NULL;
    src[1] = j.rhs.ent >= 0 ? M->v[j.rhs.ent]->e[j.rhs.idx].list : NULL;
    gather(x, &rel[0], q->rels[p->frel], p->fcol, src[0]);
    gather(x, &rel[1], q->rels[p->srel], p->scol, src[1]);
    return j.variant;
}

/* fix_all on this entity would re-materialise nothing: it holds no other relation's entry */
static int fix_all_trivial(const mra_t* M, exists_t ex, uint64_t relR, uint64_t relS) {
    if (ex.idx == -1) return 1;
    const entity_t* E = M->v[ex.ent];
    for (size_t i = 0; i < E->n; i++)
        if (E->e[i].h.relation != relR && E->e[i].h.relation != relS) return 0;
    return 1;
}

/* the join's lists may stay unmaterialised: no later predicate reads either binding and
 * update_mid_results only stores them (no join_payloads needs their content) */
static int aggregate_ok(exec_t* x, const query_t* q, const pred_t* p, const mra_t* M, int v) {
    if (x->pred_live[p->frel] || x->pred_live[p->srel]) return 0;
    const uint64_t relR = q->rels[p->frel], relS = q->rels[p->srel];
    const exists_t exR = relation_exists(M, relR, p->frel), exS = relation_exists(M, relS, p->srel);
    switch (v) {
    case CLASSIC_JOIN: return fix_all_trivial(M, exR, relR, relS) && fix_all_trivial(M, exS, relR, relS);
    case JOIN_SORT_LHS: return fix_all_trivial(M, exS, relR, relS);
    case JOIN_SORT_RHS: return fix_all_trivial(M, exR, relR, relS);
    }
    return 0;
}

static void keep_agg(exec_t* x, qe_list* l, qe_pairs* p, uint64_t P) {
    if (x->naggs == x->capaggs) {
        x->capaggs = x->capaggs ? 2 * x->capaggs : 8;
        x->aggs = realloc(x->aggs, x->capaggs * sizeof(*x->aggs));
    }
    x->aggs[x->naggs].l = l;
    x->aggs[x->naggs].p = *p;
    x->naggs++;
    memset(p, 0, sizeof(*p));        /* ownership moved: execute_join's free is a no-op */
    l->d = NULL;
    l->n = P;
    l->cap = 0;
    l->flags = QE_LIST_AGG;
}

/* qe_merge_join, or its aggregate form for a join too large to materialise */
static void merge(exec_t* x, const query_t* q, const pred_t* p, const mra_t* M, int v, qe_pairs rel[2],
                  jres_t* jr) {
    int rc = qe_merge_join(x->q, &rel[0], &rel[1], jr->res[0], jr->res[1]);
    if (rc != QE_ETOOBIG) {
        chk(x, rc);
        return;
    }
    if (!aggregate_ok(x, q, p, M, v)) chk(x, rc);
    uint64_t P = 0;
    chk(x, qe_merge_join_counts(x->q, &rel[0], &rel[1], &P));
    keep_agg(x, jr->res[0], &rel[0], P);
    keep_agg(x, jr->res[1], &rel[1], P);
}

/* The query's last join, of two base columns, whose lists only print_sums reads and whose
 * bindings' selects each name one column with values < 2^32: qe_join_aggregate computes the
 * pair count and both checksums from value-carrying sorts and one counting pass -- the numbers
 * print_sums would compute over the materialised lists, whatever their size.  Joins of fewer
 * than QE_AGG_MIN rows (both sides; default 2^24) keep the merge path. */
static uint64_t agg_min(void) {
    static uint64_t v = (uint64_t)-1;
    if (v == (uint64_t)-1) {
        const char* e = getenv("QE_AGG_MIN");
        v = e ? strtoull(e, NULL, 10) : (1ull << 24);
    }
    return v;
}

/* the one column the selects read from binding b (1), none (0), or several / invalid (-1) */
static int select_col(exec_t* x, const query_t* q, uint64_t b, uint64_t* col) {
    int found = 0;
    for (size_t i = 0; i < q->nsel; i++) {
        if (q->sel[2 * i] != b) continue;
        if (found && q->sel[2 * i + 1] != *col) return -1;
        *col = q->sel[2 * i + 1];
        found = 1;
    }
    if (!found) return 0;
    qe_col c;
    uint64_t kor = 0, kand = 0;
    if (qe_relation_column(x->q, (int)q->rels[b], (int)*col, &c) != 0) return -1;
    if (qe_relation_column_bits(x->q, (int)q->rels[b], (int)*col, &kor, &kand) != 0 || (kor >> 32)) return -1;
    return 1;
}

static int join_aggregate(exec_t* x, const query_t* q, const pred_t* p, const mra_t* M, int v, const qe_pairs rel[2],
                          const qe_list* src[2], jres_t* jr) {
    if (!x->last_pred || v != CLASSIC_JOIN || src[0] || src[1]) return 0;
    if (rel[0].n + rel[1].n < agg_min() || !aggregate_ok(x, q, p, M, v)) return 0;
    uint64_t cR = 0, cS = 0, kb[4];
    const int hR = select_col(x, q, p->frel, &cR), hS = select_col(x, q, p->srel, &cS);
    if (hR < 0 || hS < 0) return 0;
    if (qe_relation_column_bits(x->q, (int)q->rels[p->frel], (int)p->fcol, &kb[0], &kb[1]) != 0 ||
        qe_relation_column_bits(x->q, (int)q->rels[p->srel], (int)p->scol, &kb[2], &kb[3]) != 0)
        return 0;
    const uint64_t vary = (kb[0] | kb[2]) & ~(kb[1] & kb[3]);
    if (vary && 64 - __builtin_clzll(vary) - __builtin_ctzll(vary) > 32) return 0;
    qe_col vR = {NULL, 0}, vS = {NULL, 0};
    if (hR) vR = column(x, q->rels[p->frel], cR);
    if (hS) vS = column(x, q->rels[p->srel], cS);
    uint64_t out[3];
    chk(x, qe_join_aggregate(x->q, column(x, q->rels[p->frel], p->fcol), vR, column(x, q->rels[p->srel], p->scol), vS,
                             out));
    x->nsums = 0;
    for (int side = 0; side < 2; side++) {
        qe_list* l = jr->res[side];
        l->d = NULL;
        l->n = out[0];
        l->cap = 0;
        l->flags = QE_LIST_AGG;
        if (side == 0 ? hR : hS) {
            x->sums[x->nsums].l = l;
            x->sums[x->nsums].col = side == 0 ? cR : cS;
            x->sums[x->nsums].sum = out[1 + side];
            x->nsums++;
        }
    }
    return 1;
}

/* execute_join (src/join.c:630-679) */
static int execute_join(exec_t* x, const query_t* q, const pred_t* p, mra_t* M) {
    qe_pairs rel[2];
    memset(rel, 0, sizeof(rel));
    const qe_list* src[2] = {NULL, NULL};
    int v = build_relations(x, q, p, M, rel, src);
    if (v == DO_NOTHING) return 0;
    jres_t jr;
    jr.res[0] = new_list(x);
    jr.res[1] = new_list(x);
    jr.src[0] = src[0];
    jr.src[1] = src[1];
    jr.R = &rel[0];
    jr.S = &rel[1];
    switch (join_aggregate(x, q, p, M, v, rel, src, &jr) ? -2 : v) {
    case -2:
        break;
    case CLASSIC_JOIN:
        chk(x, qe_sort_pairs(x->q, &rel[0]));
        chk(x, qe_sort_pairs(x->q, &rel[1]));
        merge(x, q, p, M, v, rel, &jr);
        break;
    case JOIN_SORT_LHS:
        chk(x, qe_sort_pairs(x->q, &rel[0]));
        ensure_sorted_flag(x, &rel[1]);
        merge(x, q, p, M, v, rel, &jr);
        break;
    case JOIN_SORT_RHS:
        chk(x, qe_sort_pairs(x->q, &rel[1]));
        ensure_sorted_flag(x, &rel[0]);
        merge(x, q, p, M, v, rel, &jr);
        break;
    case SCAN_JOIN:
        chk(x, qe_scan_join(x->q, &rel[0], &rel[1], jr.res[0], jr.res[1]));
        break;
    default:
        return -1;
    }
    update_mid_results(x, &jr, M, q->rels[p->frel], p->frel, p->fcol, q->rels[p->srel], p->srel, p->scol, v);
    qe_pairs_free(x->q, &rel[0]);
    qe_pairs_free(x->q, &rel[1]);
    return 0;
}

static int op_valid(char op) { return op == '=' || op == '<' || op == '>'; }

/* execute_filter (src/filter.c:66-100) */
static int execute_filter(exec_t* x, const query_t* q, const pred_t* p, mra_t* M) {
    uint64_t relation = q->rels[p->frel];
    qe_col col = column(x, relation, p->fcol);
    entity_t* E = M->n == 0 ? new_entity(M) : M->v[M->n - 1];
    exists_t ex = relation_exists(M, relation, p->frel);
    if (ex.idx != -1) {                                           /* exec_filter_rel_exists */
        qe_list* l = M->v[ex.ent]->e[ex.idx].list;
        need_data(x, l);
        if (!op_valid(p->op)) {
            if (l->n != 0) {
                fprintf(stderr, "[ERROR] Wrong operator\n");
                return -1;
            }
        } else {
            chk(x, qe_filter_refine(x->q, col, p->op, p->cval, l));
        }
        fprintf(x->out, "%d\n", (int)(uint32_t)l->n);             /* src/filter.c:32 */
    } else {                                                      /* exec_filter_rel_no_exists */
        mid_t m = {{relation, p->frel, -1}, new_list(x)};
        entity_push(E, m);
        qe_list* l = m.list;
        if (!op_valid(p->op)) {
            l->n = 0;
            if (col.n != 0) {
                fprintf(stderr, "[ERROR] Wrong operator\n");
                return -1;
            }
            return 0;
        }
        chk(x, qe_filter_scan(x->q, col, p->op, p->cval, l));
    }
    return 0;
}

/* print_sums (src/utilities.c:197-224) */
static void print_sums(exec_t* x, const query_t* q, const mra_t* M) {
    if (q->nsel > 0) {
        exists_t e0 = relation_exists(M, q->rels[q->sel[0]], q->sel[0]);
        if (e0.idx != -1) qe_set_last_result_rows(x->q, M->v[e0.ent]->e[e0.idx].list->n);
    }
    /* the plain sums of the selects before the first missing binding are computed together (one
     * host round trip); the line is then printed in order exactly as the loop below prints it */
    size_t nb = 0;
    qe_col* bc = (qe_col*)calloc(q->nsel ? q->nsel : 1, sizeof(qe_col));
    const qe_list** bl = (const qe_list**)calloc(q->nsel ? q->nsel : 1, sizeof(qe_list*));
    uint64_t* bs = (uint64_t*)calloc(q->nsel ? q->nsel : 1, sizeof(uint64_t));
    for (size_t i = 0; i < q->nsel; i++) {
        uint64_t b = q->sel[2 * i], colno = q->sel[2 * i + 1];
        exists_t ex = relation_exists(M, q->rels[b], b);
        if (ex.idx == -1) break;
        const qe_list* l = M->v[ex.ent]->e[ex.idx].list;
        if (l->n == 0 || (l->flags & (QE_LIST_AGG | QE_LIST_DEAD))) continue;
        if (qe_relation_column(x->q, (int)q->rels[b], (int)colno, &bc[nb]) != 0) break;   /* fails in order below */
        bl[nb++] = l;
    }
    int brc = nb ? qe_checksums(x->q, (int)nb, bc, bl, bs) : 0;
    free(bc);
    free(bl);
    if (brc != 0) {
        free(bs);
        chk(x, brc);
    }
    size_t k = 0;
    for (size_t i = 0; i < q->nsel; i++) {
        uint64_t b = q->sel[2 * i], colno = q->sel[2 * i + 1];
        uint32_t relation = q->rels[b];
        exists_t ex = relation_exists(M, relation, b);
        if (ex.idx == -1) {
            free(bs);
            fail(x, QE_EEXIT, "Something went really wrong...");
        }
        const qe_list* l = M->v[ex.ent]->e[ex.idx].list;
        if (l->n == 0) {
            fputs("NULL ", x->out);
        } else {
            uint64_t s = 0;
            const qe_pairs* agg = NULL;
            for (size_t a = 0; a < x->naggs && (l->flags & QE_LIST_AGG); a++)
                if (x->aggs[a].l == l) agg = &x->aggs[a].p;
            const struct agg_sum* as = NULL;
            for (size_t a = 0; a < x->nsums && (l->flags & QE_LIST_AGG); a++)
                if (x->sums[a].l == l && x->sums[a].col == colno) as = &x->sums[a];
            if (as) {
                (void)column(x, relation, colno);   /* the same validation, at its place in the line */
                s = as->sum;
            } else if (agg) {
                chk(x, qe_checksum_weighted(x->q, column(x, relation, colno), agg, &s));
            } else if (!(l->flags & (QE_LIST_AGG | QE_LIST_DEAD)) && k < nb) {
                (void)column(x, relation, colno);   /* the same validation, at its place in the line */
                s = bs[k++];
            } else {
                need_data(x, l);
                chk(x, qe_checksum(x->q, column(x, relation, colno), l, &s));
            }
            fprintf(x->out, "%lu ", (unsigned long)s);
        }
    }
    free(bs);
    fputc('\n', x->out);
}

/* ------------------------------------------------------------------------------------------ */
/* frontend                                                                                     */
/* ------------------------------------------------------------------------------------------ */

static int query_valid(exec_t* x, const query_t* q) {
    int nrel = qe_relation_count(x->q);
    for (size_t i = 0; i < q->nrels; i++)
        if ((int)q->rels[i] >= nrel) return 0;
    for (size_t i = 0; i < q->npreds; i++) {
        const pred_t* p = &q->preds[i];
        if (p->type < 0 || p->frel >= q->nrels) return 0;
        qe_col c;
        if (qe_relation_column(x->q, (int)q->rels[p->frel], (int)p->fcol, &c) != 0) return 0;
        if (p->type == 0) {
            if (p->srel >= q->nrels) return 0;
            if (qe_relation_column(x->q, (int)q->rels[p->srel], (int)p->scol, &c) != 0) return 0;
        }
    }
    for (size_t i = 0; i < q->nsel; i++) {
        qe_col c;
        if (q->sel[2 * i] >= q->nrels) return 0;
        if (qe_relation_column(x->q, (int)q->rels[q->sel[2 * i]], (int)q->sel[2 * i + 1], &c) != 0) return 0;
    }
    return 1;
}

/* execute_query (src/utilities.c:258-287): a failed predicate drops the output line */
static void execute_query(exec_t* x, query_t* q) {
    mra_t M;
    memset(&M, 0, sizeof(M));
    int ok = query_valid(x, q);   /* out-of-range ids are undefined in the reference: no line */
    uint8_t* live = (uint8_t*)calloc(q->nrels ? q->nrels : 1, 1);
    uint8_t* pred_live = (uint8_t*)calloc(q->nrels ? q->nrels : 1, 1);
    for (size_t i = 0; ok && i < q->npreds; i++) {
        /* bindings read after predicate i: later predicates, and those or the selects */
        memset(pred_live, 0, q->nrels ? q->nrels : 1);
        for (size_t j = i + 1; j < q->npreds; j++) {
            pred_live[q->preds[j].frel] = 1;
            if (q->preds[j].type == 0) pred_live[q->preds[j].srel] = 1;
        }
        memcpy(live, pred_live, q->nrels ? q->nrels : 1);
        for (size_t s = 0; s < q->nsel; s++) live[q->sel[2 * s]] = 1;
        x->live = live;
        x->pred_live = pred_live;
        const pred_t* p = &q->preds[i];
        x->last_pred = i + 1 == q->npreds;
        int r = p->type == 1 ? execute_filter(x, q, p, &M) : execute_join(x, q, p, &M);
        if (r == -1) ok = 0;
    }
    x->live = x->pred_live = NULL;
    x->last_pred = 0;
    free(live);
    free(pred_live);
    if (ok) print_sums(x, q, &M);
    mra_free(&M);
    free_lists(x);
}

/* execute_queries (src/utilities.c:289-300); a reference exit(EXIT_FAILURE) or a device
 * error unwinds here */
static int run_all(exec_t* x, query_t* qs, size_t nq) {
    if (setjmp(x->jb) != 0) {
        free_lists(x);
        return x->jb_code;
    }
    for (size_t qi = 0; qi < nq; qi++) {
        qe_arrange_predicates(&qs[qi]);
        execute_query(x, &qs[qi]);
    }
    return 0;
}

/* one parsed, already arranged query through the faithful executor, printing to `out` (the
 * partitioned plan's fallback for queries outside its domain, qe_plan.h) */
int qe_exec_query(qe_ctx* ctx, query_t* q, FILE* out) {
    exec_t x;
    memset(&x, 0, sizeof(x));
    x.q = ctx;
    const char* e = getenv("QE_DLE");
    x.dle = !(e && e[0] == '0');
    x.out = out;
    int rc = 0;
    if (setjmp(x.jb) != 0) {
        free_lists(&x);
        rc = x.jb_code;
    } else {
        execute_query(&x, q);
    }
    free(x.lists);
    free(x.aggs);
    return rc;
}

int qe_run_queries(qe_ctx* ctx, const char* text, char** out, size_t* outlen) {
    exec_t x;
    memset(&x, 0, sizeof(x));
    x.q = ctx;
    {
        const char* e = getenv("QE_DLE");
        x.dle = !(e && e[0] == '0');
    }
    *out = NULL;
    *outlen = 0;
    x.out = open_memstream(out, outlen);
    if (!x.out) return QE_ENOMEM;

    size_t nq = 0;
    query_t* qs = qe_parse_text(text, &nq);   /* parsed before anything runs (main/queries_main.c:31-37) */

    int rc = run_all(&x, qs, nq);
    qe_free_queries(qs, nq);
    free(x.lists);
    free(x.aggs);
    fclose(x.out);
    return rc;
}

/* ---- the concurrent batch (qe_run_queries_parallel) ----------------------------------------- */

typedef struct {
    qe_ctx* ctx;
    query_t* qs;
    size_t nq;
    atomic_size_t* next;
    char** outs;
    size_t* lens;
    int* rcs;
    atomic_int* stop;          /* the first query index known to end the batch (+1), 0 none */
    int plan;                  /* QE_EXEC_PLAN: the partitioned plan, faithful fallback */
} lane_t;

static void* lane_main(void* arg) {
    lane_t* L = (lane_t*)arg;
    qe_bind_thread(L->ctx);
    for (;;) {
        const size_t i = atomic_fetch_add(L->next, 1);
        if (i >= L->nq) break;
        const int st = atomic_load(L->stop);
        if (st && (size_t)(st - 1) < i) {       /* past a query where the reference exits */
            L->rcs[i] = 0;
            continue;
        }
        FILE* f = open_memstream(&L->outs[i], &L->lens[i]);
        if (!f) {
            L->rcs[i] = QE_ENOMEM;
        } else {
            qe_arrange_predicates(&L->qs[i]);
            L->rcs[i] = L->plan ? qe_plan_exec_query(L->ctx, &L->qs[i], f) : qe_exec_query(L->ctx, &L->qs[i], f);
            fclose(f);
        }
        if (L->rcs[i] != 0) {                   /* remember the earliest failing query */
            int cur = atomic_load(L->stop);
            while ((cur == 0 || (size_t)(cur - 1) > i) && !atomic_compare_exchange_weak(L->stop, &cur, (int)i + 1)) {
            }
        }
    }
    return NULL;
}

int qe_run_queries_parallel(qe_ctx* ctx, int workers, const char* text, char** out, size_t* outlen) {
    return qe_run_queries_lanes(ctx, workers, QE_EXEC_FAITHFUL, text, out, outlen);
}

int qe_run_queries_lanes(qe_ctx* ctx, int workers, int executor, const char* text, char** out, size_t* outlen) {
    *out = NULL;
    *outlen = 0;
    if (executor != QE_EXEC_FAITHFUL && executor != QE_EXEC_PLAN) return QE_EINVAL;
    const int plan = executor == QE_EXEC_PLAN;
    if (workers <= 1) {
        if (!plan) return qe_run_queries(ctx, text, out, outlen);
        uint64_t refused = 0;
        int rc = qe_sort_cache(ctx, 1);          /* the batch's base-column sorts, shared */
        if (rc == 0) rc = qe_run_queries_dist(ctx, NULL, text, out, outlen, &refused);
        const int rc2 = qe_sort_cache(ctx, 0);
        return rc != 0 ? rc : rc2;
    }
    qe_ctx* w[16];
    int rc = qe_workers(ctx, workers, w);
    if (rc != 0) return rc;
    if (plan && (rc = qe_sort_cache(ctx, 1)) != 0) return rc;   /* shared by the lanes */
    size_t nq = 0;
    query_t* qs = qe_parse_text(text, &nq);     /* parsed before anything runs (main/queries_main.c:31-37) */
    char** outs = (char**)calloc(nq ? nq : 1, sizeof(char*));
    size_t* lens = (size_t*)calloc(nq ? nq : 1, sizeof(size_t));
    int* rcs = (int*)calloc(nq ? nq : 1, sizeof(int));
    atomic_size_t next = 0;
    atomic_int stop = 0;
    lane_t lanes[16];
    pthread_t th[16];
    int started = 0;
    for (int k = 0; k < workers; k++) {
        lane_t l = {w[k], qs, nq, &next, outs, lens, rcs, &stop, plan};
        lanes[k] = l;
        if (pthread_create(&th[k], NULL, lane_main, &lanes[k]) == 0) started++;
        else break;
    }
    if (started == 0) lane_main(&lanes[0]);      /* no threads: run the batch on one lane */
    for (int k = 0; k < started; k++) pthread_join(th[k], NULL);
    for (int k = 0; k < workers; k++) qe_sync(w[k]);
    const int rc_cache = qe_sort_cache(ctx, 0);
    /* the reference's bytes: every query in input order, up to and including the first that ends
     * the batch (its partial output, then its status) */
    FILE* f = open_memstream(out, outlen);
    rc = 0;
    for (size_t i = 0; f && i < nq; i++) {
        if (outs[i] && lens[i]) fwrite(outs[i], 1, lens[i], f);
        if (rcs[i] != 0) {
            rc = rcs[i];
            break;
        }
    }
    if (f) fclose(f);
    else rc = QE_ENOMEM;
    if (rc == 0) rc = rc_cache;
    for (size_t i = 0; i < nq; i++) free(outs[i]);
    free(outs);
    free(lens);
    free(rcs);
    qe_free_queries(qs, nq);
    return rc;
}

