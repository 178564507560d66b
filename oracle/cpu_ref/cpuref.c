/*
 * cpuref.c -- CPU restatement of the reference query path.  TEST INFRASTRUCTURE ONLY
 * (see cpuref.h for scope, citations and how parity is pinned).  Citations are
 * path:line inside the reference tree giorgosLiako/Query-Compiler-Executor.
 */
#define _GNU_SOURCE
#include "cpuref.h"

#include <setjmp.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------ */
/* data model                                                                            */
/* ------------------------------------------------------------------------------------ */

typedef struct { uint64_t rows, ncols; const uint64_t* const* cols; } rel_t;  /* metadata, src/structs.h:17-21 */

typedef struct { uint32_t* v; uint64_t n, cap; } list_t;                  /* a payload DArray, src/DArray.h */

typedef struct {                                                           /* mid_result, src/structs.h:44-49 */
    uint64_t relation;
    uint64_t pid;          /* binding ("predicate_id") */
    int32_t  lcs;          /* last_column_sorted */
    list_t*  list;
} mid_t;

typedef struct { mid_t* e; size_t n, cap; } entity_t;                      /* DArray<mid_result> */
typedef struct { entity_t** v; size_t n, cap; } mra_t;                     /* mid_results_array */

typedef struct {                                                           /* predicate, src/structs.h:29-34 */
    int8_t   type;         /* 0 join, 1 filter, -1 unparsed (reference-undefined) */
    uint64_t frel, fcol;   /* first: (binding, column) */
    uint64_t srel, scol;   /* join: second (binding, column); filter: (constant, 0) as is_match reads it */
    char     op;
    uint64_t cval;         /* filter constant: uint32 zero-extended (src/filter.c:70) */
} pred_t;

typedef struct {                                                           /* query, src/structs.h:36-43 */
    uint32_t* rels;  size_t nrels;
    pred_t*   preds; size_t npreds;
    uint64_t* sel;   size_t nsel;   /* pairs (binding, column) */
} query_t;

typedef struct { uint64_t* key; uint32_t* pay; uint64_t n; } trel_t;       /* relation of tuples (SoA) */

typedef struct { ptrdiff_t ent, idx; } exists_t;                           /* exists_info, src/utilities.h:14-17 */

enum { CLASSIC_JOIN = 1, JOIN_SORT_LHS = 2, JOIN_SORT_RHS = 3, SCAN_JOIN = 4, DO_NOTHING = 5 }; /* src/join.h:15-19 */

struct cpuref_ctx {
    rel_t*  rels; size_t nrels, caprels;
    /* per-query allocation registry (the reference leaks or frees piecemeal; we free at query end) */
    void**  reg;  size_t nreg, capreg;
    jmp_buf exit_jmp;     /* reference exit(EXIT_FAILURE) → unwind to cpuref_run */
    FILE*   out;
};

static void* reg_add(cpuref_ctx* c, void* p) {
    if (c->nreg == c->capreg) {
        c->capreg = c->capreg ? c->capreg * 2 : 256;
        c->reg = (void**)realloc(c->reg, c->capreg * sizeof(void*));
    }
    c->reg[c->nreg++] = p;
    return p;
}
static void reg_free_all(cpuref_ctx* c) {
    for (size_t i = 0; i < c->nreg; i++) free(c->reg[i]);
    c->nreg = 0;
}
static void* xmalloc(cpuref_ctx* c, size_t bytes) {
    void* p = malloc(bytes ? bytes : 1);
    if (!p) { fprintf(stderr, "cpuref: out of memory (%zu bytes)\n", bytes); abort(); }
    return reg_add(c, p);
}

static list_t* list_new(cpuref_ctx* c, uint64_t cap) {
    list_t* l = (list_t*)xmalloc(c, sizeof(list_t));
    l->n = 0; l->cap = cap ? cap : 4;
    l->v = (uint32_t*)malloc(l->cap * sizeof(uint32_t));
    reg_add(c, l->v);
    return l;
}
static void list_push(cpuref_ctx* c, list_t* l, uint32_t x) {
    if (l->n == l->cap) {
        /* the registry holds the old pointer: swap it for the new one */
        uint32_t* old = l->v;
        l->cap *= 2;
        l->v = (uint32_t*)realloc(l->v, l->cap * sizeof(uint32_t));
        if (!l->v) { fprintf(stderr, "cpuref: out of memory\n"); abort(); }
        for (size_t i = c->nreg; i-- > 0;) if (c->reg[i] == old) { c->reg[i] = l->v; break; }
    }
    l->v[l->n++] = x;
}

static void entity_push(entity_t* E, mid_t m) {
    if (E->n == E->cap) { E->cap = E->cap ? E->cap * 2 : 4; E->e = (mid_t*)realloc(E->e, E->cap * sizeof(mid_t)); }
    E->e[E->n++] = m;
}
static entity_t* mra_new_entity(mra_t* M) {                               /* create_entity_mid_results, src/join.c:145-150 */
    if (M->n == M->cap) { M->cap = M->cap ? M->cap * 2 : 4; M->v = (entity_t**)realloc(M->v, M->cap * sizeof(entity_t*)); }
    entity_t* E = (entity_t*)calloc(1, sizeof(entity_t));
    M->v[M->n++] = E;
    return E;
}
static void mra_free(mra_t* M) {
    for (size_t i = 0; i < M->n; i++) { free(M->v[i]->e); free(M->v[i]); }
    free(M->v);
    M->v = NULL; M->n = M->cap = 0;
}

static void ref_exit_failure(cpuref_ctx* c, const char* msg) {
    fprintf(stderr, "[ERROR] %s\n", msg);
    longjmp(c->exit_jmp, 1);
}

/* relation_exists: newest entity first, entries ascending, first match (src/utilities.c:164-181) */
static exists_t relation_exists(mra_t* M, uint64_t relation, uint64_t pid) {
    exists_t ex = { -1, -1 };
    for (ptrdiff_t i = (ptrdiff_t)M->n - 1; i >= 0; i--) {
        entity_t* E = M->v[i];
        for (size_t j = 0; j < E->n; j++)
            if (E->e[j].relation == relation && E->e[j].pid == pid) { ex.ent = i; ex.idx = (ptrdiff_t)j; return ex; }
    }
    return ex;
}
/* relation_exists_current: last match within one entity (src/utilities.c:183-194) */
static ptrdiff_t relation_exists_current(entity_t* E, uint64_t relation, uint64_t pid) {
    ptrdiff_t found = -1;
    for (size_t i = 0; i < E->n; i++)
        if (E->e[i].relation == relation && E->e[i].pid == pid) found = (ptrdiff_t)i;
    return found;
}

/* ------------------------------------------------------------------------------------ */
/* primitives                                                                             */
/* ------------------------------------------------------------------------------------ */

/* Stable LSD radix sort by 64-bit key (replaces iterative_sort + random_quicksort,
 * src/join.c:5-94, src/quicksort.c:7-64; same ascending key order).  8-bit digits,
 * digits on which every key agrees are skipped. */
static void sort_trel(trel_t* r) {
    uint64_t n = r->n;
    if (n < 2) return;
    uint64_t (*hist)[256] = (uint64_t(*)[256])calloc(8, sizeof(uint64_t[256]));
    for (uint64_t i = 0; i < n; i++) {
        uint64_t k = r->key[i];
        for (int d = 0; d < 8; d++) hist[d][(k >> (8 * d)) & 0xFF]++;
    }
    uint64_t* k2 = (uint64_t*)malloc(n * sizeof(uint64_t));
    uint32_t* p2 = (uint32_t*)malloc(n * sizeof(uint32_t));
    uint64_t* ks = r->key; uint32_t* ps = r->pay;
    uint64_t* kd = k2;     uint32_t* pd = p2;
    for (int d = 0; d < 8; d++) {
        int trivial = 0;
        for (int b = 0; b < 256; b++) if (hist[d][b] == n) { trivial = 1; break; }
        if (trivial) continue;
        uint64_t off[256], s = 0;
        for (int b = 0; b < 256; b++) { off[b] = s; s += hist[d][b]; }
        for (uint64_t i = 0; i < n; i++) {
            uint64_t o = off[(ks[i] >> (8 * d)) & 0xFF]++;
            kd[o] = ks[i]; pd[o] = ps[i];
        }
        uint64_t* tk = ks; ks = kd; kd = tk;
        uint32_t* tp = ps; ps = pd; pd = tp;
    }
    if (ks != r->key) {
        memcpy(r->key, ks, n * sizeof(uint64_t));
        memcpy(r->pay, ps, n * sizeof(uint32_t));
    }
    free(k2); free(p2); free(hist);
}

static trel_t trel_alloc(cpuref_ctx* c, uint64_t n) {
    trel_t t;
    t.n = n;
    t.key = (uint64_t*)xmalloc(c, n * sizeof(uint64_t));
    t.pay = (uint32_t*)xmalloc(c, n * sizeof(uint32_t));
    return t;
}

/* allocate_relation: (key = column value, payload = rowid) over the base column (src/join.c:122-142) */
static trel_t gather_base(cpuref_ctx* c, uint64_t relation, uint64_t col) {
    const rel_t* R = &c->rels[relation];
    trel_t t = trel_alloc(c, R->rows);
    const uint64_t* v = R->cols[col];
    for (uint64_t i = 0; i < R->rows; i++) { t.key[i] = v[i]; t.pay[i] = (uint32_t)i; }
    return t;
}
/* allocate_relation_mid_results: same, in list order (src/join.c:96-120) */
static trel_t gather_list(cpuref_ctx* c, const list_t* l, uint64_t relation, uint64_t col) {
    const uint64_t* v = c->rels[relation].cols[col];
    trel_t t = trel_alloc(c, l->n);
    for (uint64_t i = 0; i < l->n; i++) { t.key[i] = v[l->v[i]]; t.pay[i] = l->v[i]; }
    return t;
}

typedef struct { list_t* res[2]; } jres_t;   /* join_result (src/join.h:21-24); non_duplicates derived on demand */

/* join_relations: the literal two-pointer loop (src/join.c:342-377), valid on unsorted input too. */
static jres_t join_relations(cpuref_ctx* c, const trel_t* R, const trel_t* S) {
    jres_t jr;
    jr.res[0] = list_new(c, 1024);
    jr.res[1] = list_new(c, 1024);
    uint64_t pr = 0, s_start = 0;
    while (pr < R->n && s_start < S->n) {
        uint64_t ps = s_start;
        int flag = 0;
        while (ps < S->n) {
            if (R->key[pr] < S->key[ps]) break;
            if (R->key[pr] > S->key[ps]) {
                ps++;
                if (flag == 0) s_start = ps;
            } else {
                list_push(c, jr.res[0], R->pay[pr]);
                list_push(c, jr.res[1], S->pay[ps]);
                flag = 1;
                ps++;
            }
        }
        pr++;
    }
    return jr;
}

/* scan_join: positional compare (src/join.c:395-423) */
static jres_t scan_join(cpuref_ctx* c, const trel_t* R, const trel_t* S) {
    jres_t jr;
    jr.res[0] = list_new(c, 1024);
    jr.res[1] = list_new(c, 1024);
    uint64_t it = R->n < S->n ? R->n : S->n;
    for (uint64_t i = 0; i < it; i++)
        if (R->key[i] == S->key[i]) { list_push(c, jr.res[0], R->pay[i]); list_push(c, jr.res[1], S->pay[i]); }
    return jr;
}

/* non_duplicates[mode]: the mode-side component of each distinct (pR,pS) pair, first
 * occurrence first (src/join.c:358-367 with Hashmap_get/set, exact pair equality,
 * src/hashmap.c:105-138).  A pure function of the aligned result lists. */
static list_t* non_duplicates(cpuref_ctx* c, const jres_t* jr, int mode) {
    uint64_t n = jr->res[0]->n;
    uint64_t cap = 16;
    while (cap < 2 * n + 16) cap <<= 1;
    uint64_t* tab = (uint64_t*)malloc(cap * sizeof(uint64_t));
    for (uint64_t i = 0; i < cap; i++) tab[i] = ~0ull;   /* pR,pS < 2^32 - 1 in practice */
    list_t* out = list_new(c, n + 1);
    for (uint64_t i = 0; i < n; i++) {
        uint64_t key = ((uint64_t)jr->res[0]->v[i] << 32) | jr->res[1]->v[i];
        uint64_t h = key * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29;
        uint64_t s = h & (cap - 1);
        for (;;) {
            if (tab[s] == ~0ull) { tab[s] = key; list_push(c, out, jr->res[mode]->v[i]); break; }
            if (tab[s] == key) break;
            s = (s + 1) & (cap - 1);
        }
    }
    free(tab);
    return out;
}

/* join_payloads (src/join.c:426-484): R = (last[i], edit[i]), S = (driver[j], 0), both
 * sorted, literal merge emitting R.payload.  The reference reads edit[i] for every
 * i < |last| (DArray_get bounds only by capacity): |edit| < |last| is undefined there. */
static list_t* join_payloads(cpuref_ctx* c, const list_t* driver, const list_t* last, const list_t* edit) {
    if (edit->n < last->n) ref_exit_failure(c, "join_payloads: |edit| < |last| (reference-undefined)");
    trel_t R = trel_alloc(c, last->n);
    for (uint64_t i = 0; i < last->n; i++) { R.key[i] = last->v[i]; R.pay[i] = edit->v[i]; }
    trel_t S = trel_alloc(c, driver->n);
    for (uint64_t i = 0; i < driver->n; i++) { S.key[i] = driver->v[i]; S.pay[i] = 0; }
    sort_trel(&R);
    sort_trel(&S);
    list_t* out = list_new(c, 1024);
    uint64_t pr = 0, s_start = 0;
    while (pr < R.n && s_start < S.n) {
        uint64_t ps = s_start;
        int flag = 0;
        while (ps < S.n) {
            if (R.key[pr] < S.key[ps]) break;
            if (R.key[pr] > S.key[ps]) {
                ps++;
                if (flag == 0) s_start = ps;
            } else {
                list_push(c, out, R.pay[pr]);
                flag = 1;
                ps++;
            }
        }
        pr++;
    }
    return out;
}

/* fix_all_mid_results (src/join.c:486-505) */
static void fix_all(cpuref_ctx* c, const jres_t* jr, exists_t ex, mra_t* M, uint32_t relR, uint32_t relS,
                    mid_t tmp, int mode) {
    list_t* nd = non_duplicates(c, jr, mode);
    entity_t* E = M->v[ex.ent];
    list_t* update_list = E->e[ex.idx].list;
    for (size_t i = 0; i < E->n; i++) {
        mid_t* ed = &E->e[i];
        if (ed->relation != relR && ed->relation != relS)
            ed->list = join_payloads(c, nd, update_list, ed->list);
    }
    E->e[ex.idx] = tmp;   /* DArray_set(mid_results, exists.index, &tmp) */
}

/* update_mid_results (src/join.c:507-628) */
static void update_mid_results(cpuref_ctx* c, const jres_t* jr, mra_t* M, uint64_t relR, uint64_t predR,
                               uint64_t colR, uint64_t relS, uint64_t predS, uint64_t colS, int join_id) {
    mid_t tR = { relR, predR, (int32_t)colR, jr->res[0] };
    mid_t tS = { relS, predS, (int32_t)colS, jr->res[1] };
    if (join_id == CLASSIC_JOIN) {
        exists_t ex = relation_exists(M, relR, predR);
        if (ex.idx == -1) entity_push(M->v[M->n - 1], tR);
        else fix_all(c, jr, ex, M, (uint32_t)relR, (uint32_t)relS, tR, 0);
        ex = relation_exists(M, relS, predS);
        if (ex.idx == -1) entity_push(M->v[M->n - 1], tS);
        else fix_all(c, jr, ex, M, (uint32_t)relR, (uint32_t)relS, tS, 1);
    } else if (join_id == JOIN_SORT_LHS) {
        exists_t ex = relation_exists(M, relR, predR);
        if (ex.idx == -1) entity_push(M->v[M->n - 1], tR);
        else M->v[ex.ent]->e[ex.idx] = tR;
        ex = relation_exists(M, relS, predS);
        if (ex.idx == -1) ref_exit_failure(c, "Something went really wrong");
        fix_all(c, jr, ex, M, (uint32_t)relR, (uint32_t)relS, tS, 1);
    } else if (join_id == JOIN_SORT_RHS) {
        exists_t ex = relation_exists(M, relS, predS);
        if (ex.idx == -1) entity_push(M->v[M->n - 1], tS);
        else M->v[ex.ent]->e[ex.idx] = tS;
        ex = relation_exists(M, relR, predR);
        if (ex.idx == -1) ref_exit_failure(c, "Something went really wrong");
        fix_all(c, jr, ex, M, (uint32_t)relR, (uint32_t)relS, tR, 0);
    } else if (join_id == SCAN_JOIN) {
        exists_t ex = relation_exists(M, relR, predR);
        if (ex.idx == -1) ref_exit_failure(c, "Something went really wrong");
        M->v[ex.ent]->e[ex.idx].list = jr->res[0];
        ex = relation_exists(M, relS, predS);
        if (ex.idx == -1) ref_exit_failure(c, "Something went really wrong");
        M->v[ex.ent]->e[ex.idx].list = jr->res[1];
    }
}

/* build_relations (src/join.c:152-292): chooses the join variant and gathers both inputs */
static int build_relations(cpuref_ctx* c, const query_t* q, const pred_t* p, mra_t* M, trel_t rel[2]) {
    uint64_t lhs_rel = q->rels[p->frel], lhs_col = p->fcol;
    uint64_t rhs_rel = q->rels[p->srel], rhs_col = p->scol;
    if (lhs_rel == rhs_rel && lhs_col == rhs_col) return DO_NOTHING;

    entity_t* E = M->n == 0 ? mra_new_entity(M) : M->v[M->n - 1];
    ptrdiff_t li = relation_exists_current(E, lhs_rel, p->frel);
    ptrdiff_t ri = relation_exists_current(E, rhs_rel, p->srel);

    if (li != -1 && ri == -1) {
        rel[0] = gather_list(c, E->e[li].list, lhs_rel, lhs_col);
        exists_t ex = relation_exists(M, rhs_rel, p->srel);
        mid_t* T = NULL;
        if (ex.idx == -1) rel[1] = gather_base(c, rhs_rel, rhs_col);
        else { T = &M->v[ex.ent]->e[ex.idx]; rel[1] = gather_list(c, T->list, rhs_rel, rhs_col); }
        mid_t* mid = &E->e[li];
        if (!T) {
            if (mid->lcs == (int32_t)lhs_col) return JOIN_SORT_RHS;
            mid->lcs = (int32_t)lhs_col;
            return CLASSIC_JOIN;
        }
        if (mid->lcs == (int32_t)lhs_col && T->lcs == (int32_t)rhs_col) return SCAN_JOIN;
        if (mid->lcs == (int32_t)lhs_col) return JOIN_SORT_RHS;
        if (T->lcs == (int32_t)rhs_col) return JOIN_SORT_LHS;
        return CLASSIC_JOIN;
    } else if (li != -1 && ri != -1) {
        rel[0] = gather_list(c, E->e[li].list, lhs_rel, lhs_col);
        rel[1] = gather_list(c, E->e[ri].list, rhs_rel, rhs_col);
        return SCAN_JOIN;
    } else if (li == -1 && ri != -1) {
        rel[1] = gather_list(c, E->e[ri].list, rhs_rel, rhs_col);
        exists_t ex = relation_exists(M, lhs_rel, p->frel);
        mid_t* T = NULL;
        if (ex.idx == -1) rel[0] = gather_base(c, lhs_rel, lhs_col);
        else { T = &M->v[ex.ent]->e[ex.idx]; rel[0] = gather_list(c, T->list, lhs_rel, lhs_col); }
        mid_t* mid = &E->e[ri];
        if (!T) {
            if (mid->lcs == (int32_t)rhs_col) return JOIN_SORT_LHS;
            mid->lcs = (int32_t)rhs_col;
            return CLASSIC_JOIN;
        }
        if (mid->lcs == (int32_t)rhs_col && T->lcs == (int32_t)lhs_col) return SCAN_JOIN;
        if (mid->lcs == (int32_t)rhs_col) return JOIN_SORT_RHS;   /* reference quirk, src/join.c:258-259 */
        if (mid->lcs == (int32_t)lhs_col) return JOIN_SORT_LHS;   /* reference quirk, src/join.c:261-262 */
        return CLASSIC_JOIN;
    }
    /* li == -1 && ri == -1: a fresh entity, both sides from the base columns (src/join.c:270-285) */
    mra_new_entity(M);
    rel[1] = gather_base(c, rhs_rel, rhs_col);
    rel[0] = gather_base(c, lhs_rel, lhs_col);
    if (rhs_rel != lhs_rel || p->frel != p->srel) return CLASSIC_JOIN;
    return SCAN_JOIN;
}

/* execute_join (src/join.c:630-679) */
static int execute_join(cpuref_ctx* c, const query_t* q, const pred_t* p, mra_t* M) {
    trel_t rel[2];
    int retval = build_relations(c, q, p, M, rel);
    jres_t jr;
    switch (retval) {
    case CLASSIC_JOIN:  sort_trel(&rel[0]); sort_trel(&rel[1]); jr = join_relations(c, &rel[0], &rel[1]); break;
    case JOIN_SORT_LHS: sort_trel(&rel[0]); jr = join_relations(c, &rel[0], &rel[1]); break;
    case JOIN_SORT_RHS: sort_trel(&rel[1]); jr = join_relations(c, &rel[0], &rel[1]); break;
    case SCAN_JOIN:     jr = scan_join(c, &rel[0], &rel[1]); break;
    case DO_NOTHING:    return 0;
    default:            return -1;
    }
    update_mid_results(c, &jr, M, q->rels[p->frel], p->frel, p->fcol, q->rels[p->srel], p->srel, p->scol, retval);
    return 0;
}

static int filter_pass(char op, uint64_t key, uint64_t number, int* bad) {
    switch (op) {
    case '=': return key == number;
    case '>': return key > number;
    case '<': return key < number;
    default:  *bad = 1; return 0;
    }
}

/* execute_filter (src/filter.c:66-100) with exec_filter_rel_exists (:3-35) and _no_exists (:37-64) */
static int execute_filter(cpuref_ctx* c, const query_t* q, const pred_t* p, mra_t* M) {
    uint64_t relation = q->rels[p->frel];
    const uint64_t* col = c->rels[relation].cols[p->fcol];
    uint64_t rows = c->rels[relation].rows;
    uint64_t number = p->cval;
    entity_t* E = M->n == 0 ? mra_new_entity(M) : M->v[M->n - 1];
    exists_t ex = relation_exists(M, relation, p->frel);
    int bad = 0;
    if (ex.idx != -1) {
        list_t* l = M->v[ex.ent]->e[ex.idx].list;
        uint64_t w = 0;
        for (uint64_t i = 0; i < l->n; i++) {
            int keep = filter_pass(p->op, col[l->v[i]], number, &bad);
            if (bad) { fprintf(stderr, "[ERROR] Wrong operator\n"); return -1; }
            if (keep) l->v[w++] = l->v[i];
        }
        l->n = w;
        fprintf(c->out, "%d\n", (int)(uint32_t)l->n);   /* the stray count line, src/filter.c:32 */
    } else {
        mid_t m = { relation, p->frel, -1, list_new(c, 1024) };
        entity_push(E, m);
        list_t* l = E->e[E->n - 1].list;
        for (uint64_t i = 0; i < rows; i++) {
            int keep = filter_pass(p->op, col[i], number, &bad);
            if (bad) { fprintf(stderr, "[ERROR] Wrong operator\n"); return -1; }
            if (keep) list_push(c, l, (uint32_t)i);
        }
    }
    return 0;
}

/* print_sums (src/utilities.c:197-224) */
static void print_sums(cpuref_ctx* c, const query_t* q, mra_t* M) {
    for (size_t i = 0; i < q->nsel; i++) {
        uint64_t b = q->sel[2 * i], col = q->sel[2 * i + 1];
        uint32_t relation = q->rels[b];
        exists_t ex = relation_exists(M, relation, b);
        if (ex.idx == -1) ref_exit_failure(c, "Something went really wrong...");
        list_t* l = M->v[ex.ent]->e[ex.idx].list;
        if (l->n == 0) {
            fputs("NULL ", c->out);
        } else {
            const uint64_t* v = c->rels[relation].cols[col];
            uint64_t sum = 0;
            for (uint64_t j = 0; j < l->n; j++) sum += v[l->v[j]];
            fprintf(c->out, "%lu ", (unsigned long)sum);
        }
    }
    fputc('\n', c->out);
}

/* ------------------------------------------------------------------------------------ */
/* frontend: parser (src/parsing.c) and arrange_predicates (src/pred_arrange.c)           */
/* ------------------------------------------------------------------------------------ */

static void parse_relations(const char* s, query_t* q) {               /* src/parsing.c:4-28 */
    size_t spaces = 0;
    for (size_t i = 0; s[i]; i++) if (s[i] == ' ') spaces++;
    q->nrels = spaces + 1;
    q->rels = (uint32_t*)calloc(q->nrels, sizeof(uint32_t));
    char cur[16];
    const char* ptr = s;
    int adv;
    size_t i = 0;
    while (i < q->nrels && sscanf(ptr, "%15[^ ]%n", cur, &adv) == 1) {
        ptr += adv;
        q->rels[i++] = (uint32_t)(int)strtol(cur, NULL, 10);
        if (*ptr != ' ') break;
        ptr++;
    }
}

static void parse_predicates(const char* s, query_t* q) {              /* src/parsing.c:30-88 */
    size_t amp = 0;
    for (size_t i = 0; s[i]; i++) if (s[i] == '&') amp++;
    q->npreds = amp + 1;
    q->preds = (pred_t*)calloc(q->npreds, sizeof(pred_t));
    for (size_t i = 0; i < q->npreds; i++) q->preds[i].type = -1;
    char cur[128];
    const char* ptr = s;
    int adv;
    size_t i = 0;
    while (i < q->npreds && sscanf(ptr, "%127[^&]%n", cur, &adv) == 1) {
        ptr += adv;
        int d1, d2, d3, d4;
        unsigned u1, u2, u3;
        char op;
        if (sscanf(cur, "%d.%d%c%d.%d", &d1, &d2, &op, &d3, &d4) == 5) {
            pred_t* p = &q->preds[i++];
            p->type = 0;
            p->frel = (uint32_t)d1; p->fcol = (uint32_t)d2;
            p->srel = (uint32_t)d3; p->scol = (uint32_t)d4;
            p->op = op;
        } else if (sscanf(cur, "%u.%u%c%u", &u1, &u2, &op, &u3) == 4) {
            pred_t* p = &q->preds[i++];
            p->type = 1;
            p->frel = u1; p->fcol = u2;
            p->op = op;
            p->cval = (uint64_t)u3;         /* 4-byte constant read as uint64_t: high word 0 */
            p->srel = (uint64_t)u3; p->scol = 0;   /* what is_match sees through `second` */
        }
        if (*ptr != '&') break;
        ptr++;
    }
}

static void parse_select(const char* s, query_t* q) {                  /* src/parsing.c:90-116 */
    size_t spaces = 0;
    for (size_t i = 0; s[i]; i++) if (s[i] == ' ') spaces++;
    q->nsel = spaces + 1;
    q->sel = (uint64_t*)calloc(2 * q->nsel, sizeof(uint64_t));
    char tmp[128];
    const char* ptr = s;
    int adv;
    size_t i = 0;
    while (i < q->nsel && sscanf(ptr, "%127[^ ]%n", tmp, &adv) == 1) {
        ptr += adv;
        int r = 0, col = 0;
        sscanf(tmp, "%d.%d", &r, &col);
        q->sel[2 * i] = (uint64_t)(int64_t)r;
        q->sel[2 * i + 1] = (uint64_t)(int64_t)col;
        i++;
        if (*ptr != ' ') break;
        ptr++;
    }
}

static void query_free(query_t* q) { free(q->rels); free(q->preds); free(q->sel); }

static void swap_preds(query_t* q, ptrdiff_t i, ptrdiff_t j) {
    if (i == j) return;
    pred_t t = q->preds[i]; q->preds[i] = q->preds[j]; q->preds[j] = t;
}

static int is_match(const pred_t* l, const pred_t* r) {               /* src/pred_arrange.c:29-48 */
    if (l->fcol == r->fcol && l->frel == r->frel) return 1;
    if (l->fcol == r->scol && l->frel == r->srel) return 1;
    if (l->scol == r->fcol && l->srel == r->frel) return 1;
    if (l->scol == r->scol && l->srel == r->srel) return 1;
    return 0;
}

static void arrange_predicates(query_t* q) {                            /* src/pred_arrange.c:50-93 */
    ptrdiff_t n = (ptrdiff_t)q->npreds;
    /* group_filters */
    ptrdiff_t index = 0;
    for (ptrdiff_t i = 1; i < n; i++) {
        if (q->preds[i].type == 1) {
            ptrdiff_t swaps = i;
            for (ptrdiff_t j = 0; j < i - index; j++) { swap_preds(q, swaps, swaps - 1); swaps--; }
            index++;
        }
    }
    /* group_matches: `current` is a pointer to slot i, so a swap into slot i changes it */
    for (ptrdiff_t i = index; i < n - 1;) {
        int swapped = 0;
        for (ptrdiff_t j = i + 1; j < n; j++) {
            if (is_match(&q->preds[i], &q->preds[j])) { swap_preds(q, ++index, j); swapped = 1; }
        }
        if (swapped) i += index - i;
        else i++;
    }
}

/* ------------------------------------------------------------------------------------ */
/* driver                                                                                 */
/* ------------------------------------------------------------------------------------ */

cpuref_ctx* cpuref_create(void) { return (cpuref_ctx*)calloc(1, sizeof(cpuref_ctx)); }

void cpuref_destroy(cpuref_ctx* c) {
    if (!c) return;
    reg_free_all(c);
    free(c->reg);
    free(c->rels);
    free(c);
}

int cpuref_add_relation(cpuref_ctx* c, uint64_t rows, uint64_t ncols, const uint64_t* const* cols) {
    if (c->nrels == c->caprels) {
        c->caprels = c->caprels ? c->caprels * 2 : 16;
        c->rels = (rel_t*)realloc(c->rels, c->caprels * sizeof(rel_t));
    }
    c->rels[c->nrels].rows = rows;
    c->rels[c->nrels].ncols = ncols;
    c->rels[c->nrels].cols = cols;
    c->nrels++;
    return (int)(c->nrels - 1);
}

/* execute_query (src/utilities.c:258-287): a failing predicate silently drops the line */
/* CPUREF_TRACE=1: after every predicate, every list, in oracle/ref_trace_main.c's format */
static void trace_mra(const mra_t* M, size_t step) {
    static int on = -1;
    if (on < 0) on = getenv("CPUREF_TRACE") != NULL;
    if (!on) return;
    for (size_t j = 0; j < M->n; j++)
        for (size_t i = 0; i < M->v[j]->n; i++) {
            const mid_t* m = &M->v[j]->e[i];
            uint64_t n = m->list->n, sum = 0, h = 1469598103934665603ull;
            for (uint64_t k = 0; k < n; k++) {
                sum += m->list->v[k];
                h = (h ^ m->list->v[k]) * 1099511628211ull;
            }
            fprintf(stderr, "step %zu ent %zu idx %zu rel %lu pid %lu lcs %d n %lu sum %lu hash %016lx head", step, j, i,
                    (unsigned long)m->relation, (unsigned long)m->pid, m->lcs, (unsigned long)n,
                    (unsigned long)sum, (unsigned long)h);
            for (uint64_t k = 0; k < n && k < 12; k++) fprintf(stderr, " %lu", (unsigned long)m->list->v[k]);
            fputc('\n', stderr);
        }
}

static int execute_query(cpuref_ctx* c, const query_t* q) {
    mra_t M = { 0 };
    int rc = 0;
    for (size_t i = 0; i < q->npreds; i++) {
        const pred_t* p = &q->preds[i];
        if (p->type < 0) { rc = -1; break; }
        /* out-of-range bindings/relations/columns are undefined in the reference */
        if (p->frel >= q->nrels || q->rels[p->frel] >= c->nrels || p->fcol >= c->rels[q->rels[p->frel]].ncols) { rc = -1; break; }
        if (p->type == 0 && (p->srel >= q->nrels || q->rels[p->srel] >= c->nrels ||
                             p->scol >= c->rels[q->rels[p->srel]].ncols)) { rc = -1; break; }
        int r = p->type == 1 ? execute_filter(c, q, p, &M) : execute_join(c, q, p, &M);
        if (getenv("CPUREF_TRACE")) fprintf(stderr, "query 0 pred %zu type %d rc %d\n", i, p->type, r);
        trace_mra(&M, i);
        if (r == -1) { rc = -1; break; }
    }
    if (rc == 0) {
        for (size_t i = 0; i < q->nsel; i++) {
            uint64_t b = q->sel[2 * i], col = q->sel[2 * i + 1];
            if (b >= q->nrels || q->rels[b] >= c->nrels || col >= c->rels[q->rels[b]].ncols) { rc = -1; break; }
        }
        if (rc == 0) print_sums(c, q, &M);
    }
    mra_free(&M);
    reg_free_all(c);
    return rc;
}

int cpuref_run(cpuref_ctx* c, const char* text, FILE* out) {
    c->out = out;
    /* parser(): every line until EOF, 'F' lines skipped; all parsed before any runs
     * (main/queries_main.c:31-37).  The three scan buffers live across lines as the
     * reference's stack arrays do, so a line that fails to scan re-uses the previous
     * line's text (src/parsing.c:129-132). */
    size_t len = strlen(text);
    char* rbuf = (char*)calloc(len + 2, 1);
    char* pbuf = (char*)calloc(len + 2, 1);
    char* sbuf = (char*)calloc(len + 2, 1);
    size_t nq = 0, capq = 16;
    query_t* volatile qs = (query_t*)malloc(capq * sizeof(query_t));
    const char* s = text;
    char* line = (char*)malloc(len + 2);
    while (*s) {
        const char* e = strchr(s, '\n');
        size_t ll = e ? (size_t)(e - s) + 1 : strlen(s);
        memcpy(line, s, ll);
        line[ll] = 0;
        s += ll;
        if (line[0] == 'F') continue;
        sscanf(line, "%[0-9 ]%*[|]%[0-9.=<>&]%*[|]%[0-9. ]", rbuf, pbuf, sbuf);
        if (nq == capq) { capq *= 2; qs = (query_t*)realloc(qs, capq * sizeof(query_t)); }
        query_t* q = &qs[nq++];
        parse_relations(rbuf, q);
        parse_predicates(pbuf, q);
        parse_select(sbuf, q);
    }
    free(line); free(rbuf); free(pbuf); free(sbuf);

    volatile int rc = 0;
    volatile size_t qi = 0;
    if (setjmp(c->exit_jmp) != 0) {
        /* reference exit(EXIT_FAILURE): stdout so far is flushed, nothing more runs */
        rc = 1;
        reg_free_all(c);
        goto done;
    }
    for (; qi < nq; qi++) {                                               /* execute_queries, src/utilities.c:289-300 */
        arrange_predicates(&qs[qi]);
        int r = execute_query(c, &qs[qi]);
        if (r < -1) { rc = -1; break; }
    }
done:
    for (size_t i = 0; i < nq; i++) query_free(&qs[i]);
    free(qs);
    fflush(out);
    return rc;
}

int cpuref_run_str(cpuref_ctx* c, const char* text, char** out, size_t* outlen) {
    FILE* f = open_memstream(out, outlen);
    int rc = cpuref_run(c, text, f);
    fclose(f);
    return rc;
}
