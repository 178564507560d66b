/*
 * qe_plan.c -- the key-partitioned plan of include/qe_plan.h: (1) the domain check, a replay of
 * the reference's mid_result state machine on bindings alone, and (2) the relational plan itself
 * over an engine (filters on rank slices, hash exchange of derived join sides, local sort-merge
 * joins, all-reduced checksums).  Host C; the engine does every row-sized step.
 *
 * Reference anchors: execute_query src/utilities.c:258-287, execute_filter src/filter.c:66-100,
 * build_relations src/join.c:152-292, update_mid_results src/join.c:507-628, fix_all_mid_results
 * src/join.c:486-505, join_payloads src/join.c:426-484, print_sums src/utilities.c:197-224.
 */
#define _GNU_SOURCE
#include "../../include/qe_plan.h"

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/qe.h"
#include "qe_query.h"

static __thread char g_why[256];

const char* qe_plan_why(void) { return g_why; }

/* ============================================================================================ */
/* (1) the domain check                                                                          */
/* ============================================================================================ */

/* A symbolic rowid list.  ok: its multiset is the projection on its binding of the relation its
 * component denotes (the relational answer); tag: lists with one tag are positionally aligned
 * (rows of one tuple sequence); len: lists with one len id have equal lengths; distinct: no rowid
 * twice; sorted: the binding column it is ascending on (-1: none). */
typedef struct { int tag, len, ok, distinct, sorted; } slist;
typedef struct { qe_mid_t h; int l; } smid;   /* mid_result, list by index */
typedef struct { smid* e; size_t n; } sent;

typedef struct {
    const query_t* q;
    slist* L; size_t nl, capl;
    sent* E; size_t ne, cape;
    size_t cap_entries;
    int fresh;
    int* parent;                /* union-find over bindings: the components joined so far */
    const uint8_t* live;        /* binding read by a later predicate or a select */
} replay_t;

static int refuse(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_why, sizeof g_why, fmt, ap);
    va_end(ap);
    return QE_ENOTSUP;
}

static int new_slist(replay_t* r, int tag, int len, int ok, int distinct, int sorted) {
    if (r->nl == r->capl) {
        r->capl = r->capl ? 2 * r->capl : 32;
        r->L = (slist*)realloc(r->L, r->capl * sizeof(slist));
    }
    slist s = {tag, len, ok, distinct, sorted};
    r->L[r->nl] = s;
    return (int)r->nl++;
}

static sent* s_new_entity(replay_t* r) {
    if (r->ne == r->cape) {
        r->cape = r->cape ? 2 * r->cape : 8;
        r->E = (sent*)realloc(r->E, r->cape * sizeof(sent));
    }
    sent* E = &r->E[r->ne++];
    E->e = (smid*)calloc(r->cap_entries, sizeof(smid));
    E->n = 0;
    return E;
}

static void s_push(replay_t* r, sent* E, smid m) {
    (void)r;
    E->e[E->n++] = m;     /* an entry is pushed only for a (relation, pid) with none anywhere */
}

typedef qe_where_t sexists_t;

/* the replay's entities as the shared view (host/qe_query.h) */
static size_t v_count(void* u) { return ((replay_t*)u)->ne; }
static size_t v_size(void* u, size_t ent) { return ((replay_t*)u)->E[ent].n; }
static qe_mid_t* v_at(void* u, size_t ent, size_t idx) { return &((replay_t*)u)->E[ent].e[idx].h; }
static void v_push_entity(void* u) { (void)s_new_entity((replay_t*)u); }

static qe_mids view(replay_t* r) {
    qe_mids v = {r, v_count, v_size, v_at, v_push_entity};
    return v;
}

static sexists_t s_exists(replay_t* r, uint64_t relation, uint64_t pid) {   /* relation_exists */
    const qe_mids v = view(r);
    return qe_mid_exists(&v, relation, pid);
}

static int uf_find(int* p, int x) {
    while (p[x] != x) x = p[x] = p[p[x]];
    return x;
}

/* the join's inputs as build_relations picks them: list index or -1 (the whole base relation) */
typedef struct { int variant; int lR, lS; } sjoin_t;

/* build_relations (src/join.c:152-292) on symbolic entries: the shared variant choice
 * (host/qe_query.c, the faithful executor's too), its side effects on the entries included */
static sjoin_t s_build_relations(replay_t* r, const pred_t* p) {
    const qe_mids v = view(r);
    const qe_join_choice_t c = qe_build_relations(&v, r->q, p);
    sjoin_t j = {c.variant, -1, -1};
    if (c.lhs.ent >= 0) j.lR = r->E[c.lhs.ent].e[c.lhs.idx].l;
    if (c.rhs.ent >= 0) j.lS = r->E[c.rhs.ent].e[c.rhs.idx].l;
    return j;
}

typedef struct { int* w; size_t n, cap; } wset;   /* lists written by the current join */

static void w_add(wset* w, int l) {
    if (w->n == w->cap) {
        w->cap = w->cap ? 2 * w->cap : 16;
        w->w = (int*)realloc(w->w, w->cap * sizeof(int));
    }
    w->w[w->n++] = l;
}

static int w_has(const wset* w, int l) {
    for (size_t i = 0; i < w->n; i++)
        if (w->w[i] == l) return 1;
    return 0;
}

/* fix_all_mid_results (src/join.c:486-505): every other entry of the entity gets
 * join_payloads(driver = the join's distinct pairs on this side, last = the updated entry's list,
 * edit = the entry's list) -- a positional zip of edit with last, each row repeated by the number
 * of DISTINCT partner rowids.  That is the relational projection only when edit is aligned with
 * last, both are relational, and the other side's rowids are distinct (so distinct pairs = matches). */
static int s_fix_all(replay_t* r, sexists_t ex, uint64_t relR, uint64_t relS, smid tmp, int other_distinct,
                     int join_len, wset* w) {
    sent* E = &r->E[ex.ent];
    const slist upd = r->L[E->e[ex.idx].l];
    const int tag = ++r->fresh;
    const int len = other_distinct ? join_len : ++r->fresh;
    for (size_t i = 0; i < E->n; i++) {
        if ((ptrdiff_t)i == ex.idx) continue;
        smid* ed = &E->e[i];
        if (ed->h.relation == relR || ed->h.relation == relS) continue;   /* left stale (post pass) */
        const slist edl = r->L[ed->l];
        if (edl.len != upd.len)
            return refuse("join_payloads on lists of possibly different lengths (binding %llu)",
                          (unsigned long long)ed->h.pid);
        const int ok = edl.tag == upd.tag && edl.ok && upd.ok && other_distinct;
        if (r->live[ed->h.pid] && !ok)
            return refuse("binding %llu is read later but join_payloads makes it %s", (unsigned long long)ed->h.pid,
                          edl.tag != upd.tag ? "a zip of misaligned lists" : "a non-relational multiset");
        ed->l = new_slist(r, tag, len, ok, 0, -1);
        w_add(w, ed->l);
    }
    E->e[ex.idx] = tmp;
    w_add(w, tmp.l);
    return 0;
}

static int s_join(replay_t* r, const pred_t* p) {
    const query_t* q = r->q;
    sjoin_t j = s_build_relations(r, p);
    if (j.variant == 5) return refuse("join of a column with itself (reference DO_NOTHING)");
    if (j.variant == 4) return refuse("positional scan_join");
    const int a = (int)p->frel, b = (int)p->srel;
    if (uf_find(r->parent, a) == uf_find(r->parent, b))
        return refuse("join inside one component (bindings %d and %d are already joined)", a, b);
    /* a whole base relation stands for its binding only while that binding has no list yet: the
     * last branch of build_relations gathers both sides from the base relations even when a
     * binding already has a (filtered or joined) list in an older entity */
    if (j.lR < 0 && s_exists(r, q->rels[p->frel], p->frel).idx != -1)
        return refuse("join reads the whole relation of binding %d, which already has a list", a);
    if (j.lS < 0 && s_exists(r, q->rels[p->srel], p->srel).idx != -1)
        return refuse("join reads the whole relation of binding %d, which already has a list", b);
    if (j.lR >= 0 && !r->L[j.lR].ok) return refuse("join input of binding %d is not relational", a);
    if (j.lS >= 0 && !r->L[j.lS].ok) return refuse("join input of binding %d is not relational", b);
    if (j.variant == 2 && (j.lS < 0 || r->L[j.lS].sorted != (int)p->scol))
        return refuse("merge on a list taken as sorted that is not (binding %d)", b);
    if (j.variant == 3 && (j.lR < 0 || r->L[j.lR].sorted != (int)p->fcol))
        return refuse("merge on a list taken as sorted that is not (binding %d)", a);
    const int dR = j.lR < 0 ? 1 : r->L[j.lR].distinct;
    const int dS = j.lS < 0 ? 1 : r->L[j.lS].distinct;
    const int tag = ++r->fresh, len = ++r->fresh;
    const uint64_t relR = q->rels[p->frel], relS = q->rels[p->srel];
    smid tR = {{relR, p->frel, (int32_t)p->fcol}, new_slist(r, tag, len, 1, 0, (int)p->fcol)};
    smid tS = {{relS, p->srel, (int32_t)p->scol}, new_slist(r, tag, len, 1, 0, (int)p->scol)};
    wset w = {NULL, 0, 0};
    int rc = 0;
    sexists_t ex;
    /* update_mid_results (src/join.c:507-628) */
    switch (j.variant) {
    case 1:
        ex = s_exists(r, relR, p->frel);
        if (ex.idx == -1) { s_push(r, &r->E[r->ne - 1], tR); w_add(&w, tR.l); }
        else rc = s_fix_all(r, ex, relR, relS, tR, dS, len, &w);
        if (rc) break;
        ex = s_exists(r, relS, p->srel);
        if (ex.idx == -1) { s_push(r, &r->E[r->ne - 1], tS); w_add(&w, tS.l); }
        else rc = s_fix_all(r, ex, relR, relS, tS, dR, len, &w);
        break;
    case 2:
        ex = s_exists(r, relR, p->frel);
        if (ex.idx == -1) s_push(r, &r->E[r->ne - 1], tR);
        else r->E[ex.ent].e[ex.idx] = tR;
        w_add(&w, tR.l);
        ex = s_exists(r, relS, p->srel);
        if (ex.idx == -1) { rc = refuse("the reference exits here (update of a missing entry)"); break; }
        rc = s_fix_all(r, ex, relR, relS, tS, dR, len, &w);
        break;
    case 3:
        ex = s_exists(r, relS, p->srel);
        if (ex.idx == -1) s_push(r, &r->E[r->ne - 1], tS);
        else r->E[ex.ent].e[ex.idx] = tS;
        w_add(&w, tS.l);
        ex = s_exists(r, relR, p->frel);
        if (ex.idx == -1) { rc = refuse("the reference exits here (update of a missing entry)"); break; }
        rc = s_fix_all(r, ex, relR, relS, tR, dS, len, &w);
        break;
    }
    if (rc == 0) {
        /* the components merge; every entry of either that this join did not rewrite is stale */
        const int ca = uf_find(r->parent, a), cb = uf_find(r->parent, b);
        for (size_t e = 0; e < r->ne; e++)
            for (size_t i = 0; i < r->E[e].n; i++) {
                smid* m = &r->E[e].e[i];
                const int c = uf_find(r->parent, (int)m->h.pid);
                if ((c == ca || c == cb) && !w_has(&w, m->l)) {
                    r->L[m->l].ok = 0;
                    r->L[m->l].len = ++r->fresh;
                }
            }
        r->parent[ca] = cb;
    }
    free(w.w);
    return rc;
}

static int op_valid(char op) { return op == '=' || op == '<' || op == '>'; }

static int s_query_valid(const qe_engine* e, const query_t* q) {
    uint32_t nrel = 0;
    if (e->rel_count(e->u, &nrel) != 0) return 0;
    uint64_t rows;
    uint32_t nc;
    for (size_t i = 0; i < q->nrels; i++)
        if (q->rels[i] >= nrel) return 0;
#define COL_OK(b, c) ((b) < q->nrels && e->rel_shape(e->u, q->rels[(b)], &rows, &nc) == 0 && (c) < nc)
    for (size_t i = 0; i < q->npreds; i++) {
        const pred_t* p = &q->preds[i];
        if (p->type < 0 || !COL_OK(p->frel, p->fcol)) return 0;
        if (p->type == 0 && !COL_OK(p->srel, p->scol)) return 0;
    }
    for (size_t i = 0; i < q->nsel; i++)
        if (!COL_OK(q->sel[2 * i], q->sel[2 * i + 1])) return 0;
#undef COL_OK
    return 1;
}

/* 0: the query's output is the relational answer the plan computes; QE_ENOTSUP otherwise */
static int plan_check(const qe_engine* e, const query_t* q) {
    g_why[0] = 0;
    if (!s_query_valid(e, q)) return refuse("out-of-range relation / column / binding (the reference is undefined)");
    if (q->nsel == 0) return refuse("no select");
    replay_t r;
    memset(&r, 0, sizeof r);
    r.q = q;
    r.cap_entries = q->nrels + 1;
    r.parent = (int*)malloc((q->nrels + 1) * sizeof(int));
    for (size_t i = 0; i <= q->nrels; i++) r.parent[i] = (int)i;
    uint8_t* live = (uint8_t*)calloc(q->nrels + 1, 1);
    r.live = live;
    int rc = 0, seen_join = 0;
    for (size_t i = 0; rc == 0 && i < q->npreds; i++) {
        memset(live, 0, q->nrels + 1);
        for (size_t k = i + 1; k < q->npreds; k++) {
            live[q->preds[k].frel] = 1;
            if (q->preds[k].type == 0) live[q->preds[k].srel] = 1;
        }
        for (size_t s = 0; s < q->nsel; s++) live[q->sel[2 * s]] = 1;
        const pred_t* p = &q->preds[i];
        if (p->type == 1) {                              /* execute_filter (src/filter.c:66-100) */
            if (!op_valid(p->op)) { rc = refuse("filter operator '%c'", p->op); break; }
            if (seen_join) { rc = refuse("filter after a join"); break; }
            sexists_t ex = s_exists(&r, q->rels[p->frel], p->frel);
            if (ex.idx != -1) {
                slist* l = &r.L[r.E[ex.ent].e[ex.idx].l];
                l->tag = ++r.fresh;
                l->len = ++r.fresh;
            } else {
                sent* E = r.ne == 0 ? s_new_entity(&r) : &r.E[r.ne - 1];
                const int tag = ++r.fresh, len = ++r.fresh;
                smid m = {{q->rels[p->frel], p->frel, -1}, new_slist(&r, tag, len, 1, 1, -1)};
                s_push(&r, E, m);
            }
        } else {
            seen_join = 1;
            rc = s_join(&r, p);
        }
    }
    for (size_t s = 0; rc == 0 && s < q->nsel; s++) {   /* print_sums (src/utilities.c:197-224) */
        const uint64_t b = q->sel[2 * s];
        sexists_t ex = s_exists(&r, q->rels[b], b);
        if (ex.idx == -1) rc = refuse("select of binding %llu without a list (the reference exits)", (unsigned long long)b);
        else if (!r.L[r.E[ex.ent].e[ex.idx].l].ok)
            rc = refuse("select of binding %llu whose list is not relational", (unsigned long long)b);
    }
    for (size_t i = 0; i < r.ne; i++) free(r.E[i].e);
    free(r.E);
    free(r.L);
    free(r.parent);
    free(live);
    return rc;
}

/* ============================================================================================ */
/* (2) the relational plan                                                                      */
/* ============================================================================================ */

#define NONE ((qe_h)0)

/* whole: every row of the relation; vcol = c + 1: rows holds column c's values; kvals (kcol = c + 1):
 * column c's values at the binding's rows -- its next join's key, delivered by the join that made
 * the component (join_carry's outxa), consumed or dropped by the component's next join */
typedef struct { int b; qe_h rows; int whole; int vcol; qe_h kvals; int kcol; } member;
typedef struct { member* m; int n; uint64_t size; int alive; } comp_t;

typedef struct {
    const qe_engine* e;
    const query_t* q;
    comp_t* C; int nc;
    int* comp_of;               /* binding -> component, -1 none */
    qe_h* list;                 /* filtered, not yet joined bindings */
    uint64_t* list_size;
    int rc;
    /* the last join ran in aggregate form (engine join_sums): its global pair count and the
     * selects' local sums, in select order */
    int agg;
    uint64_t agg_size;
    uint64_t agg_sums[64];
    /* the plan's switches, read once per query (QE_PLAN_BCAST: 0 never broadcast, 2 always, 1 the
     * cost model; QE_DIST_REORDER=0: joins in query order), and whether the ranks were checked to
     * agree on them -- the first all-reduce of a query carries them (plan_allreduce) */
    int bcast_mode, reorder, agreed;
} plan_t;

#define ECHK(call)                                   \
    do {                                             \
        int rc_ = (call);                            \
        if (rc_ != 0) { P->rc = rc_; return rc_; }   \
    } while (0)

static void owned_range(const plan_t* P, uint64_t rows, uint64_t* s, uint64_t* t) {
    const uint64_t W = P->e->world, r = P->e->rank;
    *s = rows * r / W;
    *t = rows * (r + 1) / W;
}

static uint64_t rel_rows(const plan_t* P, uint32_t rel) {
    uint64_t rows = 0;
    uint32_t nc = 0;
    P->e->rel_shape(P->e->u, rel, &rows, &nc);
    return rows;
}

/* a join's global pair count beyond the materialisation limit (the reference's DArray bound) */
static int over_limit(const plan_t* P, uint64_t pairs) { return P->e->mat_limit && pairs > *P->e->mat_limit; }

/* all-reduce v[0, nv) (nv <= 2; the engine's u64 sum).  The query's first one also carries every
 * rank's switches (mode and its square, so W * sum(x^2) == sum(x)^2 holds exactly when all ranks
 * agree): a rank whose environment differs would take a broadcast join where its peers exchange,
 * or join in another order, and the collectives would no longer pair up -- every rank fails the
 * query together instead.  It runs before the first collective a switch can change: filters'
 * counts come first, and do_join calls it (nv = 0) before its first side is started. */
static int plan_allreduce(plan_t* P, uint64_t* v, int nv) {
    const qe_engine* e = P->e;
    if (e->world == 1) return 0;
    if (P->agreed) return nv ? e->allreduce(e->u, v, nv) : 0;
    uint64_t w[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < nv; i++) w[i] = v[i];
    w[nv] = (uint64_t)P->bcast_mode;
    w[nv + 1] = (uint64_t)(P->bcast_mode * P->bcast_mode);
    w[nv + 2] = (uint64_t)P->reorder;
    w[nv + 3] = (uint64_t)(P->reorder * P->reorder);
    const int rc = e->allreduce(e->u, w, nv + 4);
    if (rc) return rc;
    P->agreed = 1;
    for (int i = 0; i < nv; i++) v[i] = w[i];
    const uint64_t W = e->world;
    if (W * w[nv + 1] != w[nv] * w[nv] || W * w[nv + 3] != w[nv + 2] * w[nv + 2]) {
        fprintf(stderr, "[qe_plan] rank %u: QE_PLAN_BCAST / QE_DIST_REORDER differ across ranks\n", e->rank);
        return QE_EINVAL;
    }
    return 0;
}

static int allreduce1(plan_t* P, uint64_t* v) { return plan_allreduce(P, v, 1); }

static void rel(plan_t* P, qe_h h) {
    if (h != NONE) P->e->release(P->e->u, h);
}

static int component(plan_t* P, int b) {
    if (P->comp_of[b] >= 0) return P->comp_of[b];
    comp_t* c = &P->C[P->nc];
    c->m = (member*)calloc(P->q->nrels + 1, sizeof(member));
    c->n = 1;
    c->alive = 1;
    c->m[0].b = b;
    if (P->list[b] != NONE) {
        c->m[0].rows = P->list[b];
        c->size = P->list_size[b];
        P->list[b] = NONE;
    } else {
        c->m[0].whole = 1;
        c->size = rel_rows(P, P->q->rels[b]);
    }
    P->comp_of[b] = P->nc;
    return P->nc++;
}

static int rows_of(plan_t* P, member* m) {
    if (m->whole) {
        uint64_t s, t;
        owned_range(P, rel_rows(P, P->q->rels[m->b]), &s, &t);
        ECHK(P->e->iota(P->e->u, s, t - s, &m->rows));
        m->whole = 0;
    }
    return 0;
}

static int member_idx(const comp_t* c, int b) {
    for (int i = 0; i < c->n; i++)
        if (c->m[i].b == b) return i;
    return -1;
}

/* one join side: keys + (vals | positions) and the bindings carried through the join */
typedef struct {
    qe_h keys, vals;            /* vals: rowids aligned with keys, or NONE (row = position / base row i) */
    int ncar;
    int car_b[64];
    qe_h car_rows[64];          /* NONE: the binding's rowids are `vals` */
    int car_v[64];              /* the member's vcol (values instead of rowids) */
    qe_h ticket;                /* an exchange in flight */
    int keep_n;
    int keep_b[64];
    int keep_v[64];
    int base;                   /* keys is a whole base column (vals NONE = row i) */
    qe_h pay;                   /* base side: the column of its binding's next join key (join_carry's xa) */
    int pay_col;                /* that column + 1 */
} side_t;

static int is_whole(const comp_t* c) { return c->n == 1 && c->m[0].whole; }

/* local: a broadcast join (bcast_join below) -- a whole base side is the whole column, a derived
 * side stays where it lies (no exchange), as at one rank */
static int side_start(plan_t* P, int cid, int b, uint32_t col, const uint8_t* need, const int* sel1, const int* kcol1,
                      const int* vok, side_t* s, int local) {
    const qe_engine* e = P->e;
    comp_t* c = &P->C[cid];
    memset(s, 0, sizeof *s);
    if (is_whole(c) && c->m[0].b == b) {                     /* a whole base relation: never exchanged */
        if (local) ECHK(e->base_side_all(e->u, P->q->rels[b], col, &s->keys, &s->vals));
        else ECHK(e->base_side(e->u, P->q->rels[b], col, &s->keys, &s->vals));
        s->base = 1;
        if (need[b]) {
            s->ncar = 1;
            s->car_b[0] = b;
            s->car_rows[0] = NONE;
            if (kcol1[b] && e->column && e->keys_of && e->join_carry) {
                /* its next join's key column rides with its rows: no gather through them later */
                const int r = e->column(e->u, P->q->rels[b], (uint32_t)(kcol1[b] - 1), &s->pay);
                if (r == 0) s->pay_col = kcol1[b];
                else if (r != QE_ENOTSUP) {
                    P->rc = r;
                    return r;
                }
            }
            if (s->pay && vok[b] && s->vals == NONE) {
                /* read later only by selects of one column (after the next join, which takes its
                 * key from the payload): the rows ride as that column's values (join_carry packs
                 * them in place of the row index) -- no gather through them at the end */
                qe_h v = NONE;
                const int r = e->column(e->u, P->q->rels[b], (uint32_t)(vok[b] - 1), &v);
                if (r == 0) {
                    s->vals = v;
                    s->car_v[0] = vok[b];
                } else if (r != QE_ENOTSUP) {
                    P->rc = r;
                    return r;
                }
            }
        }
        return 0;
    }
    member* mb = &c->m[member_idx(c, b)];
    ECHK(rows_of(P, mb));
    if (mb->kvals != NONE && mb->kcol == (int)col + 1) {     /* the key's values came with the rows */
        ECHK(e->keys_of(e->u, P->q->rels[b], col, mb->kvals, &s->keys));
    } else {
        ECHK(e->keys(e->u, P->q->rels[b], col, mb->rows, &s->keys));
    }
    for (int i = 0; i < c->n; i++) {                         /* kvals live one join: consumed or dropped */
        rel(P, c->m[i].kvals);
        c->m[i].kvals = NONE;
        c->m[i].kcol = 0;
    }
    if (e->values && sel1[b] && c->n == 1 && mb->vcol == 0) {
        /* a filtered list (ascending rowids) read after this join only by selects of one column:
         * its values ride instead of its rowids (gathered here in order, not at random later) */
        qe_h v = NONE;
        const int r = e->values(e->u, P->q->rels[b], (uint32_t)(sel1[b] - 1), mb->rows, &v);
        if (r == 0) {
            rel(P, mb->rows);
            mb->rows = v;
            mb->vcol = sel1[b];
        } else if (r != QE_ENOTSUP) {
            P->rc = r;
            return r;
        }
    }
    qe_h cols[64];
    int nk = 0;
    for (size_t x = 0; x <= P->q->nrels; x++) {               /* carried: the bindings read later */
        int mi = member_idx(c, (int)x);
        if (mi < 0 || !need[x]) continue;
        ECHK(rows_of(P, &c->m[mi]));
        s->keep_b[nk] = (int)x;
        s->keep_v[nk] = c->m[mi].vcol;
        cols[nk++] = c->m[mi].rows;
    }
    s->keep_n = nk;
    if (e->world > 1 && !local) {
        /* the carried lists travel with the keys (consumed); the others are dropped */
        for (int i = 0; i < c->n; i++) {
            int kept = 0;
            for (int k = 0; k < nk; k++) kept |= c->m[i].b == s->keep_b[k];
            if (!kept) rel(P, c->m[i].rows);
            c->m[i].rows = NONE;
        }
        ECHK(e->exchange_start(e->u, s->keys, cols, nk, &s->ticket));
        s->keys = NONE;
        return 0;
    }
    for (int k = 0; k < nk; k++) {
        s->car_b[k] = s->keep_b[k];
        s->car_v[k] = s->keep_v[k];
        s->car_rows[k] = cols[k];
    }
    s->ncar = nk;
    if (nk == 1) {                                           /* the only carried list rides as vals */
        s->vals = cols[0];
        s->car_rows[0] = NONE;
    }
    for (int i = 0; i < c->n; i++) {                         /* ownership moves to the side */
        int kept = 0;
        for (int k = 0; k < nk; k++) kept |= c->m[i].b == s->keep_b[k];
        if (!kept) rel(P, c->m[i].rows);
        c->m[i].rows = NONE;
    }
    return 0;
}

static int side_finish(plan_t* P, side_t* s) {
    if (!s->ticket) return 0;
    qe_h cols[64];
    ECHK(P->e->exchange_finish(P->e->u, s->ticket, &s->keys, cols));
    s->ticket = NONE;
    s->ncar = s->keep_n;
    for (int k = 0; k < s->keep_n; k++) {
        s->car_b[k] = s->keep_b[k];
        s->car_v[k] = s->keep_v[k];
        s->car_rows[k] = cols[k];
    }
    if (s->keep_n == 1) {
        s->vals = cols[0];
        s->car_rows[0] = NONE;
    }
    return 0;
}

static void free_comp(plan_t* P, int cid) {
    comp_t* c = &P->C[cid];
    for (int i = 0; i < c->n; i++) {
        rel(P, c->m[i].rows);
        rel(P, c->m[i].kvals);
    }
    free(c->m);
    c->m = NULL;
    c->n = 0;
    c->alive = 0;
}

/* Broadcast or partitioned, for a join of a derived side D with a whole base relation of R rows at
 * G > 1 ranks (DESIGN §5's per-rank budget).  Per rank:
 *   partitioned: D/G rows hash-partitioned (COST_PART_PS a row), 1/G of them to each peer over its
 *     own xGMI link (D * B / (G^2 * COST_LINK_GBS), B = a u32 key + 4 B per carried column), one
 *     counts all-to-all + host round trip (COST_EXCHANGE_PS); the base side is the rank's hash
 *     bucket (R/G rows, selected once per column and kept: free from the second query on);
 *   broadcast: D stays where it lies and is joined with the WHOLE column: (1 - 1/G) * R rows more
 *     through the base side's sort and the bucket join than the partitioned form's R/G.
 * Broadcast iff (1 - 1/G) * R * (COST_BASE_SORT_PS + COST_JOIN_PS) < the partitioned form's extra.
 * The per-row costs are this code's, measured on one MI355X (profiles/r06b_launches.txt: one C3
 * query's kernels -- the 1e8-row carried base side's histogram + scans + two passes 0.97 ms, the
 * chain bucket join 0.48 ms for 1e8 + 4.66e7 rows; profiles/r06e_cost_constants.json: partition_dev
 * of a 4.66e7-row side with 8-B keys and two columns); the link figure is the MI355X_MICROARCH.md
 * per-link rate, projected (no box here has two GPUs).  C3 then: broadcast at G = 2, partitioned
 * from G = 4.  QE_PLAN_BCAST: 0 never, 2 always (tests), otherwise this model.  Every rank decides
 * on the same global sizes (and the same switches: plan_allreduce). */
#define COST_BASE_SORT_PS 9.7
#define COST_JOIN_PS 3.3
#define COST_PART_PS 9.0
#define COST_LINK_GBS 153.0
#define COST_EXCHANGE_PS 5.0e7
static int bcast_join(const plan_t* P, int A, int B) {
    const qe_engine* e = P->e;
    if (e->world <= 1 || !e->base_side_all) return 0;
    const int wa = is_whole(&P->C[A]), wb = is_whole(&P->C[B]);
    if (wa == wb) return 0;                                  /* both derived, or both whole: no */
    const int mode = P->bcast_mode;            /* (read once per query, agreed across ranks) */
    if (mode != 1) return mode == 2;
    const double G = (double)e->world;
    const comp_t* Dc = wa ? &P->C[B] : &P->C[A];
    const double R = (double)(wa ? P->C[A].size : P->C[B].size), D = (double)Dc->size;
    const double bytes = 4.0 + 4.0 * (double)(Dc->n < 3 ? Dc->n : 3);   /* u32 key + carried columns */
    const double bcast_ps = (1.0 - 1.0 / G) * R * (COST_BASE_SORT_PS + COST_JOIN_PS);
    const double part_ps = D / G * COST_PART_PS + D * bytes / (G * G) / (COST_LINK_GBS * 1e9) * 1e12 + COST_EXCHANGE_PS;
    return bcast_ps < part_ps;
}

static int do_join(plan_t* P, const pred_t* p, const uint8_t* need, const int* sel1, const int* kcol1, const int* vok,
                   int last) {
    const qe_engine* e = P->e;
    const int ba = (int)p->frel, bb = (int)p->srel;
    const int A = component(P, ba), B = component(P, bb);
    if (last && e->join_agg && is_whole(&P->C[A]) && is_whole(&P->C[B]) && P->q->nsel <= 64) {
        /* the last join of two whole base relations, every select on one of them: aggregate form */
        const query_t* q = P->q;
        int side[64], ok = 1;
        uint32_t cols[64];
        for (size_t s = 0; ok && s < q->nsel; s++) {
            const int b = (int)q->sel[2 * s];
            side[s] = b == ba ? 0 : 1;
            cols[s] = (uint32_t)q->sel[2 * s + 1];
            ok = b == ba || b == bb;
        }
        if (ok) {
            uint64_t pairs = 0;
            const int jr = e->join_agg(e->u, q->rels[ba], (uint32_t)p->fcol, q->rels[bb], (uint32_t)p->scol,
                                       (int)q->nsel, side, cols, &pairs, P->agg_sums);
            if (jr == 0) {
                ECHK(allreduce1(P, &pairs));
                free_comp(P, A);
                free_comp(P, B);
                P->agg = 1;
                P->agg_size = pairs;
                return 0;
            }
            if (jr != QE_ENOTSUP) {
                P->rc = jr;
                return jr;
            }
        }
    }
    side_t sa, sb;
    ECHK(plan_allreduce(P, NULL, 0));                        /* (the switches agreed, once per query) */
    const int bc = bcast_join(P, A, B);
    /* derived sides first, so their exchanges overlap the base side's local bucket scan */
    if (is_whole(&P->C[A])) {
        ECHK(side_start(P, B, bb, (uint32_t)p->scol, need, sel1, kcol1, vok, &sb, bc));
        ECHK(side_start(P, A, ba, (uint32_t)p->fcol, need, sel1, kcol1, vok, &sa, bc));
    } else {
        ECHK(side_start(P, A, ba, (uint32_t)p->fcol, need, sel1, kcol1, vok, &sa, bc));
        ECHK(side_start(P, B, bb, (uint32_t)p->scol, need, sel1, kcol1, vok, &sb, bc));
    }
    if (sa.pay && sb.pay) {                                  /* one payload column per join */
        rel(P, sb.pay);
        sb.pay = NONE;
        sb.pay_col = 0;
        if (sb.car_v[0]) {                                   /* (its values mode goes with it) */
            rel(P, sb.vals);
            sb.vals = NONE;
            sb.car_v[0] = 0;
        }
    }
    ECHK(side_finish(P, &sa));
    ECHK(side_finish(P, &sb));
    if (last && e->join_sums) {
        /* the query's last join, read only by the selects: one side carries every selected
         * binding, the other none -- the engine returns the pair count and the sums */
        side_t* O = sa.ncar == 0 ? &sa : sb.ncar == 0 ? &sb : NULL;
        side_t* C = O == &sa ? &sb : &sa;
        const query_t* q = P->q;
        int src[64], ok = O && C->ncar >= 1 && C->ncar <= 3 && q->nsel >= 1 && q->nsel <= 4;
        for (size_t s = 0; ok && s < q->nsel; s++) {
            src[s] = -1;
            for (int i = 0; i < C->ncar; i++)
                if (C->car_b[i] == (int)q->sel[2 * s]) src[s] = i | (C->car_v[i] ? QE_PLAN_VALUES_SRC : 0);
            ok = src[s] >= 0;
        }
        if (ok) {
            uint32_t srel[64], scol[64];
            for (size_t s = 0; s < q->nsel; s++) {
                srel[s] = q->rels[q->sel[2 * s]];
                scol[s] = (uint32_t)q->sel[2 * s + 1];
            }
            if (C->ncar >= 2) {                                  /* its first binding rides as vals */
                C->vals = C->car_rows[0];
                C->car_rows[0] = NONE;
            }
            uint64_t v[2] = {0, 0};
            const int jr = e->join_sums(e->u, O->keys, O->vals, C->keys, C->vals, C->ncar - 1, &C->car_rows[1],
                                        (int)q->nsel, src, srel, scol, &v[0], P->agg_sums);
            if (jr != 0 && jr != QE_ETOOBIG) {
                P->rc = jr;
                return jr;
            }
            v[1] = jr == QE_ETOOBIG;
            ECHK(plan_allreduce(P, v, 2));                  /* every rank takes one branch */
            if (over_limit(P, v[0])) v[1] = 1;
            rel(P, sa.keys);
            rel(P, sb.keys);
            rel(P, sa.vals);
            rel(P, sb.vals);
            rel(P, sa.pay);
            rel(P, sb.pay);
            for (int k = 0; k < sa.ncar; k++) rel(P, sa.car_rows[k]);
            for (int k = 0; k < sb.ncar; k++) rel(P, sb.car_rows[k]);
            free_comp(P, A);
            free_comp(P, B);
            if (v[1]) {
                P->rc = QE_ETOOBIG;
                return QE_ETOOBIG;
            }
            P->agg = 1;
            P->agg_size = v[0];
            return 0;
        }
    }
    qe_h oa = NONE, ob = NONE;
    /* a side carrying several bindings: its first rides as the join's vals, the others (up to two)
     * ride through the engine's join beside the pairs (join_carry) instead of being taken after;
     * a base side's payload column (its binding's next join key) rides on the other side of it */
    qe_h made[2][64];
    for (int k = 0; k < 2; k++)
        for (int i = 0; i < 64; i++) made[k][i] = NONE;
    int cs = -1;
    if (e->join_carry) {
        if (sa.pay) cs = 1;
        else if (sb.pay) cs = 0;
        else if (sb.ncar >= 2 && sb.ncar <= 3 && sb.vals == NONE) cs = 1;
        else if (sa.ncar >= 2 && sa.ncar <= 3 && sa.vals == NONE) cs = 0;
    }
    int jr;
    qe_h oxa = NONE;                                        /* the payload side's next join key values */
    if (cs >= 0) {
        side_t* C = cs ? &sb : &sa;
        side_t* O = cs ? &sa : &sb;
        int nb = 0;
        if (C->ncar >= 2) {
            C->vals = C->car_rows[0];
            C->car_rows[0] = NONE;                          /* now rides as vals */
            nb = C->ncar - 1;
        }
        qe_h oo = NONE, oc = NONE, ox[64];
        for (int i = 0; i < 64; i++) ox[i] = NONE;
        jr = e->join_carry(e->u, O->keys, O->vals, C->keys, C->vals, nb, &C->car_rows[1], O->pay, &oo, &oc, ox, &oxa);
        for (int i = 1; i < C->ncar && i <= nb && jr == 0; i++) made[cs][i] = ox[i - 1];
        if (cs) {
            oa = oo;
            ob = oc;
        } else {
            oa = oc;
            ob = oo;
        }
    } else {
        jr = e->join(e->u, sa.keys, sa.vals, sb.keys, sb.vals, &oa, &ob);
    }
    if (jr != 0 && jr != QE_ETOOBIG) {
        P->rc = jr;
        return jr;
    }
    {   /* every rank learns whether any rank's bucket was too large to materialise, so all of them
         * leave the query together (the fallback then runs it) -- one all-reduce with the size */
        uint64_t v[2] = {0, jr == QE_ETOOBIG};
        if (jr == 0) ECHK(e->length(e->u, oa, &v[0]));
        ECHK(plan_allreduce(P, v, 2));
        if (over_limit(P, v[0])) v[1] = 1;
        if (v[1]) {
            rel(P, oa);
            rel(P, ob);
            rel(P, oxa);
            rel(P, sa.pay);
            rel(P, sb.pay);
            for (int k = 0; k < 2; k++)
                for (int i = 0; i < 64; i++) rel(P, made[k][i]);
            rel(P, sa.keys);
            rel(P, sb.keys);
            rel(P, sa.vals);
            rel(P, sb.vals);
            for (int k = 0; k < sa.ncar; k++) rel(P, sa.car_rows[k]);
            for (int k = 0; k < sb.ncar; k++) rel(P, sb.car_rows[k]);
            P->rc = QE_ETOOBIG;
            return QE_ETOOBIG;
        }
        P->C[A].size = v[0];    /* the join's global pair count, taken below */
    }
    /* the merged component: carried bindings, rowids = o (vals rode along) or take(rows, o) */
    member* m = (member*)calloc(P->q->nrels + 1, sizeof(member));
    int n = 0;
    side_t* sides[2] = {&sa, &sb};
    qe_h outs[2] = {oa, ob};
    int used[2] = {0, 0};
    for (int k = 0; k < 2; k++) {
        side_t* s = sides[k];
        for (int i = 0; i < s->ncar; i++) {
            m[n].b = s->car_b[i];
            m[n].vcol = s->car_v[i];
            if (s->pay && oxa != NONE) {                    /* (a base side carries its one binding) */
                m[n].kvals = oxa;
                m[n].kcol = s->pay_col;
                oxa = NONE;
            }
            if (made[k][i] != NONE) {                        /* delivered by join_carry */
                m[n].rows = made[k][i];
                rel(P, s->car_rows[i]);
            } else if (s->car_rows[i] == NONE) {
                m[n].rows = outs[k];
                used[k] = 1;
            } else {
                ECHK(e->take(e->u, s->car_rows[i], outs[k], &m[n].rows));
                rel(P, s->car_rows[i]);
            }
            n++;
        }
    }
    if (n == 0) {                                           /* nothing read later: keep the count */
        m[0].b = ba;
        m[0].rows = oa;
        used[0] = 1;
        n = 1;
    }
    rel(P, sa.keys);                     /* (a borrowed base column: the engine's release is a no-op) */
    rel(P, sb.keys);
    rel(P, sa.vals);
    rel(P, sb.vals);
    rel(P, sa.pay);
    rel(P, sb.pay);
    rel(P, oxa);                         /* (not taken by a member) */
    if (!used[0]) rel(P, oa);
    if (!used[1]) rel(P, ob);
    const uint64_t size = P->C[A].size;
    /* A absorbs B */
    free_comp(P, A);
    free_comp(P, B);
    for (size_t x = 0; x <= P->q->nrels; x++)
        if (P->comp_of[x] == A || P->comp_of[x] == B) P->comp_of[x] = A;
    P->C[A].m = m;
    P->C[A].n = n;
    P->C[A].size = size;
    P->C[A].alive = 1;
    return 0;
}

static uint64_t join_cost(plan_t* P, const pred_t* p) {
    uint64_t c = 0;
    const int bs[2] = {(int)p->frel, (int)p->srel};
    for (int k = 0; k < 2; k++) {
        const int b = bs[k];
        if (P->comp_of[b] >= 0) c += P->C[P->comp_of[b]].size;
        else if (P->list[b] != NONE) c += P->list_size[b];
        else c += rel_rows(P, P->q->rels[b]);
    }
    return c;
}

/* binding b will carry column col's values instead of its rowids (the `values` request of
 * side_start): it is joined once and every select of it reads col */
static int values_hint(const query_t* q, int b, uint64_t col) {
    int joins = 0, sels = 0;
    for (size_t i = 0; i < q->npreds; i++)
        if (q->preds[i].type == 0) joins += ((int)q->preds[i].frel == b) + ((int)q->preds[i].srel == b);
    for (size_t s = 0; s < q->nsel; s++) {
        if ((int)q->sel[2 * s] != b) continue;
        if (q->sel[2 * s + 1] != col) return 0;
        sels++;
    }
    return joins == 1 && sels > 0;
}

/* 1 + the column every join of binding b keys on (0: b joins on several columns, or not at all):
 * a fused scan of b may emit those values with its rowids (scan2's `values` bits 8..15), and b's
 * key side then takes them instead of gathering them through the list */
static int join_key_hint(const query_t* q, int b) {
    int kc = 0;
    for (size_t i = 0; i < q->npreds; i++) {
        const pred_t* p = &q->preds[i];
        if (p->type != 0) continue;
        for (int side = 0; side < 2; side++) {
            const int rb = (int)(side ? p->srel : p->frel);
            const int c = (int)(side ? p->scol : p->fcol) + 1;
            if (rb != b) continue;
            if (kc && kc != c) return 0;
            kc = c;
        }
    }
    return kc < 256 ? kc : 0;
}

static int plan_query(const qe_engine* e, const query_t* q, FILE* out, uint64_t* rows_out) {
    plan_t PP;
    plan_t* P = &PP;
    memset(P, 0, sizeof *P);
    P->e = e;
    P->q = q;
    const size_t nb = q->nrels + 1;
    P->C = (comp_t*)calloc(nb + q->npreds + 1, sizeof(comp_t));
    P->comp_of = (int*)malloc(nb * sizeof(int));
    P->list = (qe_h*)calloc(nb, sizeof(qe_h));
    P->list_size = (uint64_t*)calloc(nb, sizeof(uint64_t));
    for (size_t i = 0; i < nb; i++) P->comp_of[i] = -1;
    const char* bm = getenv("QE_PLAN_BCAST");
    P->bcast_mode = bm && (bm[0] == '0' || bm[0] == '2') ? bm[0] - '0' : 1;
    P->reorder = !(getenv("QE_DIST_REORDER") && getenv("QE_DIST_REORDER")[0] == '0');
    const int reorder = P->reorder;
    uint8_t* need = (uint8_t*)calloc(nb, 1);
    int* sel1 = (int*)calloc(nb, sizeof(int));
    int* kcol1 = (int*)calloc(nb, sizeof(int));
    int* vok = (int*)calloc(nb, sizeof(int));
    int* pending = (int*)malloc((q->npreds + 1) * sizeof(int));
    size_t k = 0;
    int rc = 0;
    while (rc == 0 && k < q->npreds) {
        const pred_t* p = &q->preds[k];
        if (p->type == 1) {                                  /* filters (they all precede the joins) */
            const int b = (int)p->frel;
            const uint32_t relid = q->rels[b];
            if (P->list[b] != NONE) {
                qe_h nl = NONE;
                rc = e->refine(e->u, relid, (uint32_t)p->fcol, P->list[b], p->op, p->cval, &nl);
                P->list[b] = nl;
                uint64_t n = 0;
                if (!rc) rc = e->length(e->u, nl, &n);
                if (!rc) rc = allreduce1(P, &n);
                P->list_size[b] = n;
                if (!rc) fprintf(out, "%d\n", (int)(uint32_t)n);        /* src/filter.c:32 */
            } else if (e->scan2 && k + 1 < q->npreds && q->preds[k + 1].type == 1 && (int)q->preds[k + 1].frel == b) {
                /* the scan and the refine after it, in one pass (only the refine prints a count) */
                const pred_t* p2 = &q->preds[k + 1];
                uint64_t s, t;
                owned_range(P, rel_rows(P, relid), &s, &t);
                const int vh = values_hint(q, b, p->fcol) && e->values != NULL;
                rc = e->scan2(e->u, relid, (uint32_t)p->fcol, p->op, p->cval, (uint32_t)p2->fcol, p2->op, p2->cval, s,
                              t, vh | join_key_hint(q, b) << 8, &P->list[b]);
                uint64_t n = 0;
                if (!rc) rc = e->length(e->u, P->list[b], &n);
                if (!rc) rc = allreduce1(P, &n);
                P->list_size[b] = n;
                if (!rc) fprintf(out, "%d\n", (int)(uint32_t)n);        /* src/filter.c:32 */
                k++;
            } else {
                uint64_t s, t;
                owned_range(P, rel_rows(P, relid), &s, &t);
                rc = e->scan(e->u, relid, (uint32_t)p->fcol, s, t, p->op, p->cval, &P->list[b]);
                uint64_t n = 0;
                if (!rc) rc = e->length(e->u, P->list[b], &n);
                if (!rc) rc = allreduce1(P, &n);
                P->list_size[b] = n;
            }
            k++;
            continue;
        }
        size_t end = k;                                      /* the run of joins */
        while (end < q->npreds && q->preds[end].type == 0) end++;
        size_t np = 0;
        for (size_t i = k; i < end; i++) pending[np++] = (int)i;
        while (rc == 0 && np) {
            size_t jbest = 0;
            if (reorder) {                                   /* greedy: the smallest |A| + |B| first */
                uint64_t best = UINT64_MAX;
                for (size_t i = 0; i < np; i++) {
                    uint64_t c = join_cost(P, &q->preds[pending[i]]);
                    if (c < best) { best = c; jbest = i; }
                }
            }
            const pred_t* jp = &q->preds[pending[jbest]];
            for (size_t i = jbest; i + 1 < np; i++) pending[i] = pending[i + 1];
            np--;
            /* bindings read later: the remaining joins, later predicates, the selects */
            memset(need, 0, nb);
            for (size_t s = 0; s < q->nsel; s++) need[q->sel[2 * s]] = 1;
            for (size_t i = 0; i < np; i++) {
                need[q->preds[pending[i]].frel] = 1;
                need[q->preds[pending[i]].srel] = 1;
            }
            for (size_t i = end; i < q->npreds; i++) {
                need[q->preds[i].frel] = 1;
                if (q->preds[i].type == 0) need[q->preds[i].srel] = 1;
            }
            /* sel1[b] = c + 1: after this join, binding b is read only by selects, all of column c */
            for (size_t x = 0; x < nb; x++) sel1[x] = 0;
            for (size_t s = 0; s < q->nsel; s++) {
                const size_t x = q->sel[2 * s];
                const int cv = (int)q->sel[2 * s + 1] + 1;
                sel1[x] = sel1[x] == 0 ? cv : sel1[x] == cv ? cv : -1;
            }
            for (size_t i = 0; i < np; i++) {
                sel1[q->preds[pending[i]].frel] = -1;
                sel1[q->preds[pending[i]].srel] = -1;
            }
            for (size_t i = end; i < q->npreds; i++) {
                sel1[q->preds[i].frel] = -1;
                if (q->preds[i].type == 0) sel1[q->preds[i].srel] = -1;
            }
            for (size_t x = 0; x < nb; x++)
                if (sel1[x] < 0) sel1[x] = 0;
            /* kcol1[b] = c + 1: binding b joins again after this join, always on its column c */
            for (size_t x = 0; x < nb; x++) kcol1[x] = 0;
            for (size_t i = 0; i < np + (q->npreds - end); i++) {
                const pred_t* r = i < np ? &q->preds[pending[i]] : &q->preds[end + (i - np)];
                if (r->type != 0) continue;
                const size_t xs[2] = {r->frel, r->srel};
                const int cs2[2] = {(int)r->fcol + 1, (int)r->scol + 1};
                for (int t = 0; t < 2; t++)
                    kcol1[xs[t]] = kcol1[xs[t]] == 0 ? cs2[t] : kcol1[xs[t]] == cs2[t] ? cs2[t] : -1;
            }
            for (size_t x = 0; x < nb; x++)
                if (kcol1[x] < 0) kcol1[x] = 0;
            /* vok[b] = c + 1 (b one of this join's bindings): every select of b reads column c, no
             * later filter reads b, and the one remaining join touching the merged component is
             * b's, on kcol1[b] -- so b's next join takes its key from the payload and nothing
             * after it needs b's rowids: b may ride as column c's values */
            for (size_t x = 0; x < nb; x++) vok[x] = 0;
            {
                const int ca = P->comp_of[jp->frel], cb2 = P->comp_of[jp->srel];
                uint8_t* inm = (uint8_t*)calloc(nb, 1);
                for (size_t x = 0; x < nb; x++)
                    inm[x] = x == jp->frel || x == jp->srel || (P->comp_of[x] >= 0 && (P->comp_of[x] == ca || P->comp_of[x] == cb2));
                int touching = 0;
                const pred_t* only = NULL;
                for (size_t i = 0; i < np + (q->npreds - end); i++) {
                    const pred_t* r = i < np ? &q->preds[pending[i]] : &q->preds[end + (i - np)];
                    if (r->type != 0) continue;
                    if (inm[r->frel] || inm[r->srel]) {
                        touching++;
                        only = r;
                    }
                }
                const size_t ends[2] = {jp->frel, jp->srel};
                for (int t = 0; t < 2 && touching == 1; t++) {
                    const size_t x = ends[t];
                    const int on_x = (only->frel == x && (int)only->fcol + 1 == kcol1[x] && !inm[only->srel]) ||
                                     (only->srel == x && (int)only->scol + 1 == kcol1[x] && !inm[only->frel]);
                    if (!on_x || !kcol1[x]) continue;
                    int c1 = 0;
                    for (size_t s = 0; s < q->nsel; s++)
                        if (q->sel[2 * s] == x) c1 = c1 == 0 || c1 == (int)q->sel[2 * s + 1] + 1 ? (int)q->sel[2 * s + 1] + 1 : -1;
                    for (size_t i = end; i < q->npreds; i++)
                        if (q->preds[i].type == 1 && q->preds[i].frel == x) c1 = -1;
                    vok[x] = c1 > 0 ? c1 : 0;
                }
                free(inm);
            }
            rc = do_join(P, jp, need, sel1, kcol1, vok, np == 0 && end == q->npreds);
        }
        k = end;
    }
    /* print_sums: every select's sum at once, one all-reduce */
    uint64_t* sums = (uint64_t*)calloc(q->nsel + 1, sizeof(uint64_t));
    uint32_t* srel = (uint32_t*)calloc(q->nsel + 1, sizeof(uint32_t));
    uint32_t* scol = (uint32_t*)calloc(q->nsel + 1, sizeof(uint32_t));
    qe_h* srows = (qe_h*)calloc(q->nsel + 1, sizeof(qe_h));
    uint64_t* ssize = (uint64_t*)calloc(q->nsel + 1, sizeof(uint64_t));
    int ns = 0;
    for (size_t s = 0; rc == 0 && P->agg && s < q->nsel; s++) {   /* the aggregate last join's sums */
        ssize[s] = P->agg_size;
        if (P->agg_size) sums[ns++] = P->agg_sums[s];
    }
    for (size_t s = 0; rc == 0 && !P->agg && s < q->nsel; s++) {
        const int b = (int)q->sel[2 * s];
        uint64_t size;
        qe_h rows;
        int vcol = 0;
        if (P->comp_of[b] >= 0) {
            comp_t* c = &P->C[P->comp_of[b]];
            member* m = &c->m[member_idx(c, b)];
            rc = rows_of(P, m);
            rows = m->rows;
            vcol = m->vcol;
            size = c->size;
        } else {
            rows = P->list[b];
            size = P->list_size[b];
        }
        ssize[s] = size;
        if (size == 0 || rc) continue;
        srel[ns] = vcol ? QE_PLAN_VALUES : q->rels[b];
        scol[ns] = (uint32_t)q->sel[2 * s + 1];
        srows[ns++] = rows;
    }
    if (rc == 0 && ns && !P->agg) rc = e->checksums(e->u, ns, srel, scol, srows, sums);
    if (rc == 0 && ns && e->world > 1) rc = e->allreduce(e->u, sums, ns);
    if (rc == 0) {
        int j = 0;
        for (size_t s = 0; s < q->nsel; s++) {
            if (ssize[s] == 0) fputs("NULL ", out);
            else fprintf(out, "%lu ", (unsigned long)sums[j++]);
        }
        fputc('\n', out);
        if (rows_out) *rows_out = ssize[0];
    }
    free(sums);
    free(srel);
    free(scol);
    free(srows);
    free(ssize);
    for (int i = 0; i < P->nc; i++)
        if (P->C[i].alive) free_comp(P, i);
    for (size_t b = 0; b < nb; b++) rel(P, P->list[b]);
    free(P->C);
    free(P->comp_of);
    free(P->list);
    free(P->list_size);
    free(need);
    free(sel1);
    free(kcol1);
    free(vok);
    free(pending);
    return rc ? rc : P->rc;
}

/* ============================================================================================ */
/* text drivers                                                                                   */
/* ============================================================================================ */

int qe_plan_check_text(const qe_engine* e, const char* text, uint8_t* accepted, size_t cap) {
    size_t nq = 0;
    query_t* qs = qe_parse_text(text, &nq);
    char first[256] = "";
    for (size_t i = 0; i < nq; i++) {
        qe_arrange_predicates(&qs[i]);
        int ok = plan_check(e, &qs[i]) == 0;
        if (!ok && !first[0]) snprintf(first, sizeof first, "%s", g_why);
        if (accepted && i < cap) accepted[i] = (uint8_t)ok;
    }
    snprintf(g_why, sizeof g_why, "%s", first);
    qe_free_queries(qs, nq);
    return (int)nq;
}

int qe_plan_run_query(const qe_engine* e, void* query, void* out, uint64_t* rows, int* refused) {
    query_t* q = (query_t*)query;
    FILE* f = (FILE*)out;
    *refused = 0;
    if (plan_check(e, q) != 0) {
        *refused = 1;
        return e->fallback ? e->fallback(e->u, q, f) : QE_ENOTSUP;
    }
    /* the query's bytes are buffered: a join too large to materialise (QE_ETOOBIG, the
     * reference's DArray bound) sends the whole query to the fallback, whose executor takes
     * the aggregate form where the reference's output allows it */
    char* qbuf = NULL;
    size_t qlen = 0;
    FILE* qf = open_memstream(&qbuf, &qlen);
    if (!qf) return QE_ENOMEM;
    uint64_t r = 0;
    int rc = plan_query(e, q, qf, &r);
    fclose(qf);
    if (rc == QE_ETOOBIG && e->fallback) {
        *refused = 1;
        rc = e->fallback(e->u, q, f);
    } else {
        if (qlen) fwrite(qbuf, 1, qlen, f);
        if (rc == 0 && rows) *rows = r;
    }
    free(qbuf);
    return rc;
}

int qe_plan_run_text(const qe_engine* e, const char* text, char** out, size_t* outlen, uint64_t* rows,
                     uint64_t* nrefused) {
    *out = NULL;
    *outlen = 0;
    FILE* f = open_memstream(out, outlen);
    if (!f) return QE_ENOMEM;
    size_t nq = 0;
    query_t* qs = qe_parse_text(text, &nq);     /* parsed before anything runs (main/queries_main.c:31-37) */
    int rc = 0;
    uint64_t refused = 0;
    char first[256] = "";
    for (size_t i = 0; rc == 0 && i < nq; i++) {
        qe_arrange_predicates(&qs[i]);
        int ref = 0;
        rc = qe_plan_run_query(e, &qs[i], f, rows, &ref);
        if (ref && !first[0]) snprintf(first, sizeof first, "%s", g_why);
        refused += (uint64_t)ref;
    }
    snprintf(g_why, sizeof g_why, "%s", first);
    qe_free_queries(qs, nq);
    fclose(f);
    if (nrefused) *nrefused = refused;
    return rc;
}
