/*
 * qe_query.c -- parsing.c + pred_arrange.c of the reference, restated (see qe_query.h).
 */
#define _GNU_SOURCE
#include "qe_query.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static void parse_relations(const char* s, query_t* q) {         /* src/parsing.c:4-28 */
    size_t sp = 0;
    for (size_t i = 0; s[i]; i++) sp += s[i] == ' ';
    q->nrels = sp + 1;
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

static void parse_predicates(const char* s, query_t* q) {        /* src/parsing.c:30-88 */
    size_t amp = 0;
    for (size_t i = 0; s[i]; i++) amp += s[i] == '&';
    q->npreds = amp + 1;
    q->preds = (pred_t*)calloc(q->npreds, sizeof(pred_t));
    for (size_t i = 0; i < q->npreds; i++) q->preds[i].type = -1;
    char cur[128];
    const char* ptr = s;
    int adv;
    size_t i = 0;
    while (i < q->npreds && sscanf(ptr, "%127[^&]%n", cur, &adv) == 1) {
        ptr += adv;
        int a, b, c2, d;
        unsigned ua, ub, uc;
        char op;
        if (sscanf(cur, "%d.%d%c%d.%d", &a, &b, &op, &c2, &d) == 5) {
            pred_t* p = &q->preds[i++];
            p->type = 0;
            p->frel = (uint32_t)a;
            p->fcol = (uint32_t)b;
            p->srel = (uint32_t)c2;
            p->scol = (uint32_t)d;
            p->op = op;
        } else if (sscanf(cur, "%u.%u%c%u", &ua, &ub, &op, &uc) == 4) {
            pred_t* p = &q->preds[i++];
            p->type = 1;
            p->frel = ua;
            p->fcol = ub;
            p->op = op;
            p->cval = (uint64_t)uc;
            p->srel = (uint64_t)uc;
            p->scol = 0;
        }
        if (*ptr != '&') break;
        ptr++;
    }
}

static void parse_select(const char* s, query_t* q) {           /* src/parsing.c:90-116 */
    size_t sp = 0;
    for (size_t i = 0; s[i]; i++) sp += s[i] == ' ';
    q->nsel = sp + 1;
    q->sel = (uint64_t*)calloc(2 * q->nsel, sizeof(uint64_t));
    char tmp[128];
    const char* ptr = s;
    int adv;
    size_t i = 0;
    while (i < q->nsel && sscanf(ptr, "%127[^ ]%n", tmp, &adv) == 1) {
        ptr += adv;
        int r = 0, c = 0;
        sscanf(tmp, "%d.%d", &r, &c);
        q->sel[2 * i] = (uint64_t)(int64_t)r;
        q->sel[2 * i + 1] = (uint64_t)(int64_t)c;
        i++;
        if (*ptr != ' ') break;
        ptr++;
    }
}

static void swap_preds(query_t* q, ptrdiff_t i, ptrdiff_t j) {
    if (i == j) return;
    pred_t t = q->preds[i];
    q->preds[i] = q->preds[j];
    q->preds[j] = t;
}

static int is_match(const pred_t* l, const pred_t* r) {         /* src/pred_arrange.c:29-48 */
    return (l->fcol == r->fcol && l->frel == r->frel) || (l->fcol == r->scol && l->frel == r->srel) ||
           (l->scol == r->fcol && l->srel == r->frel) || (l->scol == r->scol && l->srel == r->srel);
}

void qe_arrange_predicates(query_t* q) {                    /* src/pred_arrange.c:50-93 */
    ptrdiff_t n = (ptrdiff_t)q->npreds, index = 0;
    for (ptrdiff_t i = 1; i < n; i++) {                          /* group_filters: p[0] never examined */
        if (q->preds[i].type == 1) {
            ptrdiff_t s = i;
            for (ptrdiff_t j = 0; j < i - index; j++, s--) swap_preds(q, s, s - 1);
            index++;
        }
    }
    for (ptrdiff_t i = index; i < n - 1;) {                      /* group_matches, index lag kept */
        int swapped = 0;
        for (ptrdiff_t j = i + 1; j < n; j++)
            if (is_match(&q->preds[i], &q->preds[j])) {
                swap_preds(q, ++index, j);
                swapped = 1;
            }
        i = swapped ? index : i + 1;
    }
}

query_t* qe_parse_text(const char* text, size_t* nq_out) {
    size_t len = strlen(text);
    char* rb = (char*)calloc(len + 2, 1);
    char* pb = (char*)calloc(len + 2, 1);
    char* sb = (char*)calloc(len + 2, 1);
    char* line = (char*)malloc(len + 2);
    size_t nq = 0, capq = 16;
    query_t* qs = (query_t*)malloc(capq * sizeof(query_t));
    const char* s = text;
    while (*s) {
        const char* e = strchr(s, '\n');
        size_t ll = e ? (size_t)(e - s) + 1 : strlen(s);
        memcpy(line, s, ll);
        line[ll] = 0;
        s += ll;
        if (line[0] == 'F') continue;
        sscanf(line, "%[0-9 ]%*[|]%[0-9.=<>&]%*[|]%[0-9. ]", rb, pb, sb);
        if (nq == capq) {
            capq *= 2;
            qs = (query_t*)realloc(qs, capq * sizeof(query_t));
        }
        parse_relations(rb, &qs[nq]);
        parse_predicates(pb, &qs[nq]);
        parse_select(sb, &qs[nq]);
        nq++;
    }
    free(line);
    free(rb);
    free(pb);
    free(sb);
    *nq_out = nq;
    return qs;
}

qe_where_t qe_mid_exists(const qe_mids* M, uint64_t relation, uint64_t pid) {
    qe_where_t w = {-1, -1};
    for (ptrdiff_t i = (ptrdiff_t)M->count(M->u) - 1; i >= 0; i--) {
        const size_t n = M->size(M->u, (size_t)i);
        for (size_t j = 0; j < n; j++) {
            const qe_mid_t* m = M->at(M->u, (size_t)i, j);
            if (m->relation == relation && m->pid == pid) {
                w.ent = i;
                w.idx = (ptrdiff_t)j;
                return w;
            }
        }
    }
    return w;
}

ptrdiff_t qe_mid_exists_current(const qe_mids* M, size_t ent, uint64_t relation, uint64_t pid) {
    ptrdiff_t f = -1;
    const size_t n = M->size(M->u, ent);
    for (size_t i = 0; i < n; i++) {
        const qe_mid_t* m = M->at(M->u, ent, i);
        if (m->relation == relation && m->pid == pid) f = (ptrdiff_t)i;
    }
    return f;
}

qe_join_choice_t qe_build_relations(const qe_mids* M, const query_t* q, const pred_t* p) {
    qe_join_choice_t j = {0, {-1, -1}, {-1, -1}};
    const uint64_t lhs_rel = q->rels[p->frel], lhs_col = p->fcol;
    const uint64_t rhs_rel = q->rels[p->srel], rhs_col = p->scol;
    if (lhs_rel == rhs_rel && lhs_col == rhs_col) {                 /* src/join.c:159-160 */
        j.variant = QE_DO_NOTHING;
        return j;
    }
    if (M->count(M->u) == 0) M->push_entity(M->u);
    const size_t E = M->count(M->u) - 1;                            /* the current (newest) entity */
    const ptrdiff_t li = qe_mid_exists_current(M, E, lhs_rel, p->frel);
    const ptrdiff_t ri = qe_mid_exists_current(M, E, rhs_rel, p->srel);
    if (li != -1 && ri == -1) {                                     /* src/join.c:171-226 */
        j.lhs.ent = (ptrdiff_t)E;
        j.lhs.idx = li;
        j.rhs = qe_mid_exists(M, rhs_rel, p->srel);
        qe_mid_t* mid = M->at(M->u, E, (size_t)li);
        if (j.rhs.ent == -1) {
            if (mid->lcs == (int32_t)lhs_col) j.variant = QE_JOIN_SORT_RHS;
            else {
                mid->lcs = (int32_t)lhs_col;
                j.variant = QE_CLASSIC_JOIN;
            }
            return j;
        }
        const qe_mid_t* T = M->at(M->u, (size_t)j.rhs.ent, (size_t)j.rhs.idx);
        if (mid->lcs == (int32_t)lhs_col && T->lcs == (int32_t)rhs_col) j.variant = QE_SCAN_JOIN;
        else if (mid->lcs == (int32_t)lhs_col) j.variant = QE_JOIN_SORT_RHS;
        else if (T->lcs == (int32_t)rhs_col) j.variant = QE_JOIN_SORT_LHS;
        else j.variant = QE_CLASSIC_JOIN;
        return j;
    }
    if (li != -1 && ri != -1) {                                     /* src/join.c:227-236 */
        j.lhs.ent = j.rhs.ent = (ptrdiff_t)E;
        j.lhs.idx = li;
        j.rhs.idx = ri;
        j.variant = QE_SCAN_JOIN;
        return j;
    }
    if (li == -1 && ri != -1) {                                     /* src/join.c:237-268 */
        j.rhs.ent = (ptrdiff_t)E;
        j.rhs.idx = ri;
        j.lhs = qe_mid_exists(M, lhs_rel, p->frel);
        qe_mid_t* mid = M->at(M->u, E, (size_t)ri);
        if (j.lhs.ent == -1) {
            if (mid->lcs == (int32_t)rhs_col) j.variant = QE_JOIN_SORT_LHS;
            else {
                mid->lcs = (int32_t)rhs_col;
                j.variant = QE_CLASSIC_JOIN;
            }
            return j;
        }
        const qe_mid_t* T = M->at(M->u, (size_t)j.lhs.ent, (size_t)j.lhs.idx);
        if (mid->lcs == (int32_t)rhs_col && T->lcs == (int32_t)lhs_col) j.variant = QE_SCAN_JOIN;
        else if (mid->lcs == (int32_t)rhs_col) j.variant = QE_JOIN_SORT_RHS;   /* reference quirk, src/join.c:258-259 */
        else if (mid->lcs == (int32_t)lhs_col) j.variant = QE_JOIN_SORT_LHS;   /* reference quirk, src/join.c:261-262 */
        else j.variant = QE_CLASSIC_JOIN;
        return j;
    }
    M->push_entity(M->u);                                           /* src/join.c:270-285 */
    j.variant = (rhs_rel != lhs_rel || p->frel != p->srel) ? QE_CLASSIC_JOIN : QE_SCAN_JOIN;
    return j;
}

void qe_free_queries(query_t* qs, size_t nq) {
    for (size_t i = 0; i < nq; i++) {
        free(qs[i].rels);
        free(qs[i].preds);
        free(qs[i].sel);
    }
    free(qs);
}
