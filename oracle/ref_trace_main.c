/*
 * ref_trace_main.c -- TEST INFRASTRUCTURE ONLY (never part of the product).
 *
 * A driver for the reference's own execute_filter / execute_join (compiled from
 * /root/reference/src by oracle/Makefile, target `ref`) that replays each query like
 * execute_query (src/utilities.c:258-287) but, after every predicate, dumps every mid_result
 * list to stderr: relation, binding, last sorted column, length, sum, an order-sensitive hash
 * and the first rowids.  cpu_ref prints the same lines under CPUREF_TRACE=1, so the first
 * diverging list pins where a restatement departs from the reference.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "DArray.h"
#include "filter.h"
#include "join.h"
#include "parsing.h"
#include "pred_arrange.h"
#include "structs.h"
#include "utilities.h"

static void dump(DArray* mra, size_t step) {
    for (size_t j = 0; j < DArray_count(mra); j++) {
        DArray* ent = *(DArray**)DArray_get(mra, j);
        for (size_t i = 0; i < DArray_count(ent); i++) {
            mid_result* m = (mid_result*)DArray_get(ent, i);
            uint64_t n = DArray_count(m->payloads), sum = 0, h = 1469598103934665603ull;
            for (uint64_t k = 0; k < n; k++) {
                uint64_t v = *(uint64_t*)DArray_get(m->payloads, k);
                sum += v;
                h = (h ^ v) * 1099511628211ull;
            }
            fprintf(stderr, "step %zu ent %zu idx %zu rel %lu pid %lu lcs %d n %lu sum %lu hash %016lx head", step, j, i,
                    (unsigned long)m->relation, (unsigned long)m->predicate_id, m->last_column_sorted,
                    (unsigned long)n, (unsigned long)sum, (unsigned long)h);
            for (uint64_t k = 0; k < n && k < 12; k++)
                fprintf(stderr, " %lu", (unsigned long)*(uint64_t*)DArray_get(m->payloads, k));
            fputc('\n', stderr);
        }
    }
}

int main(void) {
    DArray* metadata_arr = DArray_create(sizeof(metadata), 10);
    if (read_relations(metadata_arr) == -1) return 2;
    DArray* query_list = parser();
    for (size_t qi = 0; qi < DArray_count(query_list); qi++) {
        query* q = (query*)DArray_get(query_list, qi);
        if (!q) continue;
        arrange_predicates(q);
        DArray* mra = DArray_create(sizeof(DArray*), 2);
        for (size_t i = 0; i < (size_t)q->predicates_size; i++) {
            predicate* p = &q->predicates[i];
            int r = p->type == 1 ? execute_filter(p, q->relations, metadata_arr, mra)
                                 : execute_join(p, q->relations, metadata_arr, mra);
            fprintf(stderr, "query %zu pred %zu type %d rc %d\n", qi, i, p->type, r);
            dump(mra, i);
            if (r == -1) break;
        }
    }
    return 0;
}
