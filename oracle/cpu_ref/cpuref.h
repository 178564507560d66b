/*
 * cpuref -- CPU restatement of giorgosLiako/Query-Compiler-Executor's query path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the oracle: tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may call it, as the checker or as the timed CPU baseline.
 * The product (libqe, query-compiler-executor_amd/) never links or calls it.
 *
 * It restates, in plain C, the reference's observable semantics:
 *   parser            src/parsing.c:118-148 (+parse_relations/_predicates/_select)
 *   arrange           src/pred_arrange.c:50-93 (index-lag quirk included)
 *   filter            src/filter.c:3-100
 *   join state machine src/join.c:152-292 (build_relations), 486-628 (fix_all/update), 630-679
 *   merge join        src/join.c:325-392 (literal two-pointer loop, exact pair dedup)
 *   scan join         src/join.c:395-423
 *   join_payloads     src/join.c:426-484
 *   checksums         src/utilities.c:197-224
 * with O(n log n) primitives: the randomised quicksort/MSD radix (src/join.c:5-94,
 * src/quicksort.c) is replaced by a stable LSD radix sort (same key order; tie order is
 * unobservable on the rand-invariant domain), the 1000-bucket hashmap by an
 * open-addressing set, and DArray_remove's O(n^2) refinement by an order-preserving compaction.
 *
 * Parity pinned by: the tests/golden/ fixtures, produced by the real reference binary built into
 * oracle/_ref/ (oracle/Makefile) and kept only when stdout is identical under 5 srand seeds.
 */
#ifndef CPUREF_H
#define CPUREF_H

#include <stdint.h>
#include <stddef.h>
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cpuref_ctx cpuref_ctx;

cpuref_ctx* cpuref_create(void);
void        cpuref_destroy(cpuref_ctx*);

/* Register a relation (column-major, cols[c][row]).  Pointers are borrowed, not copied.
 * Relation id = registration order (src/utilities.c:124-162). */
int cpuref_add_relation(cpuref_ctx*, uint64_t rows, uint64_t ncols, const uint64_t* const* cols);

/* Execute every query line of `text` (lines starting with 'F' skipped, src/parsing.c:127)
 * in order, writing the reference's stdout bytes to `out`.
 * Returns 0, or 1 when the reference would have called exit(EXIT_FAILURE) (output up to
 * that point is written), or -1 on an internal error (reference-undefined input). */
int cpuref_run(cpuref_ctx*, const char* text, FILE* out);

/* Same, into a malloc'd string (caller frees). */
int cpuref_run_str(cpuref_ctx*, const char* text, char** out, size_t* outlen);

#ifdef __cplusplus
}
#endif
#endif
