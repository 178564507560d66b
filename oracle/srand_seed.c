/*
 * srand_seed.c -- linked into the oracle build of the reference (oracle/_ref/queries_seeded)
 * to run it under a chosen rand() sequence: QE_SRAND=<n> calls srand(n) before main().
 * The reference's only non-determinism is the rand() pivot of its quicksort
 * (src/quicksort.c:7-14); the rand-invariance gate runs each golden query
 * under several seeds and keeps it only when stdout is identical.  TEST INFRASTRUCTURE ONLY.
 */
#include <stdlib.h>

__attribute__((constructor)) static void qe_oracle_seed_rand(void) {
    const char* s = getenv("QE_SRAND");
    if (s && *s) srand((unsigned)strtoul(s, NULL, 10));
}
