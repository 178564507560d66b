/*
 * cpuref_main.c -- the reference's stdin protocol (main/queries_main.c:24-68,
 * src/utilities.c:124-162) over the cpuref restatement.  TEST INFRASTRUCTURE ONLY.
 *
 * stdin: relation file paths, one per line, until "Done"/"done"; then query lines until
 * EOF.  stdout: the reference's bytes.  Exit status 1 where the reference exits 1.
 */
#define _GNU_SOURCE
#include "cpuref.h"

#include <fcntl.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

int main(void) {
    cpuref_ctx* c = cpuref_create();
    char* line = NULL;
    size_t cap = 0;
    ssize_t got;
    while ((got = getline(&line, &cap, stdin)) != -1) {
        if (!strncmp(line, "Done\n", 5) || !strncmp(line, "done\n", 5)) break;
        line[strlen(line) - 1] = '\0';   /* the last character is dropped, src/utilities.c:135 */
        int fd = open(line, O_RDONLY);
        if (fd < 0) { fprintf(stderr, "[ERROR] open failed: %s\n", line); return EXIT_FAILURE; }
        struct stat sb;
        if (fstat(fd, &sb) < 0) { fprintf(stderr, "[ERROR] fstat failed\n"); return EXIT_FAILURE; }
        const uint64_t* m = (const uint64_t*)mmap(NULL, sb.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) { fprintf(stderr, "[ERROR] mmap failed\n"); return EXIT_FAILURE; }
        uint64_t rows = m[0], ncols = m[1];
        const uint64_t** cols = (const uint64_t**)malloc((ncols ? ncols : 1) * sizeof(uint64_t*));
        for (uint64_t j = 0; j < ncols; j++) cols[j] = m + 2 + j * rows;   /* column-major, src/utilities.c:107-120 */
        cpuref_add_relation(c, rows, ncols, cols);
        close(fd);
    }
    /* the rest of stdin is the query batch text */
    size_t tcap = 1 << 16, tlen = 0;
    char* text = (char*)malloc(tcap);
    while ((got = getline(&line, &cap, stdin)) != -1) {
        while (tlen + (size_t)got + 1 > tcap) { tcap *= 2; text = (char*)realloc(text, tcap); }
        memcpy(text + tlen, line, (size_t)got);
        tlen += (size_t)got;
    }
    text[tlen] = 0;
    free(line);
    int rc = cpuref_run(c, text, stdout);
    fflush(stdout);
    free(text);
    return rc == 1 ? EXIT_FAILURE : EXIT_SUCCESS;
}
