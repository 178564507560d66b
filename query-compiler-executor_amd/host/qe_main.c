/*
 * qe_main.c -- `queries`: the drop-in for the reference binary (main/queries_main.c:24-68).
 *
 * stdin: relation file paths, one per line, until "Done"/"done" (src/utilities.c:124-162);
 * then query batches until EOF.  stdout: the reference's bytes.  Relations are mmap'd and
 * copied into HBM once; every query runs on the GPU through libqe.  Exit status 1 where the
 * reference calls exit(EXIT_FAILURE).  QE_DEVICE selects the GPU (default 0).
 */
#define _GNU_SOURCE
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "qe.h"

int main(void) {
    const char* dev = getenv("QE_DEVICE");
    qe_ctx* c = qe_init(dev ? atoi(dev) : 0);
    if (!c) {
        fprintf(stderr, "[ERROR] no usable GPU (libqe has no CPU path)\n");
        return EXIT_FAILURE;
    }
    char* line = NULL;
    size_t cap = 0;
    ssize_t got;
    while ((got = getline(&line, &cap, stdin)) != -1) {
        if (!strncmp(line, "Done\n", 5) || !strncmp(line, "done\n", 5)) break;
        line[strlen(line) - 1] = '\0';
        int fd = open(line, O_RDONLY);
        if (fd < 0) {
            fprintf(stderr, "[ERROR] open failed: %s\n", line);
            return EXIT_FAILURE;
        }
        struct stat sb;
        if (fstat(fd, &sb) < 0) return EXIT_FAILURE;
        const uint64_t* m = (const uint64_t*)mmap(NULL, sb.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) return EXIT_FAILURE;
        uint64_t rows = m[0], ncols = m[1];
        const uint64_t** cols = (const uint64_t**)malloc((ncols ? ncols : 1) * sizeof(uint64_t*));
        for (uint64_t j = 0; j < ncols; j++) cols[j] = m + 2 + j * rows;
        if (qe_load_relation(c, rows, ncols, cols) < 0) {
            fprintf(stderr, "[ERROR] load: %s\n", qe_last_error(c));
            return EXIT_FAILURE;
        }
        free(cols);
        munmap((void*)m, sb.st_size);
        close(fd);
    }
    size_t tcap = 1 << 16, tlen = 0;
    char* text = (char*)malloc(tcap);
    while ((got = getline(&line, &cap, stdin)) != -1) {
        while (tlen + (size_t)got + 1 > tcap) {
            tcap *= 2;
            text = (char*)realloc(text, tcap);
        }
        memcpy(text + tlen, line, (size_t)got);
        tlen += (size_t)got;
    }
    text[tlen] = 0;
    free(line);
    char* out = NULL;
    size_t outlen = 0;
    int rc = qe_run_queries(c, text, &out, &outlen);
    if (out) {
        fwrite(out, 1, outlen, stdout);
        qe_free_host(out);
    }
    fflush(stdout);
    free(text);
    qe_fini(c);
    if (rc == QE_EEXIT) return EXIT_FAILURE;
    if (rc != 0) {
        fprintf(stderr, "[ERROR] query execution failed (%d)\n", rc);
        return 139;
    }
    return EXIT_SUCCESS;
}
