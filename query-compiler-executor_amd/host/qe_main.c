/*
 * qe_main.c -- `queries`: the drop-in for the reference binary (main/queries_main.c:24-68).
 *
 * stdin: relation file paths, one per line, until "Done"/"done" (src/utilities.c:124-162);
 * then query batches until EOF.  stdout: the reference's bytes.  Relations are mmap'd and
 * copied into HBM once; every query runs on the GPU through libqe.  Exit status 1 where the
 * reference calls exit(EXIT_FAILURE).
 *
 *   QE_DEVICE=d   the GPU of a one-GPU run (default 0)
 *   QE_GPUS=N     (N >= 1) N GPUs of this node, one process per GPU (forked before any GPU is touched):
 *                 every rank loads the relations, rank 0 makes the RCCL bootstrap id and hands it
 *                 to the others over pipes, and qe_run_queries_dist runs the batch -- queries in
 *                 the relational domain key-partitioned across the ranks, the others on rank 0's
 *                 faithful executor (include/qe_plan.h).  Rank 0 prints; the exit status is its.
 *   QE_PLAN=0     (one GPU) every query through the faithful executor (the reference's state
 *                 machine restated); default: the partitioned plan, the faithful executor for the
 *                 queries it refuses -- the same bytes (include/qe_plan.h)
 *   QE_WORKERS=k  (one GPU) the batch's queries on k concurrent lanes (1..16, default 8;
 *                 qe_run_queries_lanes)
 *   QE_LOCAL_RANKS=N  (one GPU, N >= 2) the partitioned executor on N in-process ranks of this GPU
 *                 (qe_run_queries_local: the multi-GPU data path with its exchanges, rehearsed)
 *
 * Exit status: 0; 1 where the reference calls exit(EXIT_FAILURE); EXIT_LIBQE (70, sysexits'
 * EX_SOFTWARE) when libqe reports an error (a message on stderr); a rank of QE_GPUS=N killed by
 * signal s: 128 + s, as the shell reports it.
 */
#define _GNU_SOURCE
#include <fcntl.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include "qe.h"

#define EXIT_LIBQE 70   /* libqe returned an error: distinct from a crash (128 + signal) */

typedef struct { char** paths; size_t n; char* text; } input_t;

static input_t read_input(void) {
    input_t in = {NULL, 0, NULL};
    size_t pcap = 0;
    char* line = NULL;
    size_t cap = 0;
    ssize_t got;
    while ((got = getline(&line, &cap, stdin)) != -1) {
        if (!strncmp(line, "Done\n", 5) || !strncmp(line, "done\n", 5)) break;
        line[strlen(line) - 1] = '\0';     /* the last character is the newline (src/utilities.c:135) */
        if (in.n == pcap) {
            pcap = pcap ? 2 * pcap : 16;
            in.paths = (char**)realloc(in.paths, pcap * sizeof(char*));
        }
        in.paths[in.n++] = strdup(line);
    }
    size_t tcap = 1 << 16, tlen = 0;
    in.text = (char*)malloc(tcap);
    while ((got = getline(&line, &cap, stdin)) != -1) {
        while (tlen + (size_t)got + 1 > tcap) {
            tcap *= 2;
            in.text = (char*)realloc(in.text, tcap);
        }
        memcpy(in.text + tlen, line, (size_t)got);
        tlen += (size_t)got;
    }
    in.text[tlen] = 0;
    free(line);
    return in;
}

/* read_relations (src/utilities.c:124-162): each file is `u64 rows, u64 ncols`, then the columns
 * column-major.  The header is checked against the file's size before a column is touched (a
 * truncated file is an error, not a SIGBUS), and the descriptor and mapping are released on every
 * path. */
static int load_relations(qe_ctx* c, const input_t* in) {
    for (size_t i = 0; i < in->n; i++) {
        const char* path = in->paths[i];
        int fd = open(path, O_RDONLY);
        if (fd < 0) {
            fprintf(stderr, "[ERROR] open failed: %s\n", path);
            return -1;
        }
        struct stat sb;
        if (fstat(fd, &sb) < 0 || sb.st_size < 16) {
            fprintf(stderr, "[ERROR] %s: not a relation file (shorter than its 16-byte header)\n", path);
            close(fd);
            return -1;
        }
        const uint64_t* m = (const uint64_t*)mmap(NULL, (size_t)sb.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
        close(fd);                                   /* the mapping stays valid without it */
        if (m == MAP_FAILED) {
            fprintf(stderr, "[ERROR] mmap failed: %s\n", path);
            return -1;
        }
        const uint64_t rows = m[0], ncols = m[1], avail = ((uint64_t)sb.st_size - 16) / 8;
        int rc = 0;
        if ((ncols && rows > avail / ncols) || rows * ncols > avail) {
            fprintf(stderr, "[ERROR] %s: header says %llu rows x %llu columns, the file holds %llu values\n", path,
                    (unsigned long long)rows, (unsigned long long)ncols, (unsigned long long)avail);
            rc = -1;
        } else {
            const uint64_t** cols = (const uint64_t**)malloc((ncols ? ncols : 1) * sizeof(uint64_t*));
            for (uint64_t j = 0; j < ncols; j++) cols[j] = m + 2 + j * rows;
            if (qe_load_relation(c, rows, ncols, cols) < 0) {
                fprintf(stderr, "[ERROR] load %s: %s\n", path, qe_last_error(c));
                rc = -1;
            }
            free(cols);
        }
        munmap((void*)m, (size_t)sb.st_size);
        if (rc) return rc;
    }
    return 0;
}

static int env_int(const char* name, int dflt, int lo, int hi) {
    const char* v = getenv(name);
    int x = v && *v ? atoi(v) : dflt;
    return x < lo ? lo : x > hi ? hi : x;
}

static int finish(int rc, char* out, size_t outlen, int print) {
    if (out) {
        if (print) fwrite(out, 1, outlen, stdout);
        qe_free_host(out);
    }
    fflush(stdout);
    if (rc == QE_EEXIT) return EXIT_FAILURE;
    if (rc != 0) {
        fprintf(stderr, "[ERROR] query execution failed (%d)\n", rc);
        return EXIT_LIBQE;
    }
    return EXIT_SUCCESS;
}

/* one rank of a QE_GPUS=N run (a forked child; nothing touched the GPU before the fork) */
static int run_rank(const input_t* in, int rank, int world, int* to_peers, int from_root) {
    qe_ctx* c = qe_init(rank);
    if (!c) {
        fprintf(stderr, "[ERROR] rank %d: no usable GPU %d\n", rank, rank);
        return EXIT_FAILURE;
    }
    uint8_t id[128];
    if (rank == 0) {
        if (qe_comm_unique_id(id) != 0) return EXIT_FAILURE;
        for (int r = 1; r < world; r++)
            if (write(to_peers[r], id, sizeof id) != (ssize_t)sizeof id) return EXIT_FAILURE;
    } else if (read(from_root, id, sizeof id) != (ssize_t)sizeof id) {
        return EXIT_FAILURE;
    }
    if (load_relations(c, in) != 0) return EXIT_FAILURE;
    /* this rank's hash buckets of the base columns (load-time layout, include/qe.h) */
    if (qe_partition_columns(c, (uint32_t)world, (uint32_t)rank) != 0) {
        fprintf(stderr, "[ERROR] rank %d: %s\n", rank, qe_last_error(c));
        return EXIT_FAILURE;
    }
    qe_comm* m = NULL;
    if (qe_comm_init(c, world, rank, id, &m) != 0) {
        fprintf(stderr, "[ERROR] rank %d: %s\n", rank, qe_last_error(c));
        return EXIT_FAILURE;
    }
    char* out = NULL;
    size_t outlen = 0;
    uint64_t refused = 0;
    int rc = qe_run_queries_dist(c, m, in->text, &out, &outlen, &refused);
    int status = finish(rc, out, outlen, rank == 0);
    qe_comm_fini(m);
    qe_fini(c);
    return status;
}

/* the QE_GPUS launcher's wait: rank 0's status is the process's.  A rank that ends badly while
 * others still run can leave them blocked in RCCL -- whichever rank it is, the rest get 10 s to
 * finish on their own (a reference exit(1) ends every rank alike), then are killed. */
static int exit_code(int st) { return WIFEXITED(st) ? WEXITSTATUS(st) : WIFSIGNALED(st) ? 128 + WTERMSIG(st) : EXIT_LIBQE; }

static int wait_ranks(const pid_t* pid, int world) {
    int status0 = EXIT_LIBQE, left = world, done0 = 0, killed = 0;
    int* done = (int*)calloc((size_t)world, sizeof(int));
    while (left > 0) {
        int st = 0;
        pid_t p = waitpid(-1, &st, 0);
        if (p < 0) break;
        int r = 0;
        while (r < world && pid[r] != p) r++;
        if (r == world) continue;
        done[r] = 1;
        left--;
        const int code = exit_code(st);
        if (r == 0) {
            status0 = code;
            done0 = 1;
        }
        if (code == 0 || left == 0 || killed) continue;
        for (int t = 0; t < 100 && left > 0; t++) {       /* the others: 10 s to end on their own */
            int reaped = 0;
            for (int q = 0; q < world; q++)
                if (!done[q] && waitpid(pid[q], &st, WNOHANG) == pid[q]) {
                    done[q] = 1;
                    left--;
                    reaped = 1;
                    if (q == 0) {
                        status0 = exit_code(st);
                        done0 = 1;
                    }
                }
            if (!reaped) usleep(100000);
        }
        if (left > 0) {
            for (int q = 0; q < world; q++)
                if (!done[q]) kill(pid[q], SIGKILL);
            killed = 1;
            if (!done0) status0 = code;
        }
    }
    free(done);
    return status0;
}

int main(void) {
    input_t in = read_input();
    const char* g = getenv("QE_GPUS");
    const int world = g ? atoi(g) : 0;
    if (world >= 1) {                    /* (QE_GPUS=1: one rank through the same launcher) */
        int fds[64][2];
        if (world > 64) return EXIT_FAILURE;
        for (int r = 1; r < world; r++)
            if (pipe(fds[r]) != 0) return EXIT_FAILURE;
        fflush(stdout);
        pid_t pid[64];
        for (int r = 0; r < world; r++) {
            pid[r] = fork();
            if (pid[r] < 0) {
                for (int q = 0; q < r; q++) kill(pid[q], SIGKILL);
                return EXIT_FAILURE;
            }
            if (pid[r] == 0) {
                /* keep only what this rank uses -- rank 0 every write end, rank r its read end -- so
                 * a rank 0 that dies before it writes the id gives the others EOF, not a hang */
                int to_peers[64];
                for (int q = 1; q < world; q++) {
                    if (r != q) close(fds[q][0]);
                    if (r != 0) close(fds[q][1]);
                    to_peers[q] = r == 0 ? fds[q][1] : -1;
                }
                const int st = run_rank(&in, r, world, to_peers, r ? fds[r][0] : -1);
                _exit(st);
            }
        }
        for (int r = 1; r < world; r++) {    /* the parent keeps no pipe end */
            close(fds[r][0]);
            close(fds[r][1]);
        }
        return wait_ranks(pid, world);
    }
    const char* dev = getenv("QE_DEVICE");
    qe_ctx* c = qe_init(dev ? atoi(dev) : 0);
    if (!c) {
        fprintf(stderr, "[ERROR] no usable GPU (libqe has no CPU path)\n");
        return EXIT_FAILURE;
    }
    if (load_relations(c, &in) != 0) {
        qe_fini(c);
        return EXIT_FAILURE;
    }
    char* out = NULL;
    size_t outlen = 0;
    const int plan = env_int("QE_PLAN", 1, 0, 1);
    const int lranks = env_int("QE_LOCAL_RANKS", 0, 0, 16);
    int rc;
    if (lranks >= 2) {
        uint64_t refused = 0, sent = 0;
        rc = qe_run_queries_local(c, lranks, in.text, &out, &outlen, &refused, &sent);
    } else {
        rc = qe_run_queries_lanes(c, env_int("QE_WORKERS", 8, 1, 16), plan ? QE_EXEC_PLAN : QE_EXEC_FAITHFUL, in.text,
                                  &out, &outlen);
    }
    int status = finish(rc, out, outlen, 1);
    qe_fini(c);
    return status;
}
