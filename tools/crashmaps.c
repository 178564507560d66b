/* crashmaps.c -- diagnostics for a native crash that only shows under a profiler:
 * qecrash_install(path) installs a SIGSEGV / SIGBUS handler that appends the faulting address, the
 * PC and /proc/self/maps to `path` with async-signal-safe calls only, then re-raises the signal
 * under the handler that was installed before (rocprofv3's stack printer, or the default), so the
 * usual report follows.  A PC is then resolved offline: find the mapping that holds it, and
 * llvm-symbolizer --obj=<that library> <PC - mapping start + file offset>.
 * Not product code: benchmarks/c4.py loads it when QE_CRASH_MAPS names a file. */
#define _GNU_SOURCE
#include <fcntl.h>
#include <signal.h>
#include <stdint.h>
#include <string.h>
#include <sys/syscall.h>
#include <ucontext.h>
#include <unistd.h>

static char g_path[512];
static struct sigaction g_old_segv, g_old_bus;

static void put(int fd, const char* s) { (void)!write(fd, s, strlen(s)); }
static void put_hex(int fd, uint64_t v) {
    char b[19] = "0x";
    for (int i = 0; i < 16; i++) b[2 + i] = "0123456789abcdef"[(v >> (60 - 4 * i)) & 15];
    b[18] = 0;
    put(fd, b);
}

static void handler(int sig, siginfo_t* si, void* uc_) {
    const int fd = open(g_path, O_WRONLY | O_CREAT | O_APPEND, 0644);
    if (fd >= 0) {
        ucontext_t* uc = (ucontext_t*)uc_;
        put(fd, sig == SIGSEGV ? "=== SIGSEGV" : "=== SIGBUS");
        put(fd, " addr ");
        put_hex(fd, (uint64_t)(uintptr_t)si->si_addr);
#if defined(__x86_64__)
        put(fd, " pc ");
        put_hex(fd, (uint64_t)uc->uc_mcontext.gregs[REG_RIP]);
        put(fd, " sp ");
        put_hex(fd, (uint64_t)uc->uc_mcontext.gregs[REG_RSP]);
#else
        (void)uc;   /* (the PC / SP registers are x86-64 names; elsewhere the maps alone) */
#endif
        put(fd, " tid ");
        put_hex(fd, (uint64_t)syscall(SYS_gettid));
        put(fd, "\n");
        const int m = open("/proc/self/maps", O_RDONLY);
        if (m >= 0) {
            char buf[4096];
            ssize_t r;
            while ((r = read(m, buf, sizeof buf)) > 0) (void)!write(fd, buf, (size_t)r);
            close(m);
        }
        put(fd, "=== end\n");
        close(fd);
    }
    /* chain: the previous handler's report (or the default action) for the same signal */
    sigaction(sig, sig == SIGSEGV ? &g_old_segv : &g_old_bus, NULL);
    raise(sig);
}

int qecrash_install(const char* path) {
    if (!path || strlen(path) >= sizeof g_path) return -1;
    strcpy(g_path, path);
    /* a signal stack: the faulting thread's may be the problem.  sigaltstack is per thread, so
     * only the installing thread gets it; other threads' faults run the handler on their own
     * stacks (enough for a stack-intact fault such as a bad pointer) */
    static char alt[1 << 16];
    stack_t ss = {.ss_sp = alt, .ss_size = sizeof alt, .ss_flags = 0};
    sigaltstack(&ss, NULL);
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    if (sigaction(SIGSEGV, &sa, &g_old_segv) != 0) return -1;
    if (sigaction(SIGBUS, &sa, &g_old_bus) != 0) return -1;
    return 0;
}
