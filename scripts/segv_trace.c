/* Debug aid for host faults on the GPU box (no debugger is allowed there): a SIGSEGV / SIGBUS
 * handler that writes the faulting address, the native backtrace and /proc/self/maps to a file, so
 * the frames can be symbolised offline (addr2line / objdump against the same image's libraries).
 * Loaded by scripts/probe_b1.py through ctypes: segv_trace_install("gpurun_out/segv.txt").
 * Build: gcc -O1 -g -shared -fPIC -o scripts/libsegv_trace.so scripts/segv_trace.c */
#define _GNU_SOURCE
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

static char out_path[512];

static void put(int fd, const char* s) { ssize_t r = write(fd, s, strlen(s)); (void)r; }

static void handler(int sig, siginfo_t* si, void* uc) {
    (void)uc;
    int fd = open(out_path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) fd = 2;
    char line[128];
    snprintf(line, sizeof line, "signal %d at address %p\n--- backtrace\n", sig, si->si_addr);
    put(fd, line);
    void* fr[64];
    int n = backtrace(fr, 64);
    backtrace_symbols_fd(fr, n, fd);
    put(fd, "--- maps\n");
    int m = open("/proc/self/maps", O_RDONLY);
    if (m >= 0) {
        char buf[4096];
        ssize_t k;
        while ((k = read(m, buf, sizeof buf)) > 0) { ssize_t r = write(fd, buf, (size_t)k); (void)r; }
        close(m);
    }
    if (fd != 2) close(fd);
    put(2, "[segv_trace] fault recorded\n");
    signal(sig, SIG_DFL);
    raise(sig);
}

int segv_trace_install(const char* path) {
    strncpy(out_path, path, sizeof out_path - 1);
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
    sigemptyset(&sa.sa_mask);
    return sigaction(SIGSEGV, &sa, 0) | sigaction(SIGBUS, &sa, 0);
}
