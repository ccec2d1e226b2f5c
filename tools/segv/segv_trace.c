/* Debug aid (tools/run_dbg.sh): a SIGSEGV handler that prints the native backtrace and the
 * mappings of the library objects, then re-raises; installed from Python via ctypes. */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>
#include <fcntl.h>

static void on_segv(int sig, siginfo_t *si, void *uc) {
    (void)uc;
    char msg[128];
    int n = snprintf(msg, sizeof msg, "\n[segv_trace] signal %d at address %p\n", sig, si ? si->si_addr : 0);
    write(2, msg, n);
    write(2, "[segv_trace] backtrace:\n", 24);
    void *bt[64];
    int k = backtrace(bt, 64);
    backtrace_symbols_fd(bt, k, 2);
    int fd = open("/proc/self/maps", O_RDONLY);
    if (fd >= 0) {
        char buf[4096];
        ssize_t r;
        write(2, "[segv_trace] maps (ygzfe):\n", 27);
        /* crude filter: print lines mentioning libygzfe */
        char line[512];
        int li = 0;
        while ((r = read(fd, buf, sizeof buf)) > 0) {
            for (ssize_t i = 0; i < r; i++) {
                if (li < (int)sizeof line - 1) line[li++] = buf[i];
                if (buf[i] == '\n') {
                    line[li] = 0;
                    if (strstr(line, "libygzfe")) write(2, line, li);
                    li = 0;
                }
            }
        }
        close(fd);
    }
    signal(sig, SIG_DFL);
    raise(sig);
}

static char alt_stack[1 << 16];
int segv_trace_install(void) {
    stack_t ss;
    ss.ss_sp = alt_stack;
    ss.ss_size = sizeof alt_stack;
    ss.ss_flags = 0;
    sigaltstack(&ss, 0);  /* a stack overflow still gets its trace */
    void *warm[4];
    backtrace(warm, 4);  /* loads the unwinder now: the handler must not allocate */
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_segv;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    return sigaction(SIGSEGV, &sa, 0);
}
