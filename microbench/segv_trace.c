/* Diagnostic: a SIGSEGV/SIGABRT handler that prints the native backtrace (exported symbol
 * names + offsets) to stderr, for a crash inside a library in a Python process
 * (scripts/experiments/graph_probe.py loads it with ctypes). Build:
 * gcc -O1 -g -shared -fPIC -o microbench/libsegv_trace.so microbench/segv_trace.c */
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

static void handler(int sig, siginfo_t* si, void* ctx) {
    (void)ctx;
    void* bt[64];
    char msg[128];
    const int n = backtrace(bt, 64);
    const int len = snprintf(msg, sizeof msg, "native signal %d at address %p, backtrace:\n", sig, si ? si->si_addr : 0);
    if (len > 0) (void)!write(2, msg, (size_t)len);
    backtrace_symbols_fd(bt, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

int segv_trace_install(void) {
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
    sigaction(SIGSEGV, &sa, 0);
    sigaction(SIGABRT, &sa, 0);
    return 0;
}
