// hostprof.c — a sampling profiler for the host side of an e2e run (tools/e2e_llama.py --hostprof):
// a CLOCK_MONOTONIC timer signals the calling thread every period (wall clock: blocked time shows as the
// blocking call) and records its call stack (up to 12 frames) into a fixed buffer; hostprof_stop() writes the stacks and /proc/self/maps to a file that
// tools/hostprof_report.py resolves with addr2line.  Loaded with ctypes (never preloaded).
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>
#include <ucontext.h>
#include <unistd.h>
#include <sys/syscall.h>
#include <time.h>

static timer_t g_timer;

#define MAXS 5000      // a ring: the last MAXS samples (the end of the run: the decode steps)
#define DEPTH 12
static void *g_buf[MAXS][DEPTH];
static int g_tid[MAXS];
static volatile int g_n = 0;
static volatile int g_on = 0;

static void on_prof(int sig, siginfo_t *si, void *uc) {
    (void)sig;
    (void)si;
    if (!g_on) return;
    int i = __sync_fetch_and_add(&g_n, 1) % MAXS;
    void *fr[DEPTH + 2];
    int n = backtrace(fr, DEPTH + 2);
    // frame 0: this handler, 1: the signal trampoline; the interrupted PC from the context first
    ucontext_t *u = (ucontext_t *)uc;
    g_buf[i][0] = (void *)u->uc_mcontext.gregs[REG_RIP];
    for (int k = 1; k < DEPTH; k++) g_buf[i][k] = (k + 1 < n) ? fr[k + 1] : 0;
    g_tid[i] = (int)syscall(SYS_gettid);
}

int hostprof_start(int period_us) {
    void *fr[4];
    backtrace(fr, 4);   // load libgcc's unwinder outside the handler
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = on_prof;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    sigaction(SIGPROF, &sa, 0);
    g_n = 0;
    g_on = 1;
    struct sigevent ev;
    memset(&ev, 0, sizeof(ev));
    ev.sigev_notify = SIGEV_THREAD_ID;
    ev.sigev_signo = SIGPROF;
    ev._sigev_un._tid = (int)syscall(SYS_gettid);
    if (timer_create(CLOCK_MONOTONIC, &ev, &g_timer) != 0) return -1;
    struct itimerspec it;
    const long ns = (period_us > 0 ? period_us : 100) * 1000L;
    it.it_interval.tv_sec = 0;
    it.it_interval.tv_nsec = ns;
    it.it_value = it.it_interval;
    return timer_settime(g_timer, 0, &it, 0);
}

int hostprof_stop(const char *path) {
    timer_delete(g_timer);
    g_on = 0;
    FILE *f = fopen(path, "w");
    if (!f) return -1;
    FILE *m = fopen("/proc/self/maps", "r");
    char line[4096];
    while (m && fgets(line, sizeof(line), m)) fprintf(f, "M %s", line);
    if (m) fclose(m);
    int n = g_n < MAXS ? g_n : MAXS;
    for (int i = 0; i < n; i++) {
        fprintf(f, "S %d", g_tid[i]);
        for (int k = 0; k < DEPTH && g_buf[i][k]; k++) fprintf(f, " %lx", (unsigned long)(uintptr_t)g_buf[i][k]);
        fprintf(f, "\n");
    }
    fclose(f);
    return n;
}
