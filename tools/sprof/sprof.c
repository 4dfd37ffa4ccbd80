/* sprof.c -- PROFILING INFRASTRUCTURE ONLY (host code, never shipped, never on
 * a GPU box): a tiny sampling profiler for the host code of the stage-3 pass.
 * LD_PRELOAD it; every SPROF_US microseconds of process CPU time (ITIMER_PROF)
 * the interrupted thread's program counter is recorded, and at exit the
 * samples are written to $SPROF_OUT.PID (one hex PC per line) after the process's
 * /proc/self/maps, so tools/sprof/report.py can attribute them to functions
 * with addr2line.
 *   gcc -O2 -shared -fPIC -o /tmp/sprof.so tools/sprof/sprof.c
 *   SPROF_OUT=/tmp/s.txt LD_PRELOAD=/tmp/sprof.so python ...
 */
#define _GNU_SOURCE
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>
#include <execinfo.h>
#include <ucontext.h>
#include <unistd.h>

#define MAXS (1 << 20)
#define DEPTH 6 /* the sampled PC, then the return addresses above the handler's frames */
static unsigned long pcs[MAXS][DEPTH];
static volatile int nsamp;

static void on_prof(int sig, siginfo_t* si, void* uc) {
  (void)sig, (void)si;
  const ucontext_t* u = (const ucontext_t*)uc;
  const int i = __sync_fetch_and_add(&nsamp, 1);
  if (i >= MAXS) return;
  pcs[i][0] = (unsigned long)u->uc_mcontext.gregs[REG_RIP];
  void* bt[DEPTH + 3];
  const int n = backtrace(bt, DEPTH + 3); /* handler, the signal trampoline, then the interrupted frames */
  for (int d = 1; d < DEPTH; d++) pcs[i][d] = d + 2 < n ? (unsigned long)bt[d + 2] : 0ul;
}

static void dump(void) {
  const char* out = getenv("SPROF_OUT");
  if (!out) return;
  struct itimerval z;
  memset(&z, 0, sizeof(z));
  setitimer(ITIMER_PROF, &z, NULL);
  char path[4096];
  snprintf(path, sizeof(path), "%s.%d", out, (int)getpid());
  FILE* f = fopen(path, "w");
  if (!f) return;
  FILE* m = fopen("/proc/self/maps", "r");
  char line[4096];
  while (m && fgets(line, sizeof(line), m)) fprintf(f, "M %s", line);
  if (m) fclose(m);
  const int n = nsamp < MAXS ? nsamp : MAXS;
  for (int i = 0; i < n; i++) {
    for (int d = 0; d < DEPTH; d++) fprintf(f, d ? " %lx" : "%lx", pcs[i][d]);
    fprintf(f, "\n");
  }
  fclose(f);
}

__attribute__((constructor)) static void start(void) {
  if (!getenv("SPROF_OUT")) return;
  void* warm[4];
  backtrace(warm, 4); /* loads the unwinder before the first signal */
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigaction(SIGPROF, &sa, NULL);
  const char* e = getenv("SPROF_US");
  const long us = e ? atol(e) : 500;
  struct itimerval it;
  it.it_interval.tv_sec = 0;
  it.it_interval.tv_usec = us;
  it.it_value = it.it_interval;
  setitimer(ITIMER_PROF, &it, NULL);
  atexit(dump);
}
