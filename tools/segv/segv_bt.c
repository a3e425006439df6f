/* SIGSEGV/SIGABRT handler printing a native backtrace (diagnostics for host-side
 * crashes inside the HIP runtime, e.g. during graph capture).  Loaded with ctypes
 * by tools/with_bt.py; never part of the product. */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

static void on_fault(int sig, siginfo_t* si, void* uc) {
  (void)uc;
  void* frames[96];
  char msg[128];
  int n = snprintf(msg, sizeof msg, "\n*** signal %d (addr %p), native backtrace:\n", sig, si ? si->si_addr : 0);
  if (write(2, msg, n) < 0) {}
  int k = backtrace(frames, 96);
  backtrace_symbols_fd(frames, k, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

void segv_bt_install(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = on_fault;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigaction(SIGSEGV, &sa, 0);
  sigaction(SIGBUS, &sa, 0);
  sigaction(SIGABRT, &sa, 0);
}
