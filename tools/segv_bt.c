/* Debug aid (host only): a SIGSEGV handler that prints the native backtrace (glibc
 * backtrace_symbols_fd: exported symbols of each frame's library) to stderr, then hands the
 * signal to the previously installed handler (Python's faulthandler prints the Python stack).
 * Loaded with ctypes when CCMPC_SEGV_BT=1 (tests/conftest.py).  Build:
 *   gcc -O1 -g -fPIC -shared tools/segv_bt.c -o tools/libsegvbt.so */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static struct sigaction prev;

static void handler(int sig, siginfo_t *si, void *uc) {
  void *frames[64];
  static const char msg[] = "\n=== native backtrace (segv_bt) ===\n";
  write(2, msg, sizeof(msg) - 1);
  int n = backtrace(frames, 64);
  backtrace_symbols_fd(frames, n, 2);
  sigaction(SIGSEGV, &prev, NULL);
  if (prev.sa_flags & SA_SIGINFO) {
    if (prev.sa_sigaction) prev.sa_sigaction(sig, si, uc);
  } else if (prev.sa_handler != SIG_DFL && prev.sa_handler != SIG_IGN) {
    prev.sa_handler(sig);
  }
  raise(sig);
}

int segv_bt_install(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = handler;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigemptyset(&sa.sa_mask);
  return sigaction(SIGSEGV, &sa, &prev);
}
