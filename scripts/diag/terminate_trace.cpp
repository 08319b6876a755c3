// Diagnostic (not product code): a std::terminate handler and a SIGABRT
// handler that print the native backtrace of the calling thread to stderr, so
// an exit-time "terminate called without an active exception" names the
// destructor that called it.  Loaded with ctypes by scripts/diag/teardown_stress.py.
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <exception>

namespace {
void dump(const char* why) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  dprintf(2, "\n=== %s: native backtrace (pid %d) ===\n", why, getpid());
  backtrace_symbols_fd(frames, n, 2);
  dprintf(2, "=== end ===\n");
}
void on_terminate() {
  dump("std::terminate");
  std::abort();
}
void on_abrt(int) {
  dump("SIGABRT");
  signal(SIGABRT, SIG_DFL);
  raise(SIGABRT);
}
struct Install {
  Install() {
    std::set_terminate(on_terminate);
    signal(SIGABRT, on_abrt);
  }
} install;
}  // namespace

extern "C" int gs_diag_terminate_trace_installed(void) { return 1; }
