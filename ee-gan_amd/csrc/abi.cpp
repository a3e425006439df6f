// Error plumbing + version query for the C-ABI library (no global mutable
// state shared between threads: the error text is thread-local).
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "../../include/eegan_hip.h"

static thread_local char g_err[512];

void ee_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int ee_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    ee_set_error("%s: %s", what, hipGetErrorString(e));
    return -(int)e;
  }
  return 0;
}

extern "C" {
const char* eegan_last_error(void) { return g_err; }
int eegan_abi_version(void) { return EEGAN_ABI_VERSION; }
}
