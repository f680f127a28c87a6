// C-ABI plumbing for libtoued_hip.so: error state, version, device info.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include "common.h"

namespace toued {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace toued

extern "C" {
const char* toued_last_error(void) { return toued::g_err; }
int toued_abi_version(void) { return 1; }
}
