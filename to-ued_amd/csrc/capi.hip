// C-ABI plumbing for libtoued_hip.so: error state, version, device info.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <new>
#include "common.h"

namespace toued {
static thread_local char g_err[512] = "";
static toued_ctx g_default_ctx = {0};
static thread_local toued_ctx* g_current_ctx = nullptr;
toued_ctx* current_ctx() { return g_current_ctx ? g_current_ctx : &g_default_ctx; }
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

toued_ctx* toued_ctx_create(void) { return new (std::nothrow) toued_ctx{0}; }
int toued_ctx_destroy(toued_ctx* ctx) {
  if (!ctx) return 0;
  if (toued::g_current_ctx == ctx) toued::g_current_ctx = nullptr;
  delete ctx;
  return 0;
}
int toued_ctx_set_current(toued_ctx* ctx) {
  toued::g_current_ctx = ctx;
  return 0;
}
toued_ctx* toued_ctx_current(void) { return toued::current_ctx(); }
}
