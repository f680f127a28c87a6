// C-ABI plumbing for libtoued_hip.so: error state, version, contexts, the device error word and the debug hooks
// (util/jax.py:5-17's --debug / --debug_nans).
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <mutex>
#include <new>
#include "common.h"

namespace toued {
static thread_local char g_err[512] = "";
static toued_ctx g_default_ctx;
static thread_local toued_ctx* g_current_ctx = nullptr;
toued_ctx* current_ctx() { return g_current_ctx ? g_current_ctx : &g_default_ctx; }
// toued_ctx_set_current / toued_ctx_destroy / thread exit change a context's users count under this lock, so a destroy
// cannot delete a context between another thread's check and its set_current
static std::mutex g_ctx_m;
// a thread that exits with a context current gives it back (else its users count stays raised and destroy refuses)
struct CtxExitGuard {
  ~CtxExitGuard() {
    std::lock_guard<std::mutex> lk(g_ctx_m);
    if (g_current_ctx) g_current_ctx->users.fetch_sub(1);
    g_current_ctx = nullptr;
  }
};
static thread_local CtxExitGuard g_ctx_exit_guard;
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// The device error word and its host read-back (pinned word + event): allocated by the first
// toued_device_error_check, outside any graph capture, so a captured launch only takes its address.
struct DevErr {
  std::mutex m;
  unsigned* word = nullptr;
  unsigned* host = nullptr;
  hipEvent_t ev = nullptr;
  bool pending = false;
};
static DevErr g_de;
unsigned* dev_err_word() { return g_de.word; }
static const char* deverr_text(unsigned code) {
  if (code & TOUED_DEVERR_A2C_DRAW_WAIT)
    return "k_a2c_chain (toued_a2c_chain_self): a draw wave's wait for the key wave's flag expired; the update's draws "
           "and every later trajectory of that launch are invalid";
  return "unknown device error";
}
}  // namespace toued

namespace {
// count of non-finite values (NaN, +-inf) of x[0..n) added into *out: grid-stride, one atomic per wave
__global__ void __launch_bounds__(256) k_nonfinite_count(const float* __restrict__ x, long n, int* __restrict__ out) {
  int c = 0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const unsigned b = __float_as_uint(x[i]);
    c += (b & 0x7F800000u) == 0x7F800000u;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}
// the same over a row-strided block x[r * ld + c], r < rows, c < cols (blockIdx.y strides the rows)
__global__ void __launch_bounds__(256) k_nonfinite_count_2d(const float* __restrict__ x, long rows, long cols, long ld,
                                                             int* __restrict__ out) {
  int c = 0;
  for (long r = blockIdx.y; r < rows; r += gridDim.y)
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < cols; i += (long)gridDim.x * 256) {
      const unsigned b = __float_as_uint(x[r * ld + i]);
      c += (b & 0x7F800000u) == 0x7F800000u;
    }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}
}  // namespace

extern "C" {
const char* toued_last_error(void) { return toued::g_err; }
int toued_abi_version(void) { return 1; }

toued_ctx* toued_ctx_create(void) { return new (std::nothrow) toued_ctx(); }
int toued_ctx_destroy(toued_ctx* ctx) {
  if (!ctx) return 0;
  std::lock_guard<std::mutex> lk(toued::g_ctx_m);
  const int mine = toued::g_current_ctx == ctx ? 1 : 0;
  // refused while another host thread still has it current (that thread would keep a dangling pointer)
  TOUED_REQUIRE(ctx->users.load() <= mine, "toued_ctx_destroy: context is current on %d other thread(s)",
                ctx->users.load() - mine);
  if (mine) toued::g_current_ctx = nullptr;
  delete ctx;
  return 0;
}
int toued_ctx_set_current(toued_ctx* ctx) {
  (void)&toued::g_ctx_exit_guard;   // odr-use: constructs this thread's exit guard
  std::lock_guard<std::mutex> lk(toued::g_ctx_m);
  toued_ctx* old = toued::g_current_ctx;
  if (old == ctx) return 0;
  if (ctx) ctx->users.fetch_add(1);
  if (old) old->users.fetch_sub(1);
  toued::g_current_ctx = ctx;
  return 0;
}
toued_ctx* toued_ctx_current(void) { return toued::current_ctx(); }

// Reads the device error word: wait = 1 synchronises with `stream` and reports every error of the work enqueued
// before the call; wait = 0 never blocks: it reports what the previous call's read-back (already landed) saw and
// enqueues a new read-back behind the work on `stream`.  Returns -3 with toued_last_error() describing the error
// (the word is cleared), 0 when clean.
int toued_device_error_check(hipStream_t stream, int wait) {
  using namespace toued;
  std::lock_guard<std::mutex> lk(g_de.m);
  if (!g_de.word) {
    void* w = nullptr;
    void* h = nullptr;
    TOUED_REQUIRE(hipMalloc(&w, sizeof(unsigned)) == hipSuccess && hipMemset(w, 0, sizeof(unsigned)) == hipSuccess,
                  "toued_device_error_check: cannot allocate the device error word");
    TOUED_REQUIRE(hipHostMalloc(&h, sizeof(unsigned), 0) == hipSuccess,
                  "toued_device_error_check: cannot allocate the pinned read-back word");
    TOUED_REQUIRE(hipEventCreateWithFlags(&g_de.ev, hipEventDisableTiming) == hipSuccess,
                  "toued_device_error_check: cannot create the read-back event");
    *static_cast<unsigned*>(h) = 0;
    g_de.host = static_cast<unsigned*>(h);
    g_de.word = static_cast<unsigned*>(w);
  }
  unsigned code = 0;
  if (g_de.pending) {
    const hipError_t q = wait ? hipEventSynchronize(g_de.ev) : hipEventQuery(g_de.ev);
    if (q == hipSuccess) {
      code |= *g_de.host;
      g_de.pending = false;
    } else {
      TOUED_REQUIRE(q == hipErrorNotReady, "toued_device_error_check: %s", hipGetErrorString(q));
    }
  }
  auto enqueue_readback = [&] {
    TOUED_REQUIRE(hipMemcpyAsync(g_de.host, g_de.word, sizeof(unsigned), hipMemcpyDeviceToHost, stream) == hipSuccess &&
                      hipEventRecord(g_de.ev, stream) == hipSuccess,
                  "toued_device_error_check: cannot enqueue the read-back");
    g_de.pending = true;
    return 0;
  };
  if (!g_de.pending && wait) {
    if (enqueue_readback()) return -1;
    TOUED_REQUIRE(hipEventSynchronize(g_de.ev) == hipSuccess, "toued_device_error_check: read-back failed");
    code |= *g_de.host;
    g_de.pending = false;
  }
  // the clear goes in front of the next read-back, so that read-back cannot report the same bits again (an error a
  // kernel sets between the landed read-back and the clear is lost: the word only carries expired bounded waits)
  if (code)
    TOUED_REQUIRE(hipMemsetAsync(g_de.word, 0, sizeof(unsigned), stream) == hipSuccess,
                  "toued_device_error_check: cannot clear the device error word (device error 0x%x: %s)", code,
                  deverr_text(code));
  if (!g_de.pending && !wait && enqueue_readback()) return -1;
  if (code) {
    set_error("device error 0x%x: %s", code, deverr_text(code));
    return -3;
  }
  return 0;
}

// --debug (util/jax.py:12-14 runs the step without jit): synchronise the device and surface any asynchronous
// error of the work enqueued so far
int toued_sync_check(void) {
  const hipError_t e = hipDeviceSynchronize();
  TOUED_REQUIRE(e == hipSuccess, "device error after synchronize: %s", hipGetErrorString(e));
  const hipError_t l = hipGetLastError();
  TOUED_REQUIRE(l == hipSuccess, "pending HIP error: %s", hipGetErrorString(l));
  return 0;
}

// --debug_nans (util/jax.py:9-10, jax_debug_nans): *out += number of non-finite floats in x[0..n) (stream-ordered)
int toued_nonfinite_count(const float* x, long n, int* out, hipStream_t stream) {
  TOUED_REQUIRE(n >= 0 && out && (n == 0 || x), "toued_nonfinite_count: bad arguments");
  if (n == 0) return 0;
  const long blocks = (n + 255) / 256;
  hipLaunchKernelGGL(k_nonfinite_count, dim3((unsigned)(blocks < 2048 ? blocks : 2048)), dim3(256), 0, stream, x, n,
                     out);
  TOUED_CHECK_LAUNCH();
  return 0;
}
// the same for a row-strided block: rows x cols floats, row pitch ld >= cols
int toued_nonfinite_count_2d(const float* x, long rows, long cols, long ld, int* out, hipStream_t stream) {
  TOUED_REQUIRE(rows >= 0 && cols >= 0 && ld >= cols && out && (rows * cols == 0 || x),
                "toued_nonfinite_count_2d: bad arguments");
  if (rows * cols == 0) return 0;
  const long bx = (cols + 255) / 256;
  const long gx = bx < 64 ? bx : 64, gy = rows < 256 ? rows : 256;
  hipLaunchKernelGGL(k_nonfinite_count_2d, dim3((unsigned)gx, (unsigned)gy), dim3(256), 0, stream, x, rows, cols, ld,
                     out);
  TOUED_CHECK_LAUNCH();
  return 0;
}
}
