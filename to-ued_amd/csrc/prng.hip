// jax.random key plumbing on device: split / fold_in / bits / uniform / bernoulli
// over batches of keys, so the host orchestration (train loop, level sampler)
// never round-trips keys through the CPU.
#include "common.h"

namespace {

// out[i, j] = split(keys[i], num)[j]; PLANAR: the same key at out[j, i] (each j one contiguous key batch)
template <bool PLANAR>
__global__ void __launch_bounds__(256) k_split(const uint32_t* __restrict__ keys, int num, uint32_t* __restrict__ out,
                                               int n) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)n * num) return;
  const int i = (int)(t / num), j = (int)(t - (long)i * num);
  const uint2 k = split_at(make_uint2(keys[2 * i], keys[2 * i + 1]), (uint32_t)num, (uint32_t)j);
  const long o = PLANAR ? (long)j * n + i : t;
  out[2 * o] = k.x;
  out[2 * o + 1] = k.y;
}

__global__ void __launch_bounds__(256) k_fold_in(const uint32_t* __restrict__ keys, uint32_t data,
                                                 uint32_t* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint2 y = threefry(keys[2 * i], keys[2 * i + 1], 0u, data);
  out[2 * i] = y.x;
  out[2 * i + 1] = y.y;
}

// random_bits(keys[i], (m,))[j]
__global__ void __launch_bounds__(256) k_bits(const uint32_t* __restrict__ keys, int m, uint32_t* __restrict__ out,
                                              int n) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)n * m) return;
  const int i = (int)(t / m), j = (int)(t - (long)i * m);
  out[t] = random_bits_at(make_uint2(keys[2 * i], keys[2 * i + 1]), (uint32_t)m, (uint32_t)j);
}

__global__ void __launch_bounds__(256) k_uniform(const uint32_t* __restrict__ keys, int m, float lo, float hi,
                                                 float* __restrict__ out, int n) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)n * m) return;
  const int i = (int)(t / m), j = (int)(t - (long)i * m);
  out[t] = uniform_from_bits(random_bits_at(make_uint2(keys[2 * i], keys[2 * i + 1]), (uint32_t)m, (uint32_t)j), lo,
                             hi);
}

// normal(keys[i], (m,))[j] (jax.random.normal, f32): sqrt2 * erf_inv(uniform(nextafter(-1, 0), 1))
__global__ void __launch_bounds__(256) k_normal(const uint32_t* __restrict__ keys, int m, float* __restrict__ out,
                                                int n) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)n * m) return;
  const int i = (int)(t / m), j = (int)(t - (long)i * m);
  const float u = uniform_from_bits(random_bits_at(make_uint2(keys[2 * i], keys[2 * i + 1]), (uint32_t)m, (uint32_t)j),
                                    -0.99999994f, 1.0f);
  out[t] = __fmul_rn(1.41421354f, erfinv_giles(u));
}

}  // namespace

extern "C" {

int toued_split(const uint32_t* keys, int n, int num, uint32_t* out, hipStream_t stream) {
  TOUED_REQUIRE(n >= 0 && num >= 1, "toued_split: n=%d num=%d", n, num);
  const long tot = (long)n * num;
  if (tot == 0) return 0;
  hipLaunchKernelGGL(k_split<false>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, keys, num, out, n);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_split_planar(const uint32_t* keys, int n, int num, uint32_t* out, hipStream_t stream) {
  TOUED_REQUIRE(n >= 0 && num >= 1, "toued_split_planar: n=%d num=%d", n, num);
  const long tot = (long)n * num;
  if (tot == 0) return 0;
  hipLaunchKernelGGL(k_split<true>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, keys, num, out, n);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_fold_in(const uint32_t* keys, int n, uint32_t data, uint32_t* out, hipStream_t stream) {
  TOUED_REQUIRE(n >= 0, "toued_fold_in: n=%d", n);
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_fold_in, dim3((n + 255) / 256), dim3(256), 0, stream, keys, data, out, n);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_random_bits(const uint32_t* keys, int n, int m, uint32_t* out, hipStream_t stream) {
  TOUED_REQUIRE(n >= 0 && m >= 1, "toued_random_bits: n=%d m=%d", n, m);
  const long tot = (long)n * m;
  if (tot == 0) return 0;
  hipLaunchKernelGGL(k_bits, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, keys, m, out, n);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_uniform(const uint32_t* keys, int n, int m, float lo, float hi, float* out, hipStream_t stream) {
  TOUED_REQUIRE(n >= 0 && m >= 1, "toued_uniform: n=%d m=%d", n, m);
  const long tot = (long)n * m;
  if (tot == 0) return 0;
  hipLaunchKernelGGL(k_uniform, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, keys, m, lo, hi, out, n);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_normal(const uint32_t* keys, int n, int m, float* out, hipStream_t stream) {
  TOUED_REQUIRE(n >= 0 && m >= 1, "toued_normal: n=%d m=%d", n, m);
  const long tot = (long)n * m;
  if (tot == 0) return 0;
  hipLaunchKernelGGL(k_normal, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, keys, m, out, n);
  TOUED_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
