// Level-buffer sampling kernels (environments/level_sampler.py:155-408).
//
//  k_choice_cdf   jax.random.choice(key, B, (n,), replace=True, p) given the CPU-order cumsum of p
//                 (frozen buffer, level_sampler.py:157-165): searchsorted(c, c[-1]*(1-u), 'left').
#include "common.h"

namespace {

__global__ void __launch_bounds__(256) k_choice_cdf(const uint32_t* __restrict__ key, const float* __restrict__ cdf,
                                                    int B, int n, int* __restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint2 k = make_uint2(key[0], key[1]);
  const float u = bits_to_unit(random_bits_at(k, (uint32_t)n, (uint32_t)j));
  const float r = __fmul_rn(cdf[B - 1], __fsub_rn(1.0f, u));
  int lo = 0, hi = B;   // first index with cdf[i] >= r  (== count of cdf < r for a sorted array)
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (cdf[mid] < r) lo = mid + 1; else hi = mid;
  }
  out[j] = lo;
}

}  // namespace

extern "C" {

int toued_choice_cdf(const uint32_t* key, const float* cdf, int B, int n, int* out, hipStream_t stream) {
  TOUED_REQUIRE(B >= 1 && n >= 0, "toued_choice_cdf: B=%d n=%d", B, n);
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_choice_cdf, dim3((n + 255) / 256), dim3(256), 0, stream, key, cdf, B, n, out);
  TOUED_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
