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

// level_sampler.sample with score_function=random (level_sampler.py:134-194 with _sample_random_levels :268-271 and
// _create_agent :273-291), its key plumbing and termination test for agent i of this rank (global index lo + i of
// n_total) in one thread instead of ~20 launches of splits, copies and elementwise ops:
//   term = step >= lifetime; mask = term; step (and vstep) = term ? 0 : step
//   (rng1, s1) = split(rng):  keys[0] = split(s1, n_total)[lo + i]                     (the new level)
//   (rng2, s2) = split(rng1): (reset, agent) = split(split(s2, n_total)[lo + i])
//                             keys[1] = reset; (actor, critic) = split(agent)
//                             keys[2] = fold_in(actor, h), keys[3] = fold_in(critic, h)  (lecun_tables' Dense_0 key)
//   vstep given:  (_, s3) = split(rng2): keys[4] = fold_in(split(s3, n_total)[lo + i], h) (the value critic)
__global__ void __launch_bounds__(256) k_sample_random_keys(const uint32_t* __restrict__ rng, int n_total, int lo, int n,
                                                            int* __restrict__ step, const int* __restrict__ levels,
                                                            int* __restrict__ vstep, uint32_t h,
                                                            uint8_t* __restrict__ mask, uint32_t* __restrict__ keys) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int st = step[i];
  const bool term = st >= levels[(size_t)i * LEVEL_WORDS + L_LIFETIME];
  mask[i] = term ? 1 : 0;
  if (term) {
    step[i] = 0;
    if (vstep) vstep[i] = 0;
  }
  auto put = [&](int j, uint2 k) {
    keys[((size_t)j * n + i) * 2] = k.x;
    keys[((size_t)j * n + i) * 2 + 1] = k.y;
  };
  const uint32_t g = (uint32_t)(lo + i);
  uint2 rng1, s1, rng2, s2, s3, reset, agent, actor, critic;
  split2(make_uint2(rng[0], rng[1]), rng1, s1);
  put(0, split_at(s1, (uint32_t)n_total, g));
  split2(rng1, rng2, s2);
  split2(split_at(s2, (uint32_t)n_total, g), reset, agent);
  put(1, reset);
  split2(agent, actor, critic);
  put(2, threefry(actor.x, actor.y, 0u, h));
  put(3, threefry(critic.x, critic.y, 0u, h));
  if (vstep) {
    uint2 rng3;
    split2(rng2, rng3, s3);
    const uint2 v = split_at(s3, (uint32_t)n_total, g);
    put(4, threefry(v.x, v.y, 0u, h));
  }
}

}  // namespace

extern "C" {

int toued_sample_random_keys(const uint32_t* rng, int n_total, int lo, int n, int* step, const int* levels, int* vstep,
                             uint32_t dense_hash, uint8_t* mask, uint32_t* keys, hipStream_t stream) {
  TOUED_REQUIRE(n >= 0 && lo >= 0 && lo + n <= n_total, "toued_sample_random_keys: lo=%d n=%d n_total=%d", lo, n,
                n_total);
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_sample_random_keys, dim3((n + 255) / 256), dim3(256), 0, stream, rng, n_total, lo, n, step,
                     levels, vstep, dense_hash, mask, keys);
  TOUED_CHECK_LAUNCH();
  return 0;
}

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
