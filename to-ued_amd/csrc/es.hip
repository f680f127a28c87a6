// OpenES for the LPG parameters (meta/train.py:133-227, models/optim.py:21-34) — HIP for gfx950.
//
// evosax 0.1.4 OpenES (setup/requirements-base.txt:2; not vendored — restated):
//   ask:  z = jax.random.normal(rng, (P/2, nd)); x = mean + sigma * concat(z, -z)
//         (then meta/train.py:152-158 reorders so candidates 2i, 2i+1 are the antithetic pair i)
//   tell: noise = (x - mean) / sigma; grad = 1/(P sigma) * noise^T . fitness_shaped
//         (fitness_shaped = -rank_fitness: maximize=True), then the evosax optimiser step
//         (Adam b1=.99 b2=.999 eps=1e-8, or SGD), lrate / sigma exponential decay with limits.
//
//   k_es_ask    the candidate pairs of rows [row_lo, row_lo + n_rows) of z (a rank's agents)
//   k_es_grad   per-parameter partial sum over this rank's candidates (all-reduced by the host)
//   k_es_adam   optimiser step on the mean
#include "common.h"

__global__ void __launch_bounds__(256) k_es_ask(const uint32_t* __restrict__ keyp, long nd, uint32_t count, long row_lo, long n_rows,
                                                const float* __restrict__ mean, float sigma, float* __restrict__ x) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_rows * nd) return;
  const long i = e / nd, j = e - i * nd;
  const uint2 key = make_uint2(keyp[0], keyp[1]);
  const uint32_t flat = (uint32_t)((row_lo + i) * nd + j);
  const float u = uniform_from_bits(random_bits_at(key, count, flat), -0.99999994f, 1.0f);
  const float z = __fmul_rn(1.41421354f, erfinv_giles(u));
  const float m = mean[j];
  x[(2 * i) * nd + j] = __fadd_rn(m, __fmul_rn(sigma, z));
  x[(2 * i + 1) * nd + j] = __fadd_rn(m, __fmul_rn(sigma, -z));
}

__global__ void __launch_bounds__(256) k_es_grad(const float* __restrict__ x, const float* __restrict__ mean,
                                                 float sigma, const float* __restrict__ fit, int C, long nd,
                                                 float* __restrict__ out) {
  const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nd) return;
  const float m = mean[j];
  float acc = 0.0f;
  for (int c = 0; c < C; ++c) acc += ((x[(long)c * nd + j] - m) / sigma) * fit[c];
  out[j] = acc;
}

// opt: 0 = SGD (momentum 0), 1 = Adam.  bc1 = 1 - b1^(n+1), bc2 = 1 - b2^(n+1).
__global__ void __launch_bounds__(256) k_es_opt(long nd, int opt, float* __restrict__ mean,
                                                const float* __restrict__ grad, float scale, float* __restrict__ m,
                                                float* __restrict__ v, float lrate, float b1, float b2, float eps,
                                                float bc1, float bc2) {
  const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nd) return;
  const float g = scale * grad[j];
  if (opt == 0) {
    m[j] = g;
    mean[j] = mean[j] - lrate * g;
    return;
  }
  const float mj = (1.0f - b1) * g + b1 * m[j];
  const float vj = (1.0f - b2) * (g * g) + b2 * v[j];
  m[j] = mj;
  v[j] = vj;
  const float mhat = mj / bc1, vhat = vj / bc2;
  mean[j] = mean[j] - lrate * mhat / (sqrtf(vhat) + eps);
}

extern "C" {

int toued_es_ask(const uint32_t* key, long nd, long half_pop, long row_lo, long n_rows, const float* mean,
                 float sigma, float* x, hipStream_t stream) {
  TOUED_REQUIRE(key && nd > 0 && half_pop > 0 && row_lo >= 0 && n_rows >= 0 && row_lo + n_rows <= half_pop,
                "toued_es_ask: bad sizes");
  TOUED_REQUIRE((double)half_pop * (double)nd < 4294967296.0, "toued_es_ask: P/2 * nd must be < 2^32");
  if (n_rows == 0) return 0;
  const long n = n_rows * nd;
  hipLaunchKernelGGL(k_es_ask, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     key, nd, (uint32_t)(half_pop * nd), row_lo, n_rows, mean, sigma, x);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_es_grad(const float* x, const float* mean, float sigma, const float* fitness, int C, long nd, float* out,
                  hipStream_t stream) {
  TOUED_REQUIRE(C >= 0 && nd > 0, "toued_es_grad: bad sizes");
  hipLaunchKernelGGL(k_es_grad, dim3((unsigned)((nd + 255) / 256)), dim3(256), 0, stream, x, mean, sigma, fitness, C,
                     nd, out);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_es_opt(long nd, int opt, float* mean, const float* grad, float scale, float* m, float* v, float lrate,
                 float b1, float b2, float eps, float bc1, float bc2, hipStream_t stream) {
  TOUED_REQUIRE(nd > 0 && (opt == 0 || opt == 1), "toued_es_opt: bad arguments");
  hipLaunchKernelGGL(k_es_opt, dim3((unsigned)((nd + 255) / 256)), dim3(256), 0, stream, nd, opt, mean, grad, scale, m,
                     v, lrate, b1, b2, eps, bc1, bc2);
  TOUED_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
