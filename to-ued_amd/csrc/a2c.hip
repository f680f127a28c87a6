// A2C antagonist update (agents/a2c.py:19-125) — HIP for gfx950.
//
//   k_key_chain  the scan carry of train_a2c_agent (a2c.py:94-97): rng, _rng = split(rng) per update
//   k_a2c_grad   one block per agent: per-worker GAE (util/metrics.py:17-38) on the value critic
//                [T+1, 1], advantage normalisation over the agent's [W, T] (a2c.py:43), critic
//                gradient of mean((target - V)^2) with stop-gradient targets, actor gradient of
//                mean(-log(pi_a + 1e-8) [T] * adv [T,1]) (the [T,T] broadcast = -mean_t log pi *
//                mean_t adv per worker) - entropy_coeff * H(pi + 1e-8)   (a2c.py:29-63)
//   k_a2c_apply  optax clip_by_global_norm + SGD per TrainState (models/optim.py:5-11), discard when
//                the new step exceeds the lifetime (a2c.py:71-75); clears the gradient tables
//
// Trajectory layout as the rollout kernel writes it: idx/time [N][T+1][W], act/done/rew [N][T][W].
#include "common.h"

#define EPSF 1e-8f

namespace {

TOUED_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sum for 256-thread blocks; every thread gets the result.
TOUED_DEV float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int wv = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[wv] = v;
  __syncthreads();
  float s = 0.0f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  return s;
}

}  // namespace

__global__ void k_key_chain(const uint32_t* __restrict__ keys, int n, int U, uint32_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint2 k = make_uint2(keys[2 * i], keys[2 * i + 1]);
  for (int u = 0; u < U; ++u) {
    uint2 nk, sub;
    split2(k, nk, sub);
    k = nk;
    out[((size_t)u * n + i) * 2 + 0] = sub.x;
    out[((size_t)u * n + i) * 2 + 1] = sub.y;
  }
}

// loss_out[a] += {actor_loss, critic_loss} (accumulated over updates; the caller zeroes it)
__global__ void __launch_bounds__(256) k_a2c_grad(int W, int T, int D, const float* __restrict__ theta,
                                                  const float* __restrict__ vcrit, const int* __restrict__ tidx,
                                                  const int* __restrict__ ttime, const uint8_t* __restrict__ tact,
                                                  const float* __restrict__ trew, const uint8_t* __restrict__ tdone,
                                                  float gamma, float lam, float ent_coef, float* __restrict__ Ga,
                                                  float* __restrict__ Gv, float* __restrict__ loss_out) {
  extern __shared__ float lds[];
  float* adv = lds;              // [W*T]  GAE advantages, worker-major
  float* dv = lds + W * T;       // [W*T]  target - V
  float* abar = lds + 2 * W * T; // [W]    mean_t normalised advantage
  __shared__ float red[8];
  const int a = blockIdx.x;
  const int tid = threadIdx.x;
  const float* v = vcrit + (size_t)a * D;
  const float vlast = v[D - 1];
  const size_t tb = (size_t)a * (T + 1) * W;  // trajectory obs base
  const size_t sb = (size_t)a * T * W;        // trajectory step base
  // ---- per-worker GAE (reverse scan over T)
  float s_adv = 0.0f, s_cl = 0.0f;
  for (int w = tid; w < W; w += blockDim.x) {
    float vn = v[tidx[tb + (size_t)T * W + w]] + ((float)ttime[tb + (size_t)T * W + w] * 0.001f) * vlast;
    float g = 0.0f, cl = 0.0f;
    for (int t = T - 1; t >= 0; --t) {
      const size_t o = tb + (size_t)t * W + w;
      const size_t s = sb + (size_t)t * W + w;
      const float vt = v[tidx[o]] + ((float)ttime[o] * 0.001f) * vlast;
      const float nd = tdone[s] ? 0.0f : 1.0f;
      const float delta = trew[s] + (gamma * vn * nd - vt);
      g = delta + gamma * lam * nd * g;
      const float e = (g + vt) - vt;
      adv[w * T + t] = g;
      dv[w * T + t] = e;
      cl += e * e;
      s_adv += g;
      vn = vt;
    }
    s_cl += cl / (float)T;
  }
  const float n = (float)(W * T);
  const float mean = block_sum(s_adv, red) / n;
  const float closs = block_sum(s_cl, red) / (float)W;
  float s_var = 0.0f;
  for (int i = tid; i < W * T; i += blockDim.x) {
    const float d = adv[i] - mean;
    s_var += d * d;
  }
  const float inv_sd = 1.0f / (sqrtf(block_sum(s_var, red) / n) + EPSF);
  for (int w = tid; w < W; w += blockDim.x) {
    float ab = 0.0f;
    for (int t = 0; t < T; ++t) ab += (adv[w * T + t] - mean) * inv_sd;
    abar[w] = ab / (float)T;
  }
  __syncthreads();
  // ---- per-sample actor / critic gradients
  const float* th = theta + (size_t)a * D * 5;
  float* ga = Ga + (size_t)a * D * 5;
  float* gv = Gv + (size_t)a * D;
  float lastA[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) lastA[j] = th[(size_t)(D - 1) * 5 + j];
  const float inv_n = 1.0f / n;
  float accA[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f}, accV = 0.0f, s_al = 0.0f;
  for (int i = tid; i < W * T; i += blockDim.x) {
    const int t = i / W, w = i - t * W;
    const size_t o = tb + (size_t)t * W + w;
    const int idx = tidx[o];
    const float c = (float)ttime[o] * 0.001f;
    const int act = tact[sb + (size_t)t * W + w];
    float l[5], p[5], m = -__builtin_inff();
#pragma unroll
    for (int j = 0; j < 5; ++j) { l[j] = th[(size_t)idx * 5 + j] + c * lastA[j]; m = fmaxf(m, l[j]); }
    float z = 0.0f;
#pragma unroll
    for (int j = 0; j < 5; ++j) { p[j] = __expf(l[j] - m); z += p[j]; }
    const float iz = 1.0f / z;
    float pa = 0.0f, h = 0.0f, gl[5], pg = 0.0f;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      p[j] *= iz;
      pa = (j == act) ? p[j] : pa;
      const float lg = __logf(p[j] + EPSF);
      h -= (p[j] + EPSF) * lg;
      gl[j] = -(lg + 1.0f);
      pg += p[j] * gl[j];
    }
    const float ab = abar[w];
    const float rho = pa / (pa + EPSF);
    const float kap = -ab * inv_n;
    const float ke = -ent_coef * inv_n;
    float d[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      d[j] = kap * rho * ((j == act ? 1.0f : 0.0f) - p[j]) + ke * p[j] * (gl[j] - pg);
      atomicAdd(&ga[(size_t)idx * 5 + j], d[j]);
      accA[j] += c * d[j];
    }
    const float dvv = -2.0f * dv[w * T + t] * inv_n;
    atomicAdd(&gv[idx], dvv);
    accV += c * dvv;
    s_al += -__logf(pa + EPSF) * ab - ent_coef * h;
  }
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const float r = block_sum(accA[j], red);
    if (tid == 0) atomicAdd(&ga[(size_t)(D - 1) * 5 + j], r);
  }
  const float rv = block_sum(accV, red);
  const float al = block_sum(s_al, red) * inv_n;
  if (tid == 0) {
    atomicAdd(&gv[D - 1], rv);
    loss_out[a * 2 + 0] += al;
    loss_out[a * 2 + 1] += closs;
  }
}

// One block per agent.  In place on theta/vcrit; clears Ga/Gv for the next update.
__global__ void __launch_bounds__(256) k_a2c_apply(int D, float* __restrict__ theta, float* __restrict__ vcrit,
                                                   float* __restrict__ Ga, float* __restrict__ Gv, float lr_a,
                                                   float lr_c, float max_norm, int* __restrict__ step,
                                                   const int* __restrict__ levels) {
  __shared__ float red[8];
  const int a = blockIdx.x;
  const size_t na = (size_t)D * 5;
  float* ga = Ga + (size_t)a * na;
  float* gv = Gv + (size_t)a * D;
  float sa = 0.0f, sc = 0.0f;
  for (size_t i = threadIdx.x; i < na; i += blockDim.x) sa += ga[i] * ga[i];
  for (size_t i = threadIdx.x; i < (size_t)D; i += blockDim.x) sc += gv[i] * gv[i];
  const float gna = sqrtf(block_sum(sa, red));
  const float gnc = sqrtf(block_sum(sc, red));
  const int st = step[a];
  const bool applied = (st + 1) <= levels[(size_t)a * LEVEL_WORDS + L_LIFETIME];
  const bool clip_a = !(gna < max_norm), clip_c = !(gnc < max_norm);
  float* pa = theta + (size_t)a * na;
  float* pc = vcrit + (size_t)a * D;
  for (size_t i = threadIdx.x; i < na; i += blockDim.x) {
    const float g = clip_a ? (ga[i] / gna) * max_norm : ga[i];
    if (applied) pa[i] = pa[i] + (-(lr_a * g));
    ga[i] = 0.0f;
  }
  for (size_t i = threadIdx.x; i < (size_t)D; i += blockDim.x) {
    const float g = clip_c ? (gv[i] / gnc) * max_norm : gv[i];
    if (applied) pc[i] = pc[i] + (-(lr_c * g));
    gv[i] = 0.0f;
  }
  if (threadIdx.x == 0) step[a] = applied ? st + 1 : st;
}

extern "C" {

int toued_key_chain(const uint32_t* keys, int n, int U, uint32_t* out, hipStream_t stream) {
  TOUED_REQUIRE(n >= 0 && U >= 0, "toued_key_chain: bad sizes");
  if (n == 0 || U == 0) return 0;
  TOUED_REQUIRE(keys && out, "toued_key_chain: null buffer");
  hipLaunchKernelGGL(k_key_chain, dim3((n + 255) / 256), dim3(256), 0, stream, keys, n, U, out);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_a2c_grad(int N, int W, int T, int D, const float* theta, const float* vcrit, const int* tidx,
                   const int* ttime, const uint8_t* tact, const float* trew, const uint8_t* tdone, float gamma,
                   float lam, float ent_coef, float* Ga, float* Gv, float* loss_out, hipStream_t stream) {
  TOUED_REQUIRE(N >= 0 && W > 0 && T > 0 && D > 1, "toued_a2c_grad: bad sizes");
  TOUED_REQUIRE((size_t)(2 * W * T + W) * sizeof(float) <= 64 * 1024, "toued_a2c_grad: W*T too large for LDS");
  if (N == 0) return 0;
  const size_t lds = (size_t)(2 * W * T + W) * sizeof(float);
  hipLaunchKernelGGL(k_a2c_grad, dim3(N), dim3(256), lds, stream, W, T, D, theta, vcrit, tidx, ttime, tact, trew,
                     tdone, gamma, lam, ent_coef, Ga, Gv, loss_out);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_a2c_apply(int N, int D, float* theta, float* vcrit, float* Ga, float* Gv, float lr_a, float lr_c,
                    float max_norm, int* step, const int* levels, hipStream_t stream) {
  TOUED_REQUIRE(N >= 0 && D > 1, "toued_a2c_apply: bad sizes");
  if (N == 0) return 0;
  hipLaunchKernelGGL(k_a2c_apply, dim3(N), dim3(256), 0, stream, D, theta, vcrit, Ga, Gv, lr_a, lr_c, max_norm,
                     step, levels);
  TOUED_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
