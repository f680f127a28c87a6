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
// Latency structure: the agent's whole trajectory (obs rows and times, rewards, dones) is staged into LDS with
// coalesced loads, V(obs) gathered for every observation at once, and only then the per-worker GAE scans run
// out of LDS -- a handful of dependent memory round trips per update instead of two per time step.
__global__ void __launch_bounds__(256) k_a2c_grad(int W, int T, int D, const float* __restrict__ theta,
                                                  const float* __restrict__ vcrit, const int* __restrict__ tidx,
                                                  const int* __restrict__ ttime, const uint8_t* __restrict__ tact,
                                                  const float* __restrict__ trew, const uint8_t* __restrict__ tdone,
                                                  float gamma, float lam, float ent_coef, float* __restrict__ Ga,
                                                  float* __restrict__ Gv, float* __restrict__ loss_out) {
  extern __shared__ float lds[];
  const int NO = (T + 1) * W, NS = T * W;
  float* vt = lds;                                     // [T+1][W] V(obs)
  float* cc = vt + NO;                                 // [T+1][W] 0.001 * time
  int* ix = reinterpret_cast<int*>(cc + NO);           // [T+1][W] obs row
  float* rw = reinterpret_cast<float*>(ix + NO);       // [T][W] reward
  float* nd = rw + NS;                                 // [T][W] 1 - done
  float* adv = nd + NS;                                // [W*T] GAE advantages, worker-major
  float* dv = adv + NS;                                // [W*T] target - V
  float* abar = dv + NS;                               // [W] mean_t normalised advantage
  __shared__ float red[8];
  const int a = blockIdx.x;
  const int tid = threadIdx.x;
  const float* v = vcrit + (size_t)a * D;
  const float vlast = v[D - 1];
  const size_t tb = (size_t)a * (T + 1) * W;  // trajectory obs base
  const size_t sb = (size_t)a * T * W;        // trajectory step base
  // ---- stage the trajectory; V at every observation (all gathers in flight together)
  for (int i = tid; i < NO; i += blockDim.x) {
    const int idx = tidx[tb + i];
    const float c = (float)ttime[tb + i] * 0.001f;
    ix[i] = idx;
    cc[i] = c;
    vt[i] = v[idx] + c * vlast;
  }
  for (int i = tid; i < NS; i += blockDim.x) {
    rw[i] = trew[sb + i];
    nd[i] = tdone[sb + i] ? 0.0f : 1.0f;
  }
  __syncthreads();
  // ---- per-worker GAE (reverse scan over T, util/metrics.py:17-38)
  float s_adv = 0.0f, s_cl = 0.0f;
  for (int w = tid; w < W; w += blockDim.x) {
    float vn = vt[T * W + w];
    float g = 0.0f, cl = 0.0f;
    for (int t = T - 1; t >= 0; --t) {
      const float vv = vt[t * W + w];
      const float ndt = nd[t * W + w];
      const float delta = rw[t * W + w] + (gamma * vn * ndt - vv);
      g = delta + gamma * lam * ndt * g;
      const float e = (g + vv) - vv;
      adv[w * T + t] = g;
      dv[w * T + t] = e;
      cl += e * e;
      s_adv += g;
      vn = vv;
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
    const int idx = ix[i];
    const float c = cc[i];
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

// Fused update (grad + apply) with the agent's gradient tables in LDS: the per-sample contributions land in
// LDS (ds_add_f32 atomics: rows shared by many samples -- the start cell, small grids -- serialise far less
// than L2 atomics on one cache line), the global norms come from LDS, and only rows with a nonzero gradient
// are rewritten in HBM (an untouched row's update theta + -(lr * 0) is the identity).  One block per agent;
// used when D * 6 floats plus the staged trajectory fit the LDS (all_* modes: D = 3201), else grad + apply.
__global__ void __launch_bounds__(256) k_a2c_update(int W, int T, int D, float* __restrict__ theta,
                                                    float* __restrict__ vcrit, const int* __restrict__ tidx,
                                                    const int* __restrict__ ttime, const uint8_t* __restrict__ tact,
                                                    const float* __restrict__ trew, const uint8_t* __restrict__ tdone,
                                                    float gamma, float lam, float ent_coef, float lr_a, float lr_c,
                                                    float max_norm, int* __restrict__ step,
                                                    const int* __restrict__ levels, float* __restrict__ loss_out) {
  extern __shared__ float lds[];
  const int NO = (T + 1) * W, NS = T * W;
  float* GA = lds;                                     // [D][5] actor gradient
  float* GV = GA + (size_t)D * 5;                      // [D] critic gradient
  float* vt = GV + D;                                  // [T+1][W] V(obs)
  float* cc = vt + NO;                                 // [T+1][W] 0.001 * time
  int* ix = reinterpret_cast<int*>(cc + NO);           // [T+1][W] obs row
  float* rw = reinterpret_cast<float*>(ix + NO);       // [T][W] reward
  float* nd = rw + NS;                                 // [T][W] 1 - done
  float* adv = nd + NS;                                // [W*T] worker-major
  float* dv = adv + NS;                                // [W*T] target - V
  float* abar = dv + NS;                               // [W]
  __shared__ float red[8];
  const int a = blockIdx.x;
  const int tid = threadIdx.x;
  float* v = vcrit + (size_t)a * D;
  float* th = theta + (size_t)a * D * 5;
  for (int i = tid; i < D * 6; i += blockDim.x) GA[i] = 0.0f;
  const float vlast = v[D - 1];
  const size_t tb = (size_t)a * (T + 1) * W;
  const size_t sb = (size_t)a * T * W;
  for (int i = tid; i < NO; i += blockDim.x) {
    const int idx = tidx[tb + i];
    const float c = (float)ttime[tb + i] * 0.001f;
    ix[i] = idx;
    cc[i] = c;
    vt[i] = v[idx] + c * vlast;
  }
  for (int i = tid; i < NS; i += blockDim.x) {
    rw[i] = trew[sb + i];
    nd[i] = tdone[sb + i] ? 0.0f : 1.0f;
  }
  __syncthreads();
  float s_adv = 0.0f, s_cl = 0.0f;
  for (int w = tid; w < W; w += blockDim.x) {
    float vn = vt[T * W + w];
    float g = 0.0f, cl = 0.0f;
    for (int t = T - 1; t >= 0; --t) {
      const float vv = vt[t * W + w];
      const float ndt = nd[t * W + w];
      const float delta = rw[t * W + w] + (gamma * vn * ndt - vv);
      g = delta + gamma * lam * ndt * g;
      const float e = (g + vv) - vv;
      adv[w * T + t] = g;
      dv[w * T + t] = e;
      cl += e * e;
      s_adv += g;
      vn = vv;
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
  float lastA[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) lastA[j] = th[(size_t)(D - 1) * 5 + j];
  const float inv_n = 1.0f / n;
  float accA[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f}, accV = 0.0f, s_al = 0.0f;
  for (int i = tid; i < W * T; i += blockDim.x) {
    const int t = i / W, w = i - t * W;
    const int idx = ix[i];
    const float c = cc[i];
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
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const float d = kap * rho * ((j == act ? 1.0f : 0.0f) - p[j]) + ke * p[j] * (gl[j] - pg);
      atomicAdd(&GA[idx * 5 + j], d);
      accA[j] += c * d;
    }
    const float dvv = -2.0f * dv[w * T + t] * inv_n;
    atomicAdd(&GV[idx], dvv);
    accV += c * dvv;
    s_al += -__logf(pa + EPSF) * ab - ent_coef * h;
  }
  float ra[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) ra[j] = block_sum(accA[j], red);
  const float rv = block_sum(accV, red);
  const float al = block_sum(s_al, red) * inv_n;
  if (tid == 0) {   // every sample's LDS atomic is complete (block_sum's barriers)
#pragma unroll
    for (int j = 0; j < 5; ++j) GA[(D - 1) * 5 + j] += ra[j];
    GV[D - 1] += rv;
    loss_out[a * 2 + 0] += al;
    loss_out[a * 2 + 1] += closs;
  }
  __syncthreads();
  // ---- clip_by_global_norm + SGD (models/optim.py:5-11), discarded past the lifetime (a2c.py:71-75)
  float sa = 0.0f, sc = 0.0f;
  for (int i = tid; i < D * 5; i += blockDim.x) sa += GA[i] * GA[i];
  for (int i = tid; i < D; i += blockDim.x) sc += GV[i] * GV[i];
  const float gna = sqrtf(block_sum(sa, red));
  const float gnc = sqrtf(block_sum(sc, red));
  const int st = step[a];
  const bool applied = (st + 1) <= levels[(size_t)a * LEVEL_WORDS + L_LIFETIME];
  const bool clip_a = !(gna < max_norm), clip_c = !(gnc < max_norm);
  if (applied) {
    for (int r = tid; r < D; r += blockDim.x) {
      float g[5];
      bool nz = false;
#pragma unroll
      for (int j = 0; j < 5; ++j) { g[j] = GA[r * 5 + j]; nz |= g[j] != 0.0f; }
      if (nz) {
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          const float gg = clip_a ? (g[j] / gna) * max_norm : g[j];
          th[(size_t)r * 5 + j] = th[(size_t)r * 5 + j] + (-(lr_a * gg));
        }
      }
      const float gv = GV[r];
      if (gv != 0.0f) {
        const float gg = clip_c ? (gv / gnc) * max_norm : gv;
        v[r] = v[r] + (-(lr_c * gg));
      }
    }
  }
  if (tid == 0) step[a] = applied ? st + 1 : st;
}

static size_t a2c_update_lds(int W, int T, int D) {
  return ((size_t)D * 6 + 3 * (size_t)(T + 1) * W + 4 * (size_t)W * T + W) * sizeof(float);
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
  const size_t lds = (size_t)(3 * (T + 1) * W + 4 * W * T + W) * sizeof(float);
  TOUED_REQUIRE(lds <= 64 * 1024, "toued_a2c_grad: W*T too large for LDS");
  if (N == 0) return 0;
  hipLaunchKernelGGL(k_a2c_grad, dim3(N), dim3(256), lds, stream, W, T, D, theta, vcrit, tidx, ttime, tact, trew,
                     tdone, gamma, lam, ent_coef, Ga, Gv, loss_out);
  TOUED_CHECK_LAUNCH();
  return 0;
}

// 1 when the fused A2C update fits the LDS for these sizes (else use toued_a2c_grad + toued_a2c_apply)
int toued_a2c_update_fits(int W, int T, int D) {
  return W > 0 && T > 0 && D > 1 && a2c_update_lds(W, T, D) <= 150 * 1024 ? 1 : 0;
}

int toued_a2c_update(int N, int W, int T, int D, float* theta, float* vcrit, const int* tidx, const int* ttime,
                     const uint8_t* tact, const float* trew, const uint8_t* tdone, float gamma, float lam,
                     float ent_coef, float lr_a, float lr_c, float max_norm, int* step, const int* levels,
                     float* loss_out, hipStream_t stream) {
  TOUED_REQUIRE(N >= 0 && W > 0 && T > 0 && D > 1, "toued_a2c_update: bad sizes");
  const size_t lds = a2c_update_lds(W, T, D);
  TOUED_REQUIRE(lds <= 150 * 1024, "toued_a2c_update: D=%d W=%d T=%d need %zu B of LDS (use grad + apply)", D, W, T,
                lds);
  if (N == 0) return 0;
  static bool attr_set = false;
  if (!attr_set) {
    TOUED_REQUIRE(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_a2c_update),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024) == hipSuccess,
                  "toued_a2c_update: cannot raise the dynamic LDS limit");
    attr_set = true;
  }
  hipLaunchKernelGGL(k_a2c_update, dim3(N), dim3(256), lds, stream, W, T, D, theta, vcrit, tidx, ttime, tact, trew,
                     tdone, gamma, lam, ent_coef, lr_a, lr_c, max_norm, step, levels, loss_out);
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
