// Linear-softmax agent maths for the LPG meta-gradient step — HIP for gfx950.
//
// Forward (per inner update k):   agents/lpg_agent.py:31-85, :88-140
//   k_lpg_inputs   LPG inputs x = [r, d, pi, e(y_t), e(y_tp1)(, step, lifetime)] (models/lpg.py:48-77)
//   k_agent_grad   d/dtheta of mean(log(pi)*pi_hat), d/dphi of a_y*mean(KL(y_t||y_hat)), metrics
//   k_agent_apply  optax clip_by_global_norm -> scale(lr) -> scale(-1); discard if step > lifetime
//   k_entropy      util/metrics.py:5-9 batch_rollout_entropy (and its gradient, backward mode)
//   k_eval_loss    meta/train.py:61-100: frozen value critic, GAE (util/metrics.py:17-38), normalised
//                  advantage, lpg_loss with the [T] x [T,1] broadcast, value_loss
// Reverse (explicit adjoint of jax.grad through the K clipped-SGD steps, meta/train.py:174):
//   k_lpgloss_grad d lpg_loss / d theta_K
//   k_clip_dot     <G_k, adjoint> per agent -> clip-VJP coefficients
//   k_hvp          Hessian-vector products of the actor/critic losses through the linear-softmax
//                  (row-gather) parameterisation + cotangents on pi_hat / y_hat (+ L2 regularisers)
//   k_embed_bwd    embedding-MLP parameter gradient from the GRU input cotangents
//   k_adam         optax scale_by_adam + scale(lr) + scale(-1)
//
// Sample index s = (a*T + t)*W + w (trajectory layout), GRU row r = a*W + w.
// A tabular observation (idx, t) contributes logits table[idx] + (0.001 t) * table[D-1].
#include <string.h>
#include <algorithm>
#include <type_traits>
#include "common.h"
#include "wave_dev.h"

#define EPSF 1e-8f
#define SORT_MAX_TW 2048                  // samples per agent the sorted row kernel holds

namespace {

TOUED_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// logits of a compact obs: W[idx] + c * W[D-1]
template <int K>
TOUED_DEV void probs_of(const float* __restrict__ tab, const float* __restrict__ last, int idx, float c, float* p) {
  float l[K];
  float m = -__builtin_inff();
#pragma unroll
  for (int j = 0; j < K; ++j) {
    l[j] = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(tab) + ((unsigned)idx * K + j) * 4u) + c * last[j];
    m = fmaxf(m, l[j]);
  }
  float s = 0.0f;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    p[j] = __expf(l[j] - m);
    s += p[j];
  }
  const float inv = 1.0f / s;
#pragma unroll
  for (int j = 0; j < K; ++j) p[j] *= inv;
}

// base[elem] with a 32-bit byte offset: a load (or store) off a uniform base pointer takes the scalar-base form
// (one offset register, no 64-bit address pair per table)
template <class T>
TOUED_DEV T ld32(const T* base, unsigned elem) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + elem * (unsigned)sizeof(T));
}
// element j of the row at byte offset rowb from base (j in the instruction's immediate offset)
TOUED_DEV float ldrow(const float* base, unsigned rowb, int j) {
  return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(base) + rowb + j * 4);
}
template <class T>
TOUED_DEV void st32(T* base, unsigned elem, T v) {
  *reinterpret_cast<T*>(reinterpret_cast<char*>(base) + elem * (unsigned)sizeof(T)) = v;
}

// Scatter a K-vector d into rows idx and D-1 (times c) of a dense per-agent table.
// UNIF: the whole wave shares one agent -> reduce the D-1 row contribution first.
template <int K, bool UNIF>
TOUED_DEV void scatter_rows(float* __restrict__ tab, int idx, int D, float c, const float* d) {
#pragma unroll
  for (int j = 0; j < K; ++j) atomicAdd(&tab[(size_t)idx * K + j], d[j]);
  if (UNIF) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const float v = wave_sum(c * d[j]);
      if (lane == 0) atomicAdd(&tab[(size_t)(D - 1) * K + j], v);
    }
  } else {
#pragma unroll
    for (int j = 0; j < K; ++j) atomicAdd(&tab[(size_t)(D - 1) * K + j], c * d[j]);
  }
}

template <bool UNIF>
TOUED_DEV void add_metric(float* met, int a, int slot, float v) {
  if (UNIF) {
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) atomicAdd(&met[a * 8 + slot], v);
  } else {
    atomicAdd(&met[a * 8 + slot], v);
  }
}

// gstat[a] = {|G_theta|, |G_phi|, applied}: applied = step + 1 <= lifetime (lpg_agent.py:71-82)
TOUED_DEV void grad_stats(int a, float na2, float nc2, const int* step, const int* levels, float* gstat) {
  gstat[a * 4 + 0] = sqrtf(na2);
  gstat[a * 4 + 1] = sqrtf(nc2);
  gstat[a * 4 + 2] = (step[a] + 1) <= levels[(size_t)a * LEVEL_WORDS + L_LIFETIME] ? 1.0f : 0.0f;
  gstat[a * 4 + 3] = 0.0f;
}

struct SampleRef {
  int a, t, w, r, idx, idx1, act, done;
  float c, c1, rew;
};

TOUED_DEV SampleRef load_sample(long s, int T, int W, const int* __restrict__ tidx, const int* __restrict__ ttime,
                                const uint8_t* __restrict__ tact, const float* __restrict__ trew,
                                const uint8_t* __restrict__ tdone, bool uniform) {
  SampleRef q;
  const long at = s / W;
  q.w = (int)(s - at * W);
  q.a = (int)(at / T);
  q.t = (int)(at - (long)q.a * T);
  if (uniform) q.a = __builtin_amdgcn_readfirstlane(q.a);
  q.r = q.a * W + q.w;
  const size_t o0 = ((size_t)q.a * (T + 1) + q.t) * W + q.w;
  q.idx = tidx[o0];
  q.idx1 = tidx[o0 + W];
  q.c = (float)ttime[o0] * 0.001f;
  q.c1 = (float)ttime[o0 + W] * 0.001f;
  q.act = tact[s];
  q.rew = trew[s];
  q.done = tdone[s];
  return q;
}

// ---------------------------------------------------------------------------- keys
// Per agent key rng_a (already split(rng, N)[a]) -> the keys meta/train.py:88-170 consumes:
//   _rng = split(rng_a)[1] -> train_lpg_agent; inside: (t, roll_k) = split(t) for k < K
//   rng = split(rng_a)[0]; (rng, ev) = split(rng) -> eval rollout; (rng, ea) = split(rng) -> eval_agent
//   eval_agent(ea): (x, reset) = split(ea); (x, roll) = split(x)
__global__ void k_meta_keys(const uint32_t* __restrict__ agent_keys, int N, int K, uint32_t* __restrict__ roll_keys,
                            uint32_t* __restrict__ eval_keys, uint32_t* __restrict__ ea_reset,
                            uint32_t* __restrict__ ea_roll) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= N) return;
  uint2 rng = make_uint2(agent_keys[2 * a], agent_keys[2 * a + 1]);
  uint2 r0, tk;
  split2(rng, r0, tk);
  for (int k = 0; k < K; ++k) {
    uint2 rk;
    split2(tk, tk, rk);
    roll_keys[2 * ((size_t)k * N + a)] = rk.x;
    roll_keys[2 * ((size_t)k * N + a) + 1] = rk.y;
  }
  uint2 ev, ea;
  split2(r0, r0, ev);
  split2(r0, r0, ea);
  eval_keys[2 * a] = ev.x;
  eval_keys[2 * a + 1] = ev.y;
  uint2 x, rs, rr;
  split2(ea, x, rs);
  split2(x, x, rr);
  ea_reset[2 * a] = rs.x;
  ea_reset[2 * a + 1] = rs.y;
  ea_roll[2 * a] = rr.x;
  ea_roll[2 * a + 1] = rr.y;
}

// ---------------------------------------------------------------------------- LPG inputs
// X[f][t][r] (row stride xs_f between features) for one inner update.
template <bool UNIF, int F>
__global__ void __launch_bounds__(256) k_lpg_inputs(int N, int W, int T, int D, const float* __restrict__ theta,
                                                    const float* __restrict__ phi, const int* __restrict__ tidx,
                                                    const int* __restrict__ ttime, const uint8_t* __restrict__ tact,
                                                    const float* __restrict__ trew, const uint8_t* __restrict__ tdone,
                                                    const float* __restrict__ e1w, const float* __restrict__ e1b,
                                                    const float* __restrict__ e2w, const float* __restrict__ e2b,
                                                    const int* __restrict__ step, const int* __restrict__ levels,
                                                    float* __restrict__ X, long xs_f, long xs_col, long eta_stride) {
  const long s = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= (long)N * T * W) return;
  const SampleRef q = load_sample(s, T, W, tidx, ttime, tact, trew, tdone, UNIF);
  const int R = N * W;
  // per-agent LPG parameters (ES candidates) when eta_stride != 0
  e1w += q.a * eta_stride;
  e1b += q.a * eta_stride;
  e2w += q.a * eta_stride;
  e2b += q.a * eta_stride;
  const float* th = theta + (size_t)q.a * D * 5;
  const float* ph = phi + (size_t)q.a * D * 8;
  float lastA[5], lastC[8];
#pragma unroll
  for (int j = 0; j < 5; ++j) lastA[j] = th[(size_t)(D - 1) * 5 + j];
#pragma unroll
  for (int j = 0; j < 8; ++j) lastC[j] = ph[(size_t)(D - 1) * 8 + j];
  float p[5], y0[8], y1[8];
  probs_of<5>(th, lastA, q.idx, q.c, p);
  probs_of<8>(ph, lastC, q.idx, q.c, y0);
  probs_of<8>(ph, lastC, q.idx1, q.c1, y1);
  float pa = 0.0f;
#pragma unroll
  for (int j = 0; j < 5; ++j) pa = (j == q.act) ? p[j] + EPSF : pa;
  // embedding MLP [16, 1] (models/common.py:6-18) on y_t and y_tp1
  float e0 = e2b[0], e1 = e2b[0];
#pragma unroll
  for (int h = 0; h < 16; ++h) {
    float h0 = e1b[h], h1 = e1b[h];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      h0 += y0[i] * e1w[i * 16 + h];
      h1 += y1[i] * e1w[i * 16 + h];
    }
    e0 += fmaxf(h0, 0.0f) * e2w[h];
    e1 += fmaxf(h1, 0.0f) * e2w[h];
  }
  if (q.done) e1 = 0.0f;
  const size_t o = ((size_t)q.t * R + q.r) * xs_col;
  X[0 * xs_f + o] = q.rew;
  X[1 * xs_f + o] = q.done ? 1.0f : 0.0f;
  X[2 * xs_f + o] = pa;
  X[3 * xs_f + o] = e0;
  X[4 * xs_f + o] = e1;
  if (F == 7) {
    X[5 * xs_f + o] = (float)step[q.a];
    X[6 * xs_f + o] = (float)levels[(size_t)q.a * LEVEL_WORDS + L_LIFETIME];
  }
}

// The same inputs with one thread per GRU row (agent a, worker w) walking its T steps: the embedding of y_{t+1}
// (critic probabilities at the next observation) is the next step's embedding of y_t -- the same inputs, so the same
// bits -- so each step gathers one critic row instead of two and evaluates the embedding MLP once instead of twice;
// the next step's index loads and row gathers are issued before this step's arithmetic.  Bit-identical to
// k_lpg_inputs (tests/test_gpu_meta.py::test_lpg_inputs_rows_bitexact).
template <int F>
__global__ void __launch_bounds__(64) k_lpg_inputs_rows(int N, int W, int T, int D, const float* __restrict__ theta,
                                                        const float* __restrict__ phi, const int* __restrict__ tidx,
                                                        const int* __restrict__ ttime, const uint8_t* __restrict__ tact,
                                                        const float* __restrict__ trew,
                                                        const uint8_t* __restrict__ tdone,
                                                        const float* __restrict__ e1w, const float* __restrict__ e1b,
                                                        const float* __restrict__ e2w, const float* __restrict__ e2b,
                                                        const int* __restrict__ step, const int* __restrict__ levels,
                                                        float* __restrict__ X, long xs_f, long xs_col,
                                                        long eta_stride) {
  const int r = blockIdx.x * 64 + threadIdx.x;   // W % 64 == 0: the block's 64 rows belong to one agent
  if (r >= N * W) return;
  const int a = __builtin_amdgcn_readfirstlane(r / W);
  const int w = r - a * W;
  const int R = N * W;
  e1w += a * eta_stride;
  e1b += a * eta_stride;
  e2w += a * eta_stride;
  e2b += a * eta_stride;
  const float* th = theta + (size_t)a * D * 5;
  const float* ph = phi + (size_t)a * D * 8;
  float lastA[5], lastC[8];
#pragma unroll
  for (int j = 0; j < 5; ++j) lastA[j] = th[(size_t)(D - 1) * 5 + j];
#pragma unroll
  for (int j = 0; j < 8; ++j) lastC[j] = ph[(size_t)(D - 1) * 8 + j];
  auto emb = [&](const float (&y)[8]) {   // embedding MLP [16, 1] (models/common.py:6-18), k_lpg_inputs' order
    float e = e2b[0];
#pragma unroll
    for (int h = 0; h < 16; ++h) {
      float hh = e1b[h];
#pragma unroll
      for (int i = 0; i < 8; ++i) hh += y[i] * e1w[i * 16 + h];
      e += fmaxf(hh, 0.0f) * e2w[h];
    }
    return e;
  };
  float fstep = 0.0f, flife = 0.0f;
  if (F == 7) {
    fstep = (float)step[a];
    flife = (float)levels[(size_t)a * LEVEL_WORDS + L_LIFETIME];
  }
  const size_t ob = (size_t)a * (T + 1) * W + w;   // obs slot t at ob + t * W
  const size_t sb = (size_t)a * T * W + w;         // step slot t at sb + t * W
  int idx0 = tidx[ob];
  float c0 = (float)ttime[ob] * 0.001f;
  float e0;
  {
    float y0[8];
    probs_of<8>(ph, lastC, idx0, c0, y0);
    e0 = emb(y0);
  }
  int idx1 = tidx[ob + W];
  float c1 = (float)ttime[ob + W] * 0.001f;
  for (int t = 0; t < T; ++t) {
    const size_t s = sb + (size_t)t * W;
    const int act = tact[s];
    const float rew = trew[s];
    const int done = tdone[s];
    // next step's observation (slot t + 2, clamped) loaded ahead
    const int tn = t + 2 <= T ? t + 2 : T;
    const int idx2 = tidx[ob + (size_t)tn * W];
    const float c2 = (float)ttime[ob + (size_t)tn * W] * 0.001f;
    float p[5], y1[8];
    probs_of<5>(th, lastA, idx0, c0, p);
    probs_of<8>(ph, lastC, idx1, c1, y1);
    float pa = 0.0f;
#pragma unroll
    for (int j = 0; j < 5; ++j) pa = (j == act) ? p[j] + EPSF : pa;
    const float e1 = emb(y1);
    const size_t o = ((size_t)t * R + r) * xs_col;
    X[0 * xs_f + o] = rew;
    X[1 * xs_f + o] = done ? 1.0f : 0.0f;
    X[2 * xs_f + o] = pa;
    X[3 * xs_f + o] = e0;
    X[4 * xs_f + o] = done ? 0.0f : e1;
    if (F == 7) {
      X[5 * xs_f + o] = fstep;
      X[6 * xs_f + o] = flife;
    }
    e0 = e1;
    idx0 = idx1;
    c0 = c1;
    idx1 = idx2;
    c1 = c2;
  }
}

// ---------------------------------------------------------------------------- agent gradient
// met slots: 0 kl_sum, 1 pihat^2 sum, 2 sum_j yhat^2 sum, 3 actor entropy sum, 4 critic entropy sum
template <bool UNIF>
__global__ void __launch_bounds__(256) k_agent_grad(int N, int W, int T, int D, const float* __restrict__ theta,
                                                    const float* __restrict__ phi, const int* __restrict__ tidx,
                                                    const int* __restrict__ ttime, const uint8_t* __restrict__ tact,
                                                    const float* __restrict__ trew, const uint8_t* __restrict__ tdone,
                                                    const float* __restrict__ pi_hat, const float* __restrict__ y_hat,
                                                    float alpha_y, float* __restrict__ Gth, float* __restrict__ Gph,
                                                    float* __restrict__ met) {
  const long s = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= (long)N * T * W) return;
  const SampleRef q = load_sample(s, T, W, tidx, ttime, tact, trew, tdone, UNIF);
  const int R = N * W;
  const float inv_wt = 1.0f / (float)(W * T);
  const float* th = theta + (size_t)q.a * D * 5;
  const float* ph = phi + (size_t)q.a * D * 8;
  float lastA[5], lastC[8];
#pragma unroll
  for (int j = 0; j < 5; ++j) lastA[j] = th[(size_t)(D - 1) * 5 + j];
#pragma unroll
  for (int j = 0; j < 8; ++j) lastC[j] = ph[(size_t)(D - 1) * 8 + j];
  float p[5], y[8], yh[8];
  probs_of<5>(th, lastA, q.idx, q.c, p);
  probs_of<8>(ph, lastC, q.idx, q.c, y);
  const size_t o = (size_t)q.t * R + q.r;
  const float pih = pi_hat[o];
#pragma unroll
  for (int j = 0; j < 8; ++j) yh[j] = y_hat[((size_t)q.t * 8 + j) * R + q.r];
  // actor: d/dl [mean(log(pi_a + eps) * pi_hat)]
  float pa = 0.0f;
#pragma unroll
  for (int j = 0; j < 5; ++j) pa = (j == q.act) ? p[j] : pa;
  const float rho = pa / (pa + EPSF);
  float qa[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) qa[j] = pih * inv_wt * rho * ((j == q.act ? 1.0f : 0.0f) - p[j]);
  // critic: d/dm [a_y * mean KL(y || y_hat)]
  float av[8], ya = 0.0f, kl = 0.0f, y2 = 0.0f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float ly = __logf(y[j] + EPSF), lq = __logf(yh[j] + EPSF);
    kl += y[j] * (ly - lq);
    av[j] = ly - lq + y[j] / (y[j] + EPSF);
    ya += y[j] * av[j];
    y2 += yh[j] * yh[j];
  }
  float qc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) qc[j] = alpha_y * inv_wt * y[j] * (av[j] - ya);
  scatter_rows<5, UNIF>(Gth + (size_t)q.a * D * 5, q.idx, D, q.c, qa);
  scatter_rows<8, UNIF>(Gph + (size_t)q.a * D * 8, q.idx, D, q.c, qc);
  add_metric<UNIF>(met, q.a, 0, kl);
  add_metric<UNIF>(met, q.a, 1, pih * pih);
  add_metric<UNIF>(met, q.a, 2, y2);
}

// ---------------------------------------------------------------------------- apply (clipped SGD)
// Norms for the atomic gradient path (the sorted path computes them in the gradient kernel): one block per
// agent, gstat[a] = {|G_theta|, |G_phi|, applied}.
__global__ void __launch_bounds__(256) k_agent_norms(int N, int D, const float* __restrict__ Gth,
                                                     const float* __restrict__ Gph, const int* __restrict__ step,
                                                     const int* __restrict__ levels, float* __restrict__ gstat) {
  const int a = blockIdx.x;
  __shared__ float red[2][4];
  const size_t na = (size_t)D * 5, nc = (size_t)D * 8;
  const float* ga = Gth + (size_t)a * na;
  const float* gc = Gph + (size_t)a * nc;
  float sa = 0.0f, sc = 0.0f;
  for (size_t i = threadIdx.x; i < na; i += blockDim.x) sa += ga[i] * ga[i];
  for (size_t i = threadIdx.x; i < nc; i += blockDim.x) sc += gc[i] * gc[i];
  sa = wave_sum(sa);
  sc = wave_sum(sc);
  if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = sa; red[1][threadIdx.x >> 6] = sc; }
  __syncthreads();
  if (threadIdx.x == 0)
    grad_stats(a, red[0][0] + red[0][1] + red[0][2] + red[0][3], red[1][0] + red[1][1] + red[1][2] + red[1][3], step,
               levels, gstat);
}

// th1 = applied ? th0 - lr * clip(G) : th0 over both tables (a streaming pass: the norms and the lifetime
// test already sit in gstat).  Grid (chunk, agent, table): the agent's clip scale and learning rate are
// block-uniform, the table is walked in 16-byte vectors when its rows allow it (no per-element index
// division).  The first block of an agent's actor table advances its step.
// CLIP: 0 = not applied (copy), 1 = applied unclipped, 2 = applied and clipped (the per-element division
// optax's clip_by_global_norm performs, kept for bit parity, only on this block-uniform path)
template <int CLIP>
TOUED_DEV float apply_one(float p0, float g0, float gn, float max_norm, float lr) {
  if (CLIP == 0) return p0;
  const float g = CLIP == 2 ? (g0 / gn) * max_norm : g0;
  return p0 + (-(lr * g));
}

template <int CLIP>
TOUED_DEV void apply_seg(const float* __restrict__ P0, const float* __restrict__ G, float* __restrict__ P1, long per,
                         long head, float gn, float max_norm, float lr) {
  const long stride = (long)gridDim.x * blockDim.x;
  const long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long nv = (per - head) / 4;
  const float4* p4 = reinterpret_cast<const float4*>(P0 + head);
  const float4* g4 = reinterpret_cast<const float4*>(G + head);
  float4* o4 = reinterpret_cast<float4*>(P1 + head);
  for (long i = i0; i < nv; i += stride) {
    const float4 p = p4[i], g = g4[i];
    o4[i] = make_float4(apply_one<CLIP>(p.x, g.x, gn, max_norm, lr), apply_one<CLIP>(p.y, g.y, gn, max_norm, lr),
                        apply_one<CLIP>(p.z, g.z, gn, max_norm, lr), apply_one<CLIP>(p.w, g.w, gn, max_norm, lr));
  }
  for (long i = i0; i < head; i += stride) P1[i] = apply_one<CLIP>(P0[i], G[i], gn, max_norm, lr);
  for (long i = head + 4 * nv + i0; i < per; i += stride) P1[i] = apply_one<CLIP>(P0[i], G[i], gn, max_norm, lr);
}

__global__ void __launch_bounds__(256) k_agent_apply(int N, int D, const float* __restrict__ th0,
                                                     const float* __restrict__ ph0, const float* __restrict__ Gth,
                                                     const float* __restrict__ Gph, float lr_a, float lr_c,
                                                     float max_norm, int* __restrict__ step,
                                                     float* __restrict__ th1, float* __restrict__ ph1,
                                                     const float* __restrict__ gstat, int vec4) {
  const int a = blockIdx.y;
  const bool actor = blockIdx.z == 0;
  const long per = actor ? (long)D * 5 : (long)D * 8;
  const float* P0 = (actor ? th0 : ph0) + (long)a * per;
  const float* G = (actor ? Gth : Gph) + (long)a * per;
  float* P1 = (actor ? th1 : ph1) + (long)a * per;
  const float gn = gstat[a * 4 + (actor ? 0 : 1)];
  const bool applied = gstat[a * 4 + 2] > 0.5f;
  const float lr = actor ? lr_a : lr_c;
  if (actor && blockIdx.x == 0 && threadIdx.x == 0 && applied) step[a] += 1;
  // the three arrays are 16-byte aligned at their starts (vec4): the agent's segment has a scalar head up to
  // the next 16-byte boundary, a float4 body and a scalar tail
  const long head = vec4 ? std::min(per, (4 - ((long)a * per) % 4) % 4) : per;
  if (!applied) apply_seg<0>(P0, G, P1, per, head, gn, max_norm, lr);
  else if (gn < max_norm) apply_seg<1>(P0, G, P1, per, head, gn, max_norm, lr);
  else apply_seg<2>(P0, G, P1, per, head, gn, max_norm, lr);
}

// ---------------------------------------------------------------------------- entropy
// Forward: met[a][3|4] += sample entropies.  Backward (coef != 0): scatter coef * inv_wt * dH/dlogits.
template <bool UNIF>
__global__ void __launch_bounds__(256) k_entropy(int N, int W, int T, int D, const float* __restrict__ theta,
                                                 const float* __restrict__ phi, const int* __restrict__ tidx,
                                                 const int* __restrict__ ttime, float* __restrict__ met,
                                                 float coef_a, float coef_c, float* __restrict__ adj_th,
                                                 float* __restrict__ adj_ph) {
  const long s = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= (long)N * T * W) return;
  const long at = s / W;
  const int w = (int)(s - at * W);
  int a = (int)(at / T);
  const int t = (int)(at - (long)a * T);
  if (UNIF) a = __builtin_amdgcn_readfirstlane(a);
  const size_t o0 = ((size_t)a * (T + 1) + t) * W + w;
  const int idx = tidx[o0];
  const float c = (float)ttime[o0] * 0.001f;
  const float* th = theta + (size_t)a * D * 5;
  const float* ph = phi + (size_t)a * D * 8;
  float lastA[5], lastC[8];
#pragma unroll
  for (int j = 0; j < 5; ++j) lastA[j] = th[(size_t)(D - 1) * 5 + j];
#pragma unroll
  for (int j = 0; j < 8; ++j) lastC[j] = ph[(size_t)(D - 1) * 8 + j];
  float p[5], y[8];
  probs_of<5>(th, lastA, idx, c, p);
  probs_of<8>(ph, lastC, idx, c, y);
  float ha = 0.0f, hc = 0.0f, ga[5], gc[8];
#pragma unroll
  for (int j = 0; j < 5; ++j) { const float l = __logf(p[j] + EPSF); ha -= (p[j] + EPSF) * l; ga[j] = -(l + 1.0f); }
#pragma unroll
  for (int j = 0; j < 8; ++j) { const float l = __logf(y[j] + EPSF); hc -= (y[j] + EPSF) * l; gc[j] = -(l + 1.0f); }
  if (met) {
    add_metric<UNIF>(met, a, 3, ha);
    add_metric<UNIF>(met, a, 4, hc);
  }
  if (adj_th) {
    const float inv_wt = 1.0f / (float)(W * T);
    float pg = 0.0f, yg = 0.0f;
#pragma unroll
    for (int j = 0; j < 5; ++j) pg += p[j] * ga[j];
#pragma unroll
    for (int j = 0; j < 8; ++j) yg += y[j] * gc[j];
    float da[5], dc[8];
#pragma unroll
    for (int j = 0; j < 5; ++j) da[j] = coef_a * inv_wt * p[j] * (ga[j] - pg);
#pragma unroll
    for (int j = 0; j < 8; ++j) dc[j] = coef_c * inv_wt * y[j] * (gc[j] - yg);
    scatter_rows<5, UNIF>(adj_th + (size_t)a * D * 5, idx, D, c, da);
    scatter_rows<8, UNIF>(adj_ph + (size_t)a * D * 8, idx, D, c, dc);
  }
}

// Metric mode of the entropies (train_lpg_agent's batch_rollout_entropy, lpg_agent.py:119-120): one block per
// agent, fixed summation order (per-thread strided partials, then a block reduction), one writer per metric.
// The body for agent a on threads 0..255 of the calling block (every thread of the block calls it: one barrier); red
// is 8 floats of LDS.  Shared with toued_agent_step_entropy's k_rows_sorted<GradStepEntOp>, so both sum the same
// partials in the same order (bit-identical).
TOUED_DEV void entropy_metric_agent(int a, int tid, int W, int T, int D, const float* __restrict__ theta,
                                    const float* __restrict__ phi, const int* __restrict__ tidx,
                                    const int* __restrict__ ttime, float* __restrict__ met, float (*red)[4]) {
  if (tid < 256) {
    const float* th = theta + (size_t)a * D * 5;
    const float* ph = phi + (size_t)a * D * 8;
    float lastA[5], lastC[8];
#pragma unroll
    for (int j = 0; j < 5; ++j) lastA[j] = th[(size_t)(D - 1) * 5 + j];
#pragma unroll
    for (int j = 0; j < 8; ++j) lastC[j] = ph[(size_t)(D - 1) * 8 + j];
    float ha = 0.0f, hc = 0.0f;
    for (int i = tid; i < T * W; i += 256) {
      const int t = i / W, w = i - t * W;
      const size_t o0 = ((size_t)a * (T + 1) + t) * W + w;
      const int idx = tidx[o0];
      const float c = (float)ttime[o0] * 0.001f;
      float p[5], y[8];
      probs_of<5>(th, lastA, idx, c, p);
      probs_of<8>(ph, lastC, idx, c, y);
#pragma unroll
      for (int j = 0; j < 5; ++j) ha -= (p[j] + EPSF) * __logf(p[j] + EPSF);
#pragma unroll
      for (int j = 0; j < 8; ++j) hc -= (y[j] + EPSF) * __logf(y[j] + EPSF);
    }
    ha = wave_sum(ha);
    hc = wave_sum(hc);
    if ((tid & 63) == 0) { red[0][tid >> 6] = ha; red[1][tid >> 6] = hc; }
  }
  __syncthreads();
  if (tid == 0) {
    met[a * 8 + 3] += (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    met[a * 8 + 4] += (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  }
}

// entropy_metric_agent for a 512-thread block with T*W * 13 floats of LDS (`terms`): all 512 threads compute the
// samples' 13 entropy terms (p + eps) log(p + eps) into LDS, then the same 256 threads as entropy_metric_agent
// subtract them in the same order -- the same values and sums, with half the dependent gathers per thread
TOUED_DEV void entropy_metric_block(int a, int tid, int W, int T, int D, const float* __restrict__ theta,
                                    const float* __restrict__ phi, const int* __restrict__ tidx,
                                    const int* __restrict__ ttime, float* __restrict__ met, float (*red)[4],
                                    float* terms) {
  const int TW = T * W;
  {
    const float* th = theta + (size_t)a * D * 5;
    const float* ph = phi + (size_t)a * D * 8;
    float lastA[5], lastC[8];
#pragma unroll
    for (int j = 0; j < 5; ++j) lastA[j] = th[(size_t)(D - 1) * 5 + j];
#pragma unroll
    for (int j = 0; j < 8; ++j) lastC[j] = ph[(size_t)(D - 1) * 8 + j];
    const int* ti = tidx + (size_t)a * (T + 1) * W;   // sample i = t W + w
    const int* tt = ttime + (size_t)a * (T + 1) * W;
    // the thread's (at most four: T W <= 2048) samples' indices first, then their row gathers: two dependent trips
    int ix[4];
    float cx[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = tid + 512 * q;
      ix[q] = i < TW ? ld32(ti, (unsigned)i) : 0;
      cx[q] = i < TW ? (float)ld32(tt, (unsigned)i) * 0.001f : 0.0f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = tid + 512 * q;
      if (i < TW) {
        float p[5], y[8];
        probs_of<5>(th, lastA, ix[q], cx[q], p);
        probs_of<8>(ph, lastC, ix[q], cx[q], y);
        float* e = terms + (size_t)i * 13;
#pragma unroll
        for (int j = 0; j < 5; ++j) e[j] = (p[j] + EPSF) * __logf(p[j] + EPSF);
#pragma unroll
        for (int j = 0; j < 8; ++j) e[5 + j] = (y[j] + EPSF) * __logf(y[j] + EPSF);
      }
    }
  }
  __syncthreads();
  if (tid < 256) {
    float ha = 0.0f, hc = 0.0f;
    for (int i = tid; i < TW; i += 256) {
      const float* e = terms + (size_t)i * 13;
#pragma unroll
      for (int j = 0; j < 5; ++j) ha -= e[j];
#pragma unroll
      for (int j = 0; j < 8; ++j) hc -= e[5 + j];
    }
    ha = wave_sum(ha);
    hc = wave_sum(hc);
    if ((tid & 63) == 0) { red[0][tid >> 6] = ha; red[1][tid >> 6] = hc; }
  }
  __syncthreads();
  if (tid == 0) {
    met[a * 8 + 3] += (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    met[a * 8 + 4] += (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  }
}

__global__ void __launch_bounds__(256) k_entropy_metric(int W, int T, int D, const float* __restrict__ theta,
                                                        const float* __restrict__ phi, const int* __restrict__ tidx,
                                                        const int* __restrict__ ttime, float* __restrict__ met) {
  __shared__ float red[2][4];
  entropy_metric_agent(blockIdx.x, threadIdx.x, W, T, D, theta, phi, tidx, ttime, met, red);
}

// ---------------------------------------------------------------------------- eval loss
// One block (64 threads) per agent; eval trajectory (T steps).  Outputs per agent:
// out[a] = {lpg_loss, value_loss}; abar[a*W + w] = mean_t normalised advantage.
__global__ void __launch_bounds__(64) k_eval_loss(int N, int W, int T, int D, const float* __restrict__ theta,
                                                  const float* __restrict__ vcrit, const int* __restrict__ tidx,
                                                  const int* __restrict__ ttime, const uint8_t* __restrict__ tact,
                                                  const float* __restrict__ trew, const uint8_t* __restrict__ tdone,
                                                  float gamma, float lam, float* __restrict__ adv_scratch,
                                                  float* __restrict__ abar, float* __restrict__ out) {
  const int a = blockIdx.x;
  const int lane = threadIdx.x;
  const float* v = vcrit + (size_t)a * D;
  const float vlast = v[D - 1];
  const float* th = theta + (size_t)a * D * 5;
  float lastA[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) lastA[j] = th[(size_t)(D - 1) * 5 + j];
  float* adv = adv_scratch + (size_t)a * W * T;
  float s_adv = 0.0f, s_vl = 0.0f;
  for (int w = lane; w < W; w += 64) {
    float vn = v[tidx[((size_t)a * (T + 1) + T) * W + w]] + ((float)ttime[((size_t)a * (T + 1) + T) * W + w] * 0.001f) * vlast;
    float g = 0.0f, vl = 0.0f;
    for (int t = T - 1; t >= 0; --t) {
      const size_t o0 = ((size_t)a * (T + 1) + t) * W + w;
      const size_t s = ((size_t)a * T + t) * W + w;
      const float vt = v[tidx[o0]] + ((float)ttime[o0] * 0.001f) * vlast;
      const float nd = tdone[s] ? 0.0f : 1.0f;
      const float delta = trew[s] + (gamma * vn * nd - vt);
      g = delta + gamma * lam * nd * g;
      adv[(size_t)w * T + t] = g;
      const float tg = g + vt;
      vl += (tg - vt) * (tg - vt);
      s_adv += g;
      vn = vt;
    }
    s_vl += vl / (float)T;
  }
  __shared__ float sh[4];
  s_adv = wave_sum(s_adv);
  s_vl = wave_sum(s_vl);
  const float n = (float)(W * T);
  const float mean = s_adv / n;
  __syncthreads();
  float s_var = 0.0f;
  for (int i = lane; i < W * T; i += 64) { const float d = adv[i] - mean; s_var += d * d; }
  s_var = wave_sum(s_var);
  const float stdv = sqrtf(s_var / n);
  float s_loss = 0.0f;
  for (int w = lane; w < W; w += 64) {
    float ab = 0.0f, lp = 0.0f;
    for (int t = 0; t < T; ++t) {
      ab += (adv[(size_t)w * T + t] - mean) / (stdv + EPSF);
      const size_t o0 = ((size_t)a * (T + 1) + t) * W + w;
      const size_t s = ((size_t)a * T + t) * W + w;
      float p[5];
      probs_of<5>(th, lastA, tidx[o0], (float)ttime[o0] * 0.001f, p);
      float pa = p[0];
#pragma unroll
      for (int j = 1; j < 5; ++j) pa = (j == tact[s]) ? p[j] : pa;
      lp += __logf(pa + EPSF);
    }
    ab /= (float)T;
    lp /= (float)T;
    abar[(size_t)a * W + w] = ab;
    s_loss += -(lp * ab);
  }
  s_loss = wave_sum(s_loss);
  if (lane == 0) {
    out[a * 2 + 0] = s_loss / (float)W;
    out[a * 2 + 1] = s_vl / (float)W;
  }
  (void)sh;
}

// ---------------------------------------------------------------------------- d lpg_loss / d theta_K
template <bool UNIF>
__global__ void __launch_bounds__(256) k_lpgloss_grad(int N, int W, int T, int D, const float* __restrict__ theta,
                                                      const int* __restrict__ tidx, const int* __restrict__ ttime,
                                                      const uint8_t* __restrict__ tact, const float* __restrict__ abar,
                                                      float* __restrict__ adj_th) {
  const long s = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= (long)N * T * W) return;
  const long at = s / W;
  const int w = (int)(s - at * W);
  int a = (int)(at / T);
  const int t = (int)(at - (long)a * T);
  if (UNIF) a = __builtin_amdgcn_readfirstlane(a);
  const size_t o0 = ((size_t)a * (T + 1) + t) * W + w;
  const int idx = tidx[o0];
  const float c = (float)ttime[o0] * 0.001f;
  const float* th = theta + (size_t)a * D * 5;
  float lastA[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) lastA[j] = th[(size_t)(D - 1) * 5 + j];
  float p[5];
  probs_of<5>(th, lastA, idx, c, p);
  const int act = tact[s];
  float pa = 0.0f;
#pragma unroll
  for (int j = 0; j < 5; ++j) pa = (j == act) ? p[j] : pa;
  const float rho = pa / (pa + EPSF);
  const float kappa = -abar[(size_t)a * W + w] / (float)(W * T);
  float d[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) d[j] = kappa * rho * ((j == act ? 1.0f : 0.0f) - p[j]);
  scatter_rows<5, UNIF>(adj_th + (size_t)a * D * 5, idx, D, c, d);
}

// ---------------------------------------------------------------------------- clip VJP coefficients
// coef[a] = {alpha_a, beta_a, alpha_c, beta_c}: gbar = alpha*u + beta*G with u = -lr * adjoint.
// <G, adjoint> per table in 16-byte vectors when the tables allow it (vec4), two independent partials per
// thread and table so four vector loads are in flight per thread.
TOUED_DEV float dot4(float4 x, float4 y) { return x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w; }

// the clip VJP coefficients of agent a from sa = <G_theta, adj_theta>, sc = <G_phi, adj_phi> (optax
// clip_by_global_norm: g * max_norm / |g| when |g| >= max_norm)
TOUED_DEV void clip_coef(int a, float sa, float sc, const float* gstat, float lr_a, float lr_c, float max_norm,
                         float* coef) {
  const float gna = gstat[a * 4 + 0], gnc = gstat[a * 4 + 1];
  const bool applied = gstat[a * 4 + 2] > 0.5f;
  float aa = 0.0f, ba = 0.0f, ac = 0.0f, bc = 0.0f;
  if (applied) {
    if (gna < max_norm) { aa = 1.0f; }
    else { aa = max_norm / gna; ba = -max_norm * (-lr_a * sa) / (gna * gna * gna); }
    if (gnc < max_norm) { ac = 1.0f; }
    else { ac = max_norm / gnc; bc = -max_norm * (-lr_c * sc) / (gnc * gnc * gnc); }
  }
  coef[a * 4 + 0] = aa;
  coef[a * 4 + 1] = ba;
  coef[a * 4 + 2] = ac;
  coef[a * 4 + 3] = bc;
}

__global__ void __launch_bounds__(1024) k_clip_dot(int N, int D, const float* __restrict__ Gth,
                                                   const float* __restrict__ Gph, const float* __restrict__ adj_th,
                                                   const float* __restrict__ adj_ph, const float* __restrict__ gstat,
                                                   float lr_a, float lr_c, float max_norm, float* __restrict__ coef,
                                                   int vec4) {
  const int a = blockIdx.x;
  __shared__ float red[2][16];
  const long na = (long)D * 5, nc = (long)D * 8;
  const float* ga = Gth + (long)a * na;
  const float* ja = adj_th + (long)a * na;
  const float* gc = Gph + (long)a * nc;
  const float* jc = adj_ph + (long)a * nc;
  float da[4] = {0.0f, 0.0f, 0.0f, 0.0f}, dc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  if (vec4) {
    // the tables start 16-byte aligned: a scalar head to the agent's first 16-byte boundary, a float4 body,
    // a scalar tail
    auto seg = [&](const float* g, const float* j, long n, long off, float* acc) {
      const long head = std::min(n, (4 - off % 4) % 4), nv = (n - head) / 4;
      const float4 *g4 = reinterpret_cast<const float4*>(g + head), *j4 = reinterpret_cast<const float4*>(j + head);
      for (long i = threadIdx.x; i < nv; i += 2 * 1024) {
        acc[0] += dot4(g4[i], j4[i]);
        if (i + 1024 < nv) acc[1] += dot4(g4[i + 1024], j4[i + 1024]);
      }
      // the (at most 3 + 3) scalar elements, one per thread
      const long t = threadIdx.x < head ? threadIdx.x : head + 4 * nv + (threadIdx.x - head);
      if (t < n) acc[2] += g[t] * j[t];
    };
    seg(ga, ja, na, (long)a * na, da);
    seg(gc, jc, nc, (long)a * nc, dc);
  } else {
    for (long i = threadIdx.x; i < na; i += 4 * 1024) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long e = i + u * 1024;
        if (e < na) da[u] += ga[e] * ja[e];
      }
    }
    for (long i = threadIdx.x; i < nc; i += 4 * 1024) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long e = i + u * 1024;
        if (e < nc) dc[u] += gc[e] * jc[e];
      }
    }
  }
  float sa_ = wave_sum((da[0] + da[1]) + (da[2] + da[3]));
  float sc_ = wave_sum((dc[0] + dc[1]) + (dc[2] + dc[3]));
  if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = sa_; red[1][threadIdx.x >> 6] = sc_; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float sa = 0.0f, sc = 0.0f;
    for (int i = 0; i < 16; ++i) { sa += red[0][i]; sc += red[1][i]; }
    clip_coef(a, sa, sc, gstat, lr_a, lr_c, max_norm, coef);
  }
}

// ---------------------------------------------------------------------------- meta-step metrics
// The per-agent metrics of a meta-step (meta/train.py:101-117) in one launch: m = met * inv_wt averaged over the K
// updates (sum in update order, then divided by K, as jnp.mean's sum / n), and reg = lpg_loss - b0 H_pi + b2 |pi|^2 - b1 H_y +
// b3 |y|^2 evaluated left to right.  out rows: reg, policy_l2, policy_entropy, critic_loss, critic_l2, critic_entropy.
__global__ void k_meta_metrics(int N, int K, const float* __restrict__ met, float inv_wt,
                               const float* __restrict__ loss_out, float pec, float pl2, float tec, float tl2,
                               float* __restrict__ out) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= N) return;
  float m[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    float acc = 0.0f;
    for (int k = 0; k < K; ++k) acc = __fadd_rn(acc, __fmul_rn(met[((size_t)k * N + a) * 8 + j], inv_wt));
    m[j] = __fdiv_rn(acc, (float)K);
  }
  float reg = __fsub_rn(loss_out[a * 2], __fmul_rn(pec, m[3]));
  reg = __fadd_rn(reg, __fmul_rn(pl2, m[1]));
  reg = __fsub_rn(reg, __fmul_rn(tec, m[4]));
  reg = __fadd_rn(reg, __fmul_rn(tl2, m[2]));
  out[a] = reg;
  out[1 * N + a] = m[1];
  out[2 * N + a] = m[3];
  out[3 * N + a] = m[0];
  out[4 * N + a] = m[2];
  out[5 * N + a] = m[4];
}

// ---------------------------------------------------------------------------- HVP + LPG-output cotangents
template <bool UNIF>
__global__ void __launch_bounds__(256) k_hvp(int N, int W, int T, int D, int K, const float* __restrict__ theta,
                                             const float* __restrict__ phi, const int* __restrict__ tidx,
                                             const int* __restrict__ ttime, const uint8_t* __restrict__ tact,
                                             const float* __restrict__ pi_hat, const float* __restrict__ y_hat,
                                             const float* __restrict__ Gth, const float* __restrict__ Gph,
                                             const float* __restrict__ adj_th_in, const float* __restrict__ adj_ph_in,
                                             const float* __restrict__ coef, float lr_a, float lr_c, float alpha_y,
                                             float b2, float b3, float* __restrict__ adj_th_out,
                                             float* __restrict__ adj_ph_out, float* __restrict__ d_pi_hat,
                                             float* __restrict__ d_y_hat) {
  const long s = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= (long)N * T * W) return;
  const long at = s / W;
  const int w = (int)(s - at * W);
  int a = (int)(at / T);
  const int t = (int)(at - (long)a * T);
  if (UNIF) a = __builtin_amdgcn_readfirstlane(a);
  const int R = N * W, r = a * W + w;
  const float inv_wt = 1.0f / (float)(W * T);
  const size_t o0 = ((size_t)a * (T + 1) + t) * W + w;
  const int idx = tidx[o0];
  const float c = (float)ttime[o0] * 0.001f;
  const int act = tact[s];
  const size_t o = (size_t)t * R + r;
  const float pih = pi_hat[o];
  float yh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) yh[j] = y_hat[((size_t)t * 8 + j) * R + r];
  // regularisers beta_2 * mean(pi_hat^2), beta_3 * mean(sum y_hat^2), each averaged over K updates
  float dpih = (b2 / (float)K) * 2.0f * pih * inv_wt;
  float dyh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) dyh[j] = (b3 / (float)K) * 2.0f * yh[j] * inv_wt;
  const float aa = coef[a * 4 + 0], ba = coef[a * 4 + 1], ac = coef[a * 4 + 2], bc = coef[a * 4 + 3];
  if (aa != 0.0f) {   // update k was applied
    const size_t baseA = (size_t)a * D * 5, baseC = (size_t)a * D * 8;
    const float* th = theta + baseA;
    const float* ph = phi + baseC;
    float lastA[5], lastC[8];
#pragma unroll
    for (int j = 0; j < 5; ++j) lastA[j] = th[(size_t)(D - 1) * 5 + j];
#pragma unroll
    for (int j = 0; j < 8; ++j) lastC[j] = ph[(size_t)(D - 1) * 8 + j];
    float p[5], y[8];
    probs_of<5>(th, lastA, idx, c, p);
    probs_of<8>(ph, lastC, idx, c, y);
    // ---- actor
    float v[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const float adj = adj_th_in[baseA + (size_t)idx * 5 + j] + c * adj_th_in[baseA + (size_t)(D - 1) * 5 + j];
      const float g = Gth[baseA + (size_t)idx * 5 + j] + c * Gth[baseA + (size_t)(D - 1) * 5 + j];
      v[j] = -lr_a * aa * adj + ba * g;
    }
    float pa = 0.0f, va = 0.0f, pv = 0.0f;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      pa = (j == act) ? p[j] : pa;
      va = (j == act) ? v[j] : va;
      pv += p[j] * v[j];
    }
    const float rho = pa / (pa + EPSF);
    dpih += inv_wt * rho * (va - pv);
    const float ws = pih * inv_wt;
    const float drs = EPSF * pa / ((pa + EPSF) * (pa + EPSF));
    float da[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const float drho = drs * ((k == act ? 1.0f : 0.0f) - p[k]);
      da[k] = ws * (drho * (va - pv) - rho * p[k] * (v[k] - pv));
    }
    scatter_rows<5, UNIF>(adj_th_out + baseA, idx, D, c, da);
    // ---- critic
    float vc[8], av[8], ay = 0.0f, yv = 0.0f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float adj = adj_ph_in[baseC + (size_t)idx * 8 + j] + c * adj_ph_in[baseC + (size_t)(D - 1) * 8 + j];
      const float g = Gph[baseC + (size_t)idx * 8 + j] + c * Gph[baseC + (size_t)(D - 1) * 8 + j];
      vc[j] = -lr_c * ac * adj + bc * g;
      av[j] = __logf(y[j] + EPSF) - __logf(yh[j] + EPSF) + y[j] / (y[j] + EPSF);
      ay += av[j] * y[j];
      yv += y[j] * vc[j];
    }
    const float scale = alpha_y * inv_wt;
    float sv[8], ys = 0.0f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float b = vc[j] - yv;
      dyh[j] += scale * (-y[j] * b / (yh[j] + EPSF));
      const float ye = y[j] + EPSF;
      const float adash = 1.0f / ye + EPSF / (ye * ye);
      sv[j] = y[j] * b * adash + av[j] * b - vc[j] * ay;
      ys += y[j] * sv[j];
    }
    float dc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) dc[j] = scale * y[j] * (sv[j] - ys);
    scatter_rows<8, UNIF>(adj_ph_out + baseC, idx, D, c, dc);
  }
  d_pi_hat[o] = dpih;
#pragma unroll
  for (int j = 0; j < 8; ++j) d_y_hat[((size_t)t * 8 + j) * R + r] = dyh[j];
}

// ---------------------------------------------------------------------------- embedding MLP backward
#ifndef EMBED_V
#define EMBED_V 3   // k_embed_bwd3 (one lane per sample, e1_w / e1_b on the matrix cores); 1: k_embed_bwd
#endif
#ifndef EMBED_WPE
#define EMBED_WPE 3   // k_embed_bwd3's waves per SIMD (its register budget: 512 / EMBED_WPE)
#endif
// grad layout (161 floats): e1_b[16], e1_w[8*16], e2_b[1], e2_w[16] (flat-eta order within MLP_0)
// Inputs: y_t / y_tp1 recomputed from phi_k; cotangents dX3 (pyt), dX4 (pyt1, masked by done).
// Four lanes per sample, each owning four of the 16 hidden units (41 accumulators per lane instead of 161:
// occupancy); the quad recomputes the sample's critic output y.  Lane sums are reduced over the 16 samples
// of a wave with cross-lane adds, then over the block; partial[block][161] in the flat layout below.
template <bool UNIF>
__global__ void __launch_bounds__(256) k_embed_bwd(int N, int W, int T, int D, int K, const float* __restrict__ phi_hist,
                                                   long phi_stride, int phi_slot0, const int* __restrict__ tidx_hist, long tidx_stride,
                                                   const int* __restrict__ ttime_hist, const uint8_t* __restrict__ tdone_hist,
                                                   long tstep_stride, const float* __restrict__ dX3,
                                                   const float* __restrict__ dX4, long dx_stride_k,
                                                   const float* __restrict__ e1w, const float* __restrict__ e1b,
                                                   const float* __restrict__ e2w, float* __restrict__ partial) {
  const int q = threadIdx.x & 3;                 // hidden units 4q .. 4q+3
  float w1[8][4], b1[4], w2[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    b1[u] = e1b[4 * q + u];
    w2[u] = e2w[4 * q + u];
#pragma unroll
    for (int i = 0; i < 8; ++i) w1[i][u] = e1w[i * 16 + 4 * q + u];
  }
  float aw[8][4], ab[4], a2[4], ac = 0.0f;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    ab[u] = 0.0f; a2[u] = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; ++i) aw[i][u] = 0.0f;
  }
  // sample indices fit 31 bits (checked by the launcher): 32-bit index maths, no 64-bit divisions
  const int NTW = N * T * W;
  const int total = K * NTW;
  const int R = N * W;
  const int nthr = gridDim.x * (blockDim.x >> 2);
  // a sample's loads that do not depend on its observation rows: issued one sample ahead (the clamped index keeps
  // the prefetch unconditional, so the wait counts stay per load)
  struct In {
    const float* ph;
    int ix[2];
    float cx[2], cg[2], lastC[8];
  };
  auto load_in = [&](int g) {
    In v;
    const int k = (unsigned)g / (unsigned)NTW;
    const int s = g - k * NTW;
    const int at = (unsigned)s / (unsigned)W;
    const int w = s - at * W;
    const int a = (unsigned)at / (unsigned)T;
    const int t = at - a * T;
    const int r = a * W + w;
    const int* tidx = tidx_hist + k * tidx_stride;
    const int* ttime = ttime_hist + k * tidx_stride;
    const uint8_t* tdone = tdone_hist + k * tstep_stride;
    const int slot = k + phi_slot0 > K ? k + phi_slot0 - (K + 1) : k + phi_slot0;   // ring of K + 1 slots
    v.ph = phi_hist + slot * phi_stride + (size_t)a * D * 8;
    const size_t o0 = ((size_t)a * (T + 1) + t) * W + w;
#pragma unroll
    for (int j = 0; j < 8; ++j) v.lastC[j] = v.ph[(size_t)(D - 1) * 8 + j];
    const size_t o = (size_t)k * dx_stride_k + (size_t)t * R + r;
    v.ix[0] = tidx[o0];
    v.ix[1] = tidx[o0 + W];
    v.cx[0] = (float)ttime[o0] * 0.001f;
    v.cx[1] = (float)ttime[o0 + W] * 0.001f;
    v.cg[0] = dX3[o];
    v.cg[1] = tdone[s] ? 0.0f : dX4[o];
    return v;
  };
  const int g0 = blockIdx.x * (blockDim.x >> 2) + (threadIdx.x >> 2);
  In nx = load_in(min(g0, total - 1));
  for (int g = g0; g < total; g += nthr) {
    const In cur = nx;
    nx = load_in(min(g + nthr, total - 1));
    const float* ph = cur.ph;
    const int (&ix)[2] = cur.ix;
    const float (&cx)[2] = cur.cx;
    const float (&cgs)[2] = cur.cg;
    const float (&lastC)[8] = cur.lastC;
    // both observations' row gathers issued before either is used (two independent chains per sample)
    float ys[2][8];
#pragma unroll
    for (int which = 0; which < 2; ++which) probs_of<8>(ph, lastC, ix[which], cx[which], ys[which]);
#pragma unroll
    for (int which = 0; which < 2; ++which) {
      const float cg = cgs[which];
      if (cg == 0.0f) continue;
      const float (&y)[8] = ys[which];
      if (q == 0) ac += cg;  // e2_b
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float pre = b1[u];
#pragma unroll
        for (int i = 0; i < 8; ++i) pre += y[i] * w1[i][u];
        const float hid = fmaxf(pre, 0.0f);
        a2[u] += hid * cg;                               // e2_w
        const float dh = pre > 0.0f ? w2[u] * cg : 0.0f;
        ab[u] += dh;                                     // e1_b
#pragma unroll
        for (int i = 0; i < 8; ++i) aw[i][u] += y[i] * dh;   // e1_w
      }
    }
  }
  // lanes with the same q: sum over the wave's 16 samples (xor 4, 8, 16, 32), then over the block's waves
  auto qsum = [](float v) {
#pragma unroll
    for (int o = 4; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
    return v;
  };
  __shared__ float red[4][161];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int h = 4 * q + u;
    const float vb = qsum(ab[u]), v2 = qsum(a2[u]);
    if (lane < 4) { red[wv][h] = vb; red[wv][145 + h] = v2; }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float vw = qsum(aw[i][u]);
      if (lane < 4) red[wv][16 + i * 16 + h] = vw;
    }
  }
  {
    const float vc = qsum(ac);
    if (lane == 0) red[wv][144] = vc;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 161; i += blockDim.x) {
    float v = 0.0f;
    for (int qq = 0; qq < (int)(blockDim.x >> 6); ++qq) v += red[qq][i];
    partial[(size_t)blockIdx.x * 161 + i] = v;
  }
}

// probs_of on a row already in registers (the same operations in the same order: bit-identical)
template <int K>
TOUED_DEV void probs_regs(const float* row, const float* last, float c, float* p) {
  float l[K];
  float m = -__builtin_inff();
#pragma unroll
  for (int j = 0; j < K; ++j) {
    l[j] = row[j] + c * last[j];
    m = fmaxf(m, l[j]);
  }
  float s = 0.0f;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    p[j] = __expf(l[j] - m);
    s += p[j];
  }
  const float inv = 1.0f / s;
#pragma unroll
  for (int j = 0; j < K; ++j) p[j] *= inv;
}

// The same gradient with one lane per sample and the e1_w / e1_b reduction on the matrix cores.  A wave takes 64
// consecutive samples per round (each load instruction covers 64 samples: 256 contiguous bytes of an index or
// cotangent array, where k_embed_bwd's quad-per-sample layout covered 16 and repeated the loads and the softmax in
// four lanes); a lane computes its sample's critic outputs y and, per observation, the 16 hidden units (e1_w / e1_b /
// e2_w broadcast from LDS: no per-lane weight registers), accumulates e2_w / e2_b itself, and writes the item's
// rows a = [y, 1] and d = dh (the hidden cotangents) to the wave's LDS tile; sixteen v_mfma_f32_16x16x4_f32 then add
// A^T D over the 64 items into a 16 x 16 accumulator (rows 0..7 e1_w, row 8 e1_b) -- 4 accumulator registers
// instead of 41 per lane, so the kernel runs at 6 waves per SIMD.  The next round's index / time / cotangent loads
// are issued before this round's maths.  f32 products and sums, in another order than k_embed_bwd.
template <bool UNIF>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(EMBED_WPE))) k_embed_bwd3(int N, int W, int T, int D, int K, const float* __restrict__ phi_hist,
                                                    long phi_stride, int phi_slot0, const int* __restrict__ tidx_hist, long tidx_stride,
                                                    const int* __restrict__ ttime_hist, const uint8_t* __restrict__ tdone_hist,
                                                    long tstep_stride, const float* __restrict__ dX3,
                                                    const float* __restrict__ dX4, long dx_stride_k,
                                                    const float* __restrict__ e1w, const float* __restrict__ e1b,
                                                    const float* __restrict__ e2w, float* __restrict__ partial) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __shared__ float4 sw1[8][4];                   // e1_w [8][16] as float4 rows of four units
  __shared__ float4 sb1[4], sw2[4];              // e1_b, e2_w
  __shared__ float4 tA[4][64][3];                // per wave: item rows [y0..y7, 1, 0, 0, 0] (12 floats)
  __shared__ float4 tD[4][64][4];                // per wave: item rows dh[16]
  __shared__ float red[4][161];
  if (threadIdx.x < 32) sw1[threadIdx.x >> 2][threadIdx.x & 3] = reinterpret_cast<const float4*>(e1w)[threadIdx.x];
  if (threadIdx.x < 4) {
    sb1[threadIdx.x] = reinterpret_cast<const float4*>(e1b)[threadIdx.x];
    sw2[threadIdx.x] = reinterpret_cast<const float4*>(e2w)[threadIdx.x];
  }
  __syncthreads();
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  float a2[16], ac = 0.0f;
#pragma unroll
  for (int u = 0; u < 16; ++u) a2[u] = 0.0f;
  const int NTW = N * T * W;
  const int total = K * NTW;
  const int R = N * W;
  const int stride = gridDim.x * blockDim.x;     // samples per round of the grid
  struct In {
    const float* ph;
    int ix[2];
    float cx[2], cg[2];
  };
  auto load_in = [&](int g) {
    In v;
    const bool live = g < total;
    g = live ? g : total - 1;
    const int k = (unsigned)g / (unsigned)NTW;
    const int s = g - k * NTW;
    const int at = (unsigned)s / (unsigned)W;
    const int w = s - at * W;
    const int a = (unsigned)at / (unsigned)T;
    const int t = at - a * T;
    const int r = a * W + w;
    const int* tidx = tidx_hist + k * tidx_stride;
    const int* ttime = ttime_hist + k * tidx_stride;
    const uint8_t* tdone = tdone_hist + k * tstep_stride;
    const int slot = k + phi_slot0 > K ? k + phi_slot0 - (K + 1) : k + phi_slot0;   // ring of K + 1 slots
    v.ph = phi_hist + slot * phi_stride + (size_t)a * D * 8;
    const size_t o0 = ((size_t)a * (T + 1) + t) * W + w;
    const size_t o = (size_t)k * dx_stride_k + (size_t)t * R + r;
    v.ix[0] = tidx[o0];
    v.ix[1] = tidx[o0 + W];
    v.cx[0] = (float)ttime[o0] * 0.001f;
    v.cx[1] = (float)ttime[o0 + W] * 0.001f;
    v.cg[0] = live ? dX3[o] : 0.0f;
    v.cg[1] = (!live || tdone[s]) ? 0.0f : dX4[o];
    return v;
  };
  float4 (*A)[3] = tA[wv];
  float4 (*Dt)[4] = tD[wv];
  const float* Af = reinterpret_cast<const float*>(A);
  const float* Df = reinterpret_cast<const float*>(Dt);
  // MFMA operands: lane l supplies A[m = l & 15][k = l >> 4] and B[k][n = l & 15]; feature rows m >= 12 re-read row
  // 11's zero (their accumulator rows are not used)
  const int am = (lane & 15) < 12 ? (lane & 15) : 11, kq = lane >> 4, bn = lane & 15;
  const int g0 = blockIdx.x * blockDim.x + threadIdx.x;
  In nx = load_in(g0);
  for (int gb = g0 - lane; gb < total; gb += stride) {   // gb: the wave's first sample this round (wave-uniform)
    const In cur = nx;
    nx = load_in(gb + lane + stride);
    float last[8], row[2][8];
    {
      const float4* lp = reinterpret_cast<const float4*>(cur.ph + (size_t)(D - 1) * 8);
      const float4 l0 = lp[0], l1 = lp[1];
      last[0] = l0.x; last[1] = l0.y; last[2] = l0.z; last[3] = l0.w;
      last[4] = l1.x; last[5] = l1.y; last[6] = l1.z; last[7] = l1.w;
#pragma unroll
      for (int which = 0; which < 2; ++which) {
        const float4* rp = reinterpret_cast<const float4*>(cur.ph + (size_t)cur.ix[which] * 8);
        const float4 r0 = rp[0], r1 = rp[1];
        row[which][0] = r0.x; row[which][1] = r0.y; row[which][2] = r0.z; row[which][3] = r0.w;
        row[which][4] = r1.x; row[which][5] = r1.y; row[which][6] = r1.z; row[which][7] = r1.w;
      }
    }
#pragma unroll
    for (int which = 0; which < 2; ++which) {
      float y[8];
      probs_regs<8>(row[which], last, cur.cx[which], y);
      const float cg = cur.cg[which];
      ac += cg;                                          // e2_b
      // keep the weights in LDS (hoisted copies would take 160 registers per lane)
      __asm__ volatile("" ::: "memory");
      float dh[16];
#pragma unroll
      for (int uq = 0; uq < 4; ++uq) {
        const float4 bb = sb1[uq], ww = sw2[uq];
        float pre[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float4 wv4 = sw1[i][uq];
          pre[0] += y[i] * wv4.x;
          pre[1] += y[i] * wv4.y;
          pre[2] += y[i] * wv4.z;
          pre[3] += y[i] * wv4.w;
        }
        const float w2v[4] = {ww.x, ww.y, ww.z, ww.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          a2[4 * uq + u] += fmaxf(pre[u], 0.0f) * cg;     // e2_w
          dh[4 * uq + u] = pre[u] > 0.0f ? w2v[u] * cg : 0.0f;
        }
        __builtin_amdgcn_sched_barrier(0);   // one group's weights live at a time
      }
      A[lane][0] = make_float4(y[0], y[1], y[2], y[3]);
      A[lane][1] = make_float4(y[4], y[5], y[6], y[7]);
      A[lane][2] = make_float4(1.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
      for (int c = 0; c < 4; ++c) Dt[lane][c] = make_float4(dh[4 * c], dh[4 * c + 1], dh[4 * c + 2], dh[4 * c + 3]);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int kg = 0; kg < 16; ++kg) {
        const int it = 4 * kg + kq;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(Af[it * 12 + am], Df[it * 16 + bn], acc, 0, 0, 0);
        if ((kg & 3) == 3) __builtin_amdgcn_sched_barrier(0);   // operands of four products in flight at a time
      }
      // the tile's reads are in registers before the next item's writes (in-order LDS within the wave)
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_sched_barrier(0);   // one observation's values live at a time
    }
  }
  // accumulator: lane l holds C[m = 4 (l >> 4) + r][n = l & 15], r = 0..3 (m < 8: e1_w[m][n], m = 8: e1_b[n])
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = 4 * kq + r;
    if (m < 8) red[wv][16 + m * 16 + bn] = acc[r];
    else if (m == 8) red[wv][bn] = acc[r];
  }
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const float v = wsum_dpp(a2[u]);
    if (lane == 0) red[wv][145 + u] = v;
  }
  {
    const float v = wsum_dpp(ac);
    if (lane == 0) red[wv][144] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 161; i += blockDim.x) {
    float v = 0.0f;
    for (int qq = 0; qq < (int)(blockDim.x >> 6); ++qq) v += red[qq][i];
    partial[(size_t)blockIdx.x * 161 + i] = v;
  }
}

// ---------------------------------------------------------------------------- Adam
__global__ void __launch_bounds__(256) k_adam(int P, float* __restrict__ eta, const float* __restrict__ grad,
                                              float* __restrict__ m, float* __restrict__ v, float n_mean, float lr,
                                              float b1, float omb1, float b2, float omb2, float eps, float bc1,
                                              float bc2) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  // meta/train.py:128 x.mean(axis=0): the agent sum divided by the count
  const float g = grad[i] / n_mean;
  // optax 0.1.5 update_moment / update_moment_per_elem_norm: (1 - decay) * g + decay * t, with (1 - decay)
  // rounded once from the python float (omb1, omb2) and g**2 formed before the scale
  const float mi = omb1 * g + b1 * m[i];
  const float vi = omb2 * (g * g) + b2 * v[i];
  m[i] = mi;
  v[i] = vi;
  // bias_correction: t / (1 - decay**count); updates = mu_hat / (sqrt(nu_hat + 0) + eps); scale(lr); scale(-1)
  const float mh = mi / bc1, vh = vi / bc2;
  eta[i] = eta[i] + (-(lr * (mh / (sqrtf(vh) + eps))));
}

// ---------------------------------------------------------------------------- agent init
// agents/agents.py:31-95 create_agent / create_value_critic: bias-free Dense kernels with flax's
// lecun_normal (truncated normal in [-2, 2], stddev sqrt(1/fan_in)/0.87962566).  Here the kernel of
// table i is drawn from keys[i] directly (flax's per-module key derivation is not reproduced: parity
// unpinned).  u = uniform(lo=erf(-sqrt2), hi=erf(sqrt2)); z = sqrt2*erfinv(u), clipped.

__global__ void __launch_bounds__(256) k_init_tables(const uint32_t* __restrict__ keys, int n, int cols, int D,
                                                     float lo, float hi, float stddev, float* __restrict__ out,
                                                     const uint8_t* __restrict__ mask) {
  // grid (chunk, table i): no per-element index division; masked tables exit at once
  const int i = blockIdx.y;
  if (i >= n || (mask && !mask[i])) return;
  const long per = (long)D * cols;
  const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= per) return;
  const long e = (long)i * per + j;
  const uint2 key = make_uint2(keys[2 * i], keys[2 * i + 1]);
  const float u = uniform_from_bits(random_bits_at(key, (uint32_t)per, (uint32_t)j), lo, hi);
  float z = 1.41421356237f * erfinv_giles(u);
  z = fminf(fmaxf(z, -1.99999988f), 1.99999988f);
  out[e] = z * stddev;
}

// The masked form for the level sampler (few tables of many rewritten per call): one block per table looping over
// its D * cols elements, so the unmasked tables cost one exiting block each instead of ceil(D * cols / 256); the
// same element values as k_init_tables.
__global__ void __launch_bounds__(256) k_init_tables_blk(const uint32_t* __restrict__ keys, int n, int cols, int D,
                                                         float lo, float hi, float stddev, float* __restrict__ out,
                                                         const uint8_t* __restrict__ mask) {
  const int i = blockIdx.x;
  if (i >= n || !mask[i]) return;
  const long per = (long)D * cols;
  const uint2 key = make_uint2(keys[2 * i], keys[2 * i + 1]);
  for (long j = threadIdx.x; j < per; j += blockDim.x) {
    const float u = uniform_from_bits(random_bits_at(key, (uint32_t)per, (uint32_t)j), lo, hi);
    float z = 1.41421356237f * erfinv_giles(u);
    z = fminf(fmaxf(z, -1.99999988f), 1.99999988f);
    out[(long)i * per + j] = z * stddev;
  }
}

// out[dst[i]] += src[si[i]], every dst index distinct (one plain read-modify-write per element, as index_add_ with
// unique indices): the GRU weight-gradient blocks into eta's flat layout in one launch
__global__ void __launch_bounds__(256) k_gather_add(float* __restrict__ out, const float* __restrict__ src,
                                                    const int* __restrict__ si, const int* __restrict__ di, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[di[i]] += src[si[i]];
}

// out[j] += the sum over i < rows of part[i][j]: the embedding gradient's per-block partials.  One workgroup per column:
// thread t sums rows t, t + 256, ... (independent loads in flight), then a fixed-order tree over the 256 partial sums
// (deterministic).  (One thread per column walking the 768 rows serially took 0.18 ms of dependent loads.)
__global__ void __launch_bounds__(256) k_sum_rows_add(const float* __restrict__ part, int rows, int cols,
                                                      float* __restrict__ out) {
  __shared__ float sred[256];
  const int j = blockIdx.x, tid = threadIdx.x;
  float acc = 0.0f;
  for (int i = tid; i < rows; i += 256) acc += part[(size_t)i * cols + j];
  sred[tid] = acc;
  __syncthreads();
#pragma unroll
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) sred[tid] += sred[tid + o];
    __syncthreads();
  }
  if (tid == 0) out[j] += sred[0];
}

}  // namespace

// ============================================================================ C ABI
// ---------------------------------------------------------------------------- sorted per-agent row scatter
// The table gradients above scatter every sample's 5 + 8 row cotangents with float atomics (8.5M per call at
// N=512, W=64, T=20).  For T*W <= 2048 the kernels below instead give each agent one workgroup: the
// samples' row vectors go to LDS, their row indices are sorted (bitonic, key = row << 12 | sample), and one
// thread per distinct row sums its segment in sample order and adds it to the table with a plain
// read-modify-write (each row has exactly one writer in the grid).  Same sums, no atomics, and the result is
// deterministic.  The time row (D-1, every sample contributes c * v) is a block reduction added by its
// segment's owner (or thread 0).

struct GradOp {   // k_agent_grad (+ the global norms and the lifetime test of the update it feeds)
  static constexpr int NA = 5, NC = 8, NM = 3;
  static constexpr bool NORMS = true, APPLY = false, WRITE_G = false, CLIPDOT = false;
  const float* theta; const float* phi; const int* tidx; const int* ttime; const uint8_t* tact; const float* trew;
  const uint8_t* tdone; const float* pi_hat; const float* y_hat; float alpha_y; float* Gth; float* Gph; float* met;
  const int* step; const int* levels; float* gstat;
  int N, W, T, D;
  static constexpr int NLAST = 13;   // the time rows theta[D-1], phi[D-1]: the same for every sample of the agent
  TOUED_DEV float last_val(int a, int i) const {
    return i < 5 ? theta[((size_t)a * D + D - 1) * 5 + i] : phi[((size_t)a * D + D - 1) * 8 + (i - 5)];
  }
  TOUED_DEV bool sample(int a, int t, int w, int idx, float c, float* v, float* m, const float* lastv) const {
    const long s = ((long)a * T + t) * W + w;
    const int R = N * W;
    const int qr = a * W + w, qact = tact[s];
    const float inv_wt = 1.0f / (float)(W * T);
    const float* th = theta + (size_t)a * D * 5;
    const float* ph = phi + (size_t)a * D * 8;
    const float* lastA = lastv;
    const float* lastC = lastv + 5;
    float p[5], y[8], yh[8];
    probs_of<5>(th, lastA, idx, c, p);
    probs_of<8>(ph, lastC, idx, c, y);
    const size_t o = (size_t)t * R + qr;
    const float pih = pi_hat[o];
#pragma unroll
    for (int j = 0; j < 8; ++j) yh[j] = y_hat[((size_t)t * 8 + j) * R + qr];
    float pa = 0.0f;
#pragma unroll
    for (int j = 0; j < 5; ++j) pa = (j == qact) ? p[j] : pa;
    const float rho = pa / (pa + EPSF);
#pragma unroll
    for (int j = 0; j < 5; ++j) v[j] = pih * inv_wt * rho * ((j == qact ? 1.0f : 0.0f) - p[j]);
    float av[8], ya = 0.0f, kl = 0.0f, y2 = 0.0f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float ly = __logf(y[j] + EPSF), lq = __logf(yh[j] + EPSF);
      kl += y[j] * (ly - lq);
      av[j] = ly - lq + y[j] / (y[j] + EPSF);
      ya += y[j] * av[j];
      y2 += yh[j] * yh[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[5 + j] = alpha_y * inv_wt * y[j] * (av[j] - ya);
    m[0] = kl; m[1] = pih * pih; m[2] = y2;
    return true;
  }
  TOUED_DEV float* rowA(int a, int r) const { return Gth + ((size_t)a * D + r) * 5; }
  TOUED_DEV float* rowC(int a, int r) const { return Gph + ((size_t)a * D + r) * 8; }
  TOUED_DEV void metrics(int a, const float* m) const { for (int j = 0; j < NM; ++j) met[a * 8 + j] += m[j]; }
  TOUED_DEV void finish(int a, float na2, float nc2) const { grad_stats(a, na2, nc2, step, levels, gstat); }
};

// GradOp fused with apply_gradients for an agent chain that never reads the gradient tables (the ES candidates'
// train_lpg_agent): the segment sums stay in LDS, the global norms are reduced in the block, then clip + SGD rewrite
// the touched rows of theta/phi IN PLACE (an untouched row's update p + -(lr * 0) is the identity, so this is
// bit-identical to k_agent_grad into zeroed tables + k_agent_apply), the step counter advances and gstat is filled.
struct GradApplyOp : GradOp {
  static constexpr bool APPLY = true;
  float* theta_w; float* phi_w; float lr_a, lr_c, max_norm; int* step_w;
};

// The meta-gradient's inner update k (toued_agent_step): GradApplyOp reading theta_k / phi_k (GradOp::theta, phi)
// and rewriting the touched rows of theta_{k+1} / phi_{k+1} (theta_w, phi_w: copies of theta_k / phi_k made
// beforehand), and keeping the gradient rows it touched (Gth / Gph) for the reverse pass; rows never touched are left
// as they were (the reverse pass reads touched rows only: toued_entropy_clip, toued_hvp).
struct GradStepOp : GradApplyOp {
  static constexpr bool WRITE_G = true;
};

// toued_agent_step_entropy: GradStepOp, then the metric-mode entropies of the new policy (theta_{k+1} / phi_{k+1},
// toued_entropy with met) on the same block -- the rows they read are the rows the block just wrote (its samples'
// rows and the time row) or theta_k's copies, so one barrier orders them; one launch less per inner update.
struct GradStepEntOp : GradStepOp {
  static constexpr bool ENTROPY_AFTER = true;
};
// ops whose sample is register-heavy accumulate the time row's partial sums after the sample loop (HvpOp)
template <class Op, class = void>
struct defer_time_row : std::false_type {};
template <class Op>
struct defer_time_row<Op, std::void_t<decltype(Op::DEFER_TIME_ROW)>> : std::bool_constant<Op::DEFER_TIME_ROW> {};
template <class Op, class = void>
struct entropy_after : std::false_type {};
template <class Op>
struct entropy_after<Op, std::void_t<decltype(Op::ENTROPY_AFTER)>> : std::bool_constant<Op::ENTROPY_AFTER> {};

struct EntropyBwdOp {   // k_entropy, gradient mode
  static constexpr int NA = 5, NC = 8, NM = 1;
  static constexpr bool NORMS = false, APPLY = false, WRITE_G = false, CLIPDOT = false;
  const float* theta; const float* phi; const int* tidx; const int* ttime; float coef_a, coef_c;
  float* adj_th; float* adj_ph;
  int N, W, T, D;
  static constexpr int NLAST = 13;   // the time rows theta[D-1], phi[D-1]: the same for every sample of the agent
  TOUED_DEV float last_val(int a, int i) const {
    return i < 5 ? theta[((size_t)a * D + D - 1) * 5 + i] : phi[((size_t)a * D + D - 1) * 8 + (i - 5)];
  }
  TOUED_DEV bool sample(int a, int t, int w, int idx, float c, float* v, float* m, const float* lastv) const {
    const float* th = theta + (size_t)a * D * 5;
    const float* ph = phi + (size_t)a * D * 8;
    const float* lastA = lastv;
    const float* lastC = lastv + 5;
    float p[5], y[8];
    probs_of<5>(th, lastA, idx, c, p);
    probs_of<8>(ph, lastC, idx, c, y);
    float ga[5], gc[8];
#pragma unroll
    for (int j = 0; j < 5; ++j) ga[j] = -(__logf(p[j] + EPSF) + 1.0f);
#pragma unroll
    for (int j = 0; j < 8; ++j) gc[j] = -(__logf(y[j] + EPSF) + 1.0f);
    const float inv_wt = 1.0f / (float)(W * T);
    float pg = 0.0f, yg = 0.0f;
#pragma unroll
    for (int j = 0; j < 5; ++j) pg += p[j] * ga[j];
#pragma unroll
    for (int j = 0; j < 8; ++j) yg += y[j] * gc[j];
#pragma unroll
    for (int j = 0; j < 5; ++j) v[j] = coef_a * inv_wt * p[j] * (ga[j] - pg);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[5 + j] = coef_c * inv_wt * y[j] * (gc[j] - yg);
    m[0] = 0.0f;
    return true;
  }
  TOUED_DEV float* rowA(int a, int r) const { return adj_th + ((size_t)a * D + r) * 5; }
  TOUED_DEV float* rowC(int a, int r) const { return adj_ph + ((size_t)a * D + r) * 8; }
  TOUED_DEV void metrics(int, const float*) const {}
  TOUED_DEV void finish(int, float, float) const {}
};

// EntropyBwdOp of the reverse pass's step k fused with the clip-VJP dot that follows it: the rows it rewrites are
// exactly the rows update k touched (the same trajectory, plus the time row), so the thread owning a row adds
// <G_k[row], adjoint[row]> as it writes the row, and thread 0 turns the block's sums into coef (k_clip_dot's
// coefficients up to the summation order: the untouched rows, zero in the dense tables, are not visited)
struct EntropyClipOp : EntropyBwdOp {
  static constexpr bool CLIPDOT = true;
  const float* Gth; const float* Gph; const float* gstat; float lr_a, lr_c, max_norm; float* coef;
  TOUED_DEV float gA(int a, int r, int j) const { return Gth[((size_t)a * D + r) * 5 + j]; }
  TOUED_DEV float gC(int a, int r, int j) const { return Gph[((size_t)a * D + r) * 8 + j]; }
};

struct LpgLossOp {   // k_lpgloss_grad
  static constexpr int NA = 5, NC = 0, NM = 1;
  static constexpr bool NORMS = false, APPLY = false, WRITE_G = false, CLIPDOT = false;
  const float* theta; const int* tidx; const int* ttime; const uint8_t* tact; const float* abar; float* adj_th;
  int N, W, T, D;
  static constexpr int NLAST = 5;   // the time row theta[D-1]
  TOUED_DEV float last_val(int a, int i) const { return theta[((size_t)a * D + D - 1) * 5 + i]; }
  TOUED_DEV bool sample(int a, int t, int w, int idx, float c, float* v, float* m, const float* lastv) const {
    const long s = ((long)a * T + t) * W + w;
    const float* th = theta + (size_t)a * D * 5;
    const float* lastA = lastv;
    float p[5];
    probs_of<5>(th, lastA, idx, c, p);
    const int act = tact[s];
    float pa = 0.0f;
#pragma unroll
    for (int j = 0; j < 5; ++j) pa = (j == act) ? p[j] : pa;
    const float rho = pa / (pa + EPSF);
    const float kappa = -abar[(size_t)a * W + w] / (float)(W * T);
#pragma unroll
    for (int j = 0; j < 5; ++j) v[j] = kappa * rho * ((j == act ? 1.0f : 0.0f) - p[j]);
    m[0] = 0.0f;
    return true;
  }
  TOUED_DEV float* rowA(int a, int r) const { return adj_th + ((size_t)a * D + r) * 5; }
  TOUED_DEV float* rowC(int, int) const { return nullptr; }
  TOUED_DEV void metrics(int, const float*) const {}
  TOUED_DEV void finish(int, float, float) const {}
};

struct HvpOp {   // k_hvp
  static constexpr int NA = 5, NC = 8, NM = 0;   // (no metrics)
  static constexpr bool DEFER_TIME_ROW = true;
  static constexpr bool NORMS = false, APPLY = false, WRITE_G = false, CLIPDOT = false;
  const float* theta; const float* phi; const int* tidx; const int* ttime; const uint8_t* tact;
  const float* pi_hat; const float* y_hat; const float* Gth; const float* Gph; const float* adj_th_in;
  const float* adj_ph_in; const float* coef; float lr_a, lr_c, alpha_y, b2, b3;
  float* adj_th_out; float* adj_ph_out; float* d_pi_hat; float* d_y_hat;
  int N, W, T, D, K;
  // per-agent values every sample reads: theta[D-1] (0..4), phi[D-1] (5..12), adj_th_in[D-1] (13..17),
  // Gth[D-1] (18..22), adj_ph_in[D-1] (23..30), Gph[D-1] (31..38), coef[a] (39..42)
  static constexpr int NLAST = 43;
  TOUED_DEV float last_val(int a, int i) const {
    const size_t rA = ((size_t)a * D + D - 1) * 5, rC = ((size_t)a * D + D - 1) * 8;
    if (i < 5) return theta[rA + i];
    if (i < 13) return phi[rC + (i - 5)];
    if (i < 18) return adj_th_in[rA + (i - 13)];
    if (i < 23) return Gth[rA + (i - 18)];
    if (i < 31) return adj_ph_in[rC + (i - 23)];
    if (i < 39) return Gph[rC + (i - 31)];
    return coef[a * 4 + (i - 39)];
  }
  // The sample's loads go through per-agent base pointers (uniform in the block: scalar registers) plus 32-bit
  // element offsets, so every gather is a scalar-base load with one offset register per table shape instead of a
  // 64-bit address pair per table (toued_hvp / toued_entropy_clip_hvp check that the offsets fit)
  TOUED_DEV bool sample(int a, int t, int w, int idx, float c, float* vout, float* m, const float* lastv) const {
    const unsigned R = (unsigned)(N * W), tw = (unsigned)(t * W + w), tr = (unsigned)t * R + (unsigned)w;
    const float inv_wt = 1.0f / (float)(W * T);
    const size_t ow = (size_t)a * W;
    const int act = ld32(tact + (size_t)a * T * W, tw);
    const float pih = ld32(pi_hat + ow, tr);
    float dpih = (b2 / (float)K) * 2.0f * pih * inv_wt;
    const float aa = lastv[39], ba = lastv[40], ac = lastv[41], bc = lastv[42];
    const bool applied = aa != 0.0f;
    const size_t baseA = (size_t)a * D * 5, baseC = (size_t)a * D * 8;
    // two stages, each issuing its rows' loads together: the policy half (rows idx of theta, adj_th, G_th), then
    // the critic half (phi, adj_ph, G_ph rows and y_hat); fenced so the two halves' registers are never live at once
    if (applied) {
      const unsigned bA = (unsigned)idx * 20u;
      float thr[5], adA[5], gA[5];
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        thr[j] = ldrow(theta + baseA, bA, j);
        adA[j] = ldrow(adj_th_in + baseA, bA, j);
        gA[j] = ldrow(Gth + baseA, bA, j);
      }
      float p[5];
      probs_regs<5>(thr, lastv, c, p);
      float v[5];
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        const float adj = adA[j] + c * lastv[13 + j];
        const float g = gA[j] + c * lastv[18 + j];
        v[j] = -lr_a * aa * adj + ba * g;
      }
      float pa = 0.0f, va = 0.0f, pv = 0.0f;
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        pa = (j == act) ? p[j] : pa;
        va = (j == act) ? v[j] : va;
        pv += p[j] * v[j];
      }
      const float rho = pa / (pa + EPSF);
      dpih += inv_wt * rho * (va - pv);
      const float ws = pih * inv_wt;
      const float drs = EPSF * pa / ((pa + EPSF) * (pa + EPSF));
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const float drho = drs * ((k == act ? 1.0f : 0.0f) - p[k]);
        vout[k] = ws * (drho * (va - pv) - rho * p[k] * (v[k] - pv));
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    float yh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) yh[j] = ld32(y_hat + ow, (unsigned)(8 * t + j) * R + (unsigned)w);
    float dyh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) dyh[j] = (b3 / (float)K) * 2.0f * yh[j] * inv_wt;
    if (applied) {
      const unsigned bC = (unsigned)idx * 32u;
      float phr[8], adC[8], gC[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        phr[j] = ldrow(phi + baseC, bC, j);
        adC[j] = ldrow(adj_ph_in + baseC, bC, j);
        gC[j] = ldrow(Gph + baseC, bC, j);
      }
      float y[8];
      probs_regs<8>(phr, lastv + 5, c, y);
      float vc[8], av[8], ay = 0.0f, yv = 0.0f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float adj = adC[j] + c * lastv[23 + j];
        const float g = gC[j] + c * lastv[31 + j];
        vc[j] = -lr_c * ac * adj + bc * g;
        av[j] = __logf(y[j] + EPSF) - __logf(yh[j] + EPSF) + y[j] / (y[j] + EPSF);
        ay += av[j] * y[j];
        yv += y[j] * vc[j];
      }
      const float scale = alpha_y * inv_wt;
      float sv[8], ys = 0.0f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float b = vc[j] - yv;
        dyh[j] += scale * (-y[j] * b / (yh[j] + EPSF));
        const float ye = y[j] + EPSF;
        const float adash = 1.0f / ye + EPSF / (ye * ye);
        sv[j] = y[j] * b * adash + av[j] * b - vc[j] * ay;
        ys += y[j] * sv[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) vout[5 + j] = scale * y[j] * (sv[j] - ys);
    }
    st32(d_pi_hat + ow, tr, dpih);
#pragma unroll
    for (int j = 0; j < 8; ++j) st32(d_y_hat + ow, (unsigned)(8 * t + j) * R + (unsigned)w, dyh[j]);
    return applied;
  }
  TOUED_DEV float* rowA(int a, int r) const { return adj_th_out + ((size_t)a * D + r) * 5; }
  TOUED_DEV float* rowC(int a, int r) const { return adj_ph_out + ((size_t)a * D + r) * 8; }
  TOUED_DEV void metrics(int, const float*) const {}
  TOUED_DEV void finish(int, float, float) const {}
};

#ifndef ROWS_PRIO
#define ROWS_PRIO 3   // C2 20.29-20.31 ms at 0, 19.96-20.00 at 3 (profiles/r04/c2_rows_prio_r04j.txt)
#endif
// One agent's block (k_rows_sorted below).  PRESORTED: `key` already holds the block's sorted sample keys from an
// earlier body over the same samples (every sample kept by both ops, as EntropyClipOp and HvpOp do), so only the row
// vectors and partial sums are rebuilt and the sort is skipped.
#ifdef ROWS_STAMPS
// timing instrumentation (tools/rows_stamps.py, built by tools/build_variant.py agent.hip ROWS_STAMPS=1): thread 0 of
// blocks < 64 records the shader clock at 7 points of the body (slot 0 = k_rows_sorted's body, 1 and 2 =
// k_rows_sorted2's first and second); every block records the 100 MHz real-time clock at its body's start and end
// and its placement (XCC_ID, HW_ID); both per launch (a ring of 8 launches per slot).  The clock
// reads are volatile asm with their waits, so they stay between the phases they bracket.
__device__ unsigned long long g_rows_stamps[3 * 8 * 64 * 8];   // [slot][launch ring][block][stamp]
__device__ unsigned long long g_rows_span[3 * 8 * 1024 * 4];
__device__ unsigned g_rows_ctr[3];
TOUED_DEV unsigned long long rs_clock() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
  return t;
}
TOUED_DEV unsigned long long rs_rtc() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
  return t;
}
#define ROWS_STAMP(ph)                                                                                 \
  do {                                                                                                 \
    if (tid == 0) {                                                                                    \
      const unsigned long long tc = rs_clock(), tr = rs_rtc();                                         \
      if ((ph) == 0) rs_launch = (atomicAdd(&g_rows_ctr[SLOT], 1u) / gridDim.x) & 7u;                 \
      if (blockIdx.x < 64) g_rows_stamps[((SLOT * 8 + rs_launch) * 64 + blockIdx.x) * 8 + (ph)] = tc;  \
      if (blockIdx.x < 1024 && ((ph) == 0 || (ph) == 6)) {                                             \
        unsigned long long* e = g_rows_span + (((size_t)SLOT * 8 + rs_launch) * 1024 + blockIdx.x) * 4; \
        e[(ph) == 6] = tr;                                                                             \
        if ((ph) == 0) {                                                                               \
          e[2] = (unsigned)__builtin_amdgcn_s_getreg((3 << 11) | 20);                                  \
          e[3] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);                                  \
        }                                                                                              \
      }                                                                                                \
    }                                                                                                  \
  } while (0)
#else
#define ROWS_STAMP(ph) do {} while (0)
#endif
template <class Op, bool PRESORTED, int SLOT = 0>
TOUED_DEV void rows_sorted_body(const Op& op) {
  constexpr int NA = Op::NA, NC = Op::NC, NV = NA + NC, NM = Op::NM;
  constexpr uint32_t NONE = 0xFFFFFFFFu, SMASK = 4095u;
  // unpadded vector stride (odd strides are bank-conflict free): 13-float rows keep a block's LDS at 75 KB,
  // so two agents' blocks share a CU and all N = 512 blocks are resident in one round
  constexpr int NVP = NV;
  constexpr int CH = 4;                                 // sorted entries per thread
  extern __shared__ float lds[];
  __shared__ float red[8][NV + NM];
  __shared__ float tot[NV + NM];
  __shared__ int has_last;
  __shared__ int any_kept;   // PRESORTED: did this op keep any sample (HvpOp keeps none of an agent not updated)
  __shared__ int scan_a[8];
  __shared__ float scan_b[8][NV];
  __shared__ float lastv[Op::NLAST];   // the op's per-agent values (time rows ...), read once per block
  uint32_t* key = reinterpret_cast<uint32_t*>(lds);   // [2048]
  float* vec = lds + 2048;                            // [T*W][NVP]
  // (the thread index through an opaque move: two bodies in one kernel share no tid-derived addresses, which the
  // compiler would otherwise keep live from the first body into the second)
  int tid_l;
  asm volatile("v_mov_b32 %0, %1" : "=v"(tid_l) : "v"((int)threadIdx.x));
  const int a = blockIdx.x, tid = tid_l, W = op.W, T = op.T, D = op.D, TW = T * W;
  const int lane = tid & 63, wv = tid >> 6;
  constexpr bool DEFER = defer_time_row<Op>::value;
  // APPLY: the step counter and lifetime (the lifetime test below), loaded at the start, off the critical path
  int app_step = 0, app_life = 0;
  if constexpr (Op::APPLY) {
    app_step = op.step[a];
    app_life = op.levels[(size_t)a * LEVEL_WORDS + L_LIFETIME];
  }
  if (tid == 0) { has_last = 0; any_kept = 0; }
  if (tid < Op::NLAST) lastv[tid] = op.last_val(a, tid);
#ifdef ROWS_STAMPS
  unsigned rs_launch = 0;
#endif
  ROWS_STAMP(0);
  float part[NV + NM];
#pragma unroll
  for (int j = 0; j < NV + NM; ++j) part[j] = 0.0f;
  __syncthreads();
  // 1) per-sample row vectors -> LDS, sort keys, time-row and metric partial sums
  uint32_t kept = 0u;   // DEFER: the iterations whose sample was kept
  // every op's sample sl = t W + w is row tidx[a][t][w] at time c = ttime[a][t][w] / 1000 (the [N][T + 1][W] index
  // arrays): the body loads them, one iteration ahead, so a sample's row gathers do not wait behind its own index load
  // (only in the one-op kernel, SLOT 0, and not for HvpOp: with the two more live registers k_rows_sorted2's two
  // bodies and k_rows_sorted<HvpOp> spill)
  constexpr bool AHEAD = SLOT == 0 && !DEFER;
  int nidx = 0, ntt = 0;
  if (AHEAD && tid < TW) {
    nidx = ld32(op.tidx + (size_t)a * (T + 1) * W, (unsigned)tid);
    ntt = ld32(op.ttime + (size_t)a * (T + 1) * W, (unsigned)tid);
  }
  for (int sl = tid, it = 0; sl < 2048; sl += 512, ++it) {
    uint32_t kk = NONE;
    if (!AHEAD && sl < TW) {
      nidx = ld32(op.tidx + (size_t)a * (T + 1) * W, (unsigned)sl);
      ntt = ld32(op.ttime + (size_t)a * (T + 1) * W, (unsigned)sl);
    }
    const int idx = nidx, tcur = ntt;
    if (AHEAD && sl + 512 < TW) {
      nidx = ld32(op.tidx + (size_t)a * (T + 1) * W, (unsigned)(sl + 512));
      ntt = ld32(op.ttime + (size_t)a * (T + 1) * W, (unsigned)(sl + 512));
    }
    if (sl < TW) {
      const int t = sl / W, w = sl - t * W;
      const float c = (float)tcur * 0.001f;
      float v[NV], m[NM > 0 ? NM : 1];
      // (an opaque zero offset keeps the per-agent values' LDS reads in the iteration that uses them: hoisted out
      // of the loop they would hold up to 43 registers across it)
      int z0;
      asm volatile("s_mov_b32 %0, 0" : "=s"(z0));
      if (op.sample(a, t, w, idx, c, v, m, lastv + z0)) {
        kk = ((uint32_t)idx << 12) | (uint32_t)sl;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          vec[sl * NVP + j] = v[j];
          if constexpr (!DEFER) part[j] += c * v[j];
        }
        if constexpr (DEFER) kept |= 1u << it;
        if (idx == D - 1) has_last = 1;
        if (PRESORTED) any_kept = 1;
      } else if (PRESORTED) {
        // a sample the first op kept and this one drops: its slot in the shared sort adds zeros
#pragma unroll
        for (int j = 0; j < NV; ++j) vec[sl * NVP + j] = 0.0f;
      }
#pragma unroll
      for (int j = 0; j < NM; ++j) part[NV + j] += m[j];
    }
    if (!PRESORTED) key[sl] = kk;
  }
  if constexpr (DEFER) {
    // the time row's partial sums after the loop, from the stored row vectors: the same products in the same order,
    // with 13 fewer registers live across the sample loop
    const int* tt = op.ttime + (size_t)a * (T + 1) * W;   // c of sample sl = t W + w
    for (int sl = tid, it = 0; sl < TW; sl += 512, ++it) {
      if ((kept >> it) & 1u) {
        const float c = (float)ld32(tt, (unsigned)sl) * 0.001f;
#pragma unroll
        for (int j = 0; j < NV; ++j) part[j] += c * vec[sl * NVP + j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NV + NM; ++j) {
    const float r = wsum_dpp(part[j]);
    if (lane == 0) red[wv][j] = r;
  }
  __syncthreads();
  if (tid < NV + NM) {
    float r = 0.0f;
    for (int w = 0; w < 8; ++w) r += red[w][tid];
    tot[tid] = r;
  }
  ROWS_STAMP(1);
  // 2) sort by (row, sample)
  if constexpr (PRESORTED) __syncthreads();   // (tot and the row vectors before phase 3)
  else sort2048_reg<512>(key, tid);
  ROWS_STAMP(2);
  // 3) segmented row sums, deterministic (a fixed combination tree): thread t owns the sorted entries
  //    [CH t, CH t + CH) as runs of equal rows; the part of a segment in earlier chunks (the carry) reaches the chunk
  //    where the segment ends through a segmented scan over the 512 chunks (carry_t = a_t carry_{t-1} + b_t, b_t the
  //    sum of chunk t's last run, a_t = 1 iff chunk t is one run continuing chunk t-1's segment); the thread holding a
  //    segment's last entry adds the segment to the table row (each row has exactly one writer in the grid)
  auto rowof = [](uint32_t k) { return k == NONE ? NONE : (k >> 12); };
  uint32_t kc[CH];
  {
    const uint4 x = reinterpret_cast<const uint4*>(key)[tid];
    // PRESORTED with every sample dropped: the segments of a sort with no keys (exactly as a launch of its own)
    if (PRESORTED && !any_kept) {
      kc[0] = kc[1] = kc[2] = kc[3] = NONE;
    } else {
      kc[0] = x.x; kc[1] = x.y; kc[2] = x.z; kc[3] = x.w;
    }
  }
  const bool keys_live = !PRESORTED || any_kept;
  const uint32_t prow = tid == 0 || !keys_live ? NONE : rowof(key[CH * tid - 1]);
  const uint32_t nrow = tid == 511 || !keys_live ? NONE : rowof(key[CH * tid + CH]);
  uint32_t endm = 0u;
#pragma unroll
  for (int e = 0; e < CH; ++e) {
    const uint32_t r = rowof(kc[e]);
    const uint32_t rn = e < CH - 1 ? rowof(kc[e + 1]) : nrow;
    if (r != NONE && rn != r) endm |= 1u << e;
  }
  const uint32_t r0 = rowof(kc[0]);
  const bool cont0 = r0 != NONE && prow == r0;
  float sb[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) sb[j] = 0.0f;
  int sa = cont0 ? 1 : 0;
  {
    uint32_t lr = r0;
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      const uint32_t r = rowof(kc[e]);
      if (r != lr) {
        sa = 0;
        lr = r;
#pragma unroll
        for (int j = 0; j < NV; ++j) sb[j] = 0.0f;
      }
      if (r != NONE) {
        const float* ve = vec + (size_t)(kc[e] & SMASK) * NVP;
#pragma unroll
        for (int j = 0; j < NV; ++j) sb[j] += ve[j];
      }
    }
  }
#pragma unroll
  for (int dd = 1; dd < 64; dd <<= 1) {
    const int oa = __shfl_up(sa, dd, 64);
    float ob[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) ob[j] = __shfl_up(sb[j], dd, 64);
    if (lane >= dd && sa) {
#pragma unroll
      for (int j = 0; j < NV; ++j) sb[j] = ob[j] + sb[j];
      sa = oa;
    }
  }
  if (lane == 63) {
    scan_a[wv] = sa;
#pragma unroll
    for (int j = 0; j < NV; ++j) scan_b[wv][j] = sb[j];
  }
  __syncthreads();
  float pb[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) pb[j] = 0.0f;
  for (int w2 = 0; w2 < wv; ++w2) {
    const bool cont = w2 > 0 && scan_a[w2];
#pragma unroll
    for (int j = 0; j < NV; ++j) pb[j] = cont ? pb[j] + scan_b[w2][j] : scan_b[w2][j];
  }
  float run[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const float x = (wv > 0 && sa) ? pb[j] + sb[j] : sb[j];   // carry at the end of this chunk
    float cj = __shfl_up(x, 1, 64);
    if (lane == 0) cj = pb[j];
    run[j] = cont0 ? cj : 0.0f;
  }
  ROWS_STAMP(3);
  float na2 = 0.0f, nc2 = 0.0f;
  {
    uint32_t rr = r0;
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      const uint32_t r = rowof(kc[e]);
      if (r != NONE) {
        if (r != rr) {
          rr = r;
#pragma unroll
          for (int j = 0; j < NV; ++j) run[j] = 0.0f;
        }
        const float* ve = vec + (size_t)(kc[e] & SMASK) * NVP;
#pragma unroll
        for (int j = 0; j < NV; ++j) run[j] += ve[j];
        if ((endm >> e) & 1u) {
          if ((int)r == D - 1) {
#pragma unroll
            for (int j = 0; j < NV; ++j) run[j] += tot[j];
          }
          if constexpr (Op::APPLY) {   // the row's gradient (0 + sum, as a zeroed table would hold it) to LDS
            float* slot = vec + (size_t)(kc[e] & SMASK) * NVP;
            float* ga = nullptr;
            float* gc = nullptr;
            if constexpr (Op::WRITE_G) { ga = op.rowA(a, (int)r); gc = op.rowC(a, (int)r); }
#pragma unroll
            for (int j = 0; j < NV; ++j) {
              const float g = 0.0f + run[j];
              slot[j] = g;
              if constexpr (Op::WRITE_G) { if (j < NA) ga[j] = g; else gc[j - NA] = g; }
              if (j < NA) na2 += g * g; else nc2 += g * g;
            }
            continue;
          }
          float* ra = op.rowA(a, (int)r);
#pragma unroll
          for (int j = 0; j < NA; ++j) {
            const float g = ra[j] + run[j];
            ra[j] = g;
            if (Op::NORMS) na2 += g * g;
            if constexpr (Op::CLIPDOT) na2 += op.gA(a, (int)r, j) * g;
          }
          if (NC > 0) {
            float* rc = op.rowC(a, (int)r);
#pragma unroll
            for (int j = 0; j < NC; ++j) {
              const float g = rc[j] + run[NA + j];
              rc[j] = g;
              if (Op::NORMS) nc2 += g * g;
              if constexpr (Op::CLIPDOT) nc2 += op.gC(a, (int)r, j) * g;
            }
          }
        }
      }
    }
  }
  ROWS_STAMP(4);
  // APPLY: the theta_k / phi_k rows this thread will rewrite (its segments' rows; thread 0 also the time row when no
  // segment holds it), loaded here so that they arrive during the norm reduction instead of after it
  float srcv[Op::APPLY ? CH + 1 : 1][Op::APPLY ? NV : 1];
  if constexpr (Op::APPLY) {
    auto load_row = [&](size_t r, float* dst) {
#pragma unroll
      for (int j = 0; j < NA; ++j) dst[j] = op.theta[((size_t)a * D + r) * NA + j];
#pragma unroll
      for (int j = 0; j < NC; ++j) dst[NA + j] = op.phi[((size_t)a * D + r) * NC + j];
    };
#pragma unroll
    for (int e = 0; e < CH; ++e)
      if ((endm >> e) & 1u) load_row(kc[e] >> 12, srcv[e]);
    if (tid == 0 && !has_last) load_row((size_t)(D - 1), srcv[CH]);
  }
  // APPLY: the step counter and lifetime test before any thread writes them
  bool applied = false;
  if constexpr (Op::APPLY) applied = app_step + 1 <= app_life;
  if (Op::APPLY && tid == 0 && !has_last) {
    float* ga = nullptr;
    float* gc = nullptr;
    if constexpr (Op::WRITE_G) { ga = op.rowA(a, D - 1); gc = op.rowC(a, D - 1); }
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const float g = 0.0f + tot[j];
      if constexpr (Op::WRITE_G) { if (j < NA) ga[j] = g; else gc[j - NA] = g; }
      if (j < NA) na2 += g * g; else nc2 += g * g;
    }
  }
  if (!Op::APPLY && tid == 0) {
    if (!has_last) {
      float* ra = op.rowA(a, D - 1);
#pragma unroll
      for (int j = 0; j < NA; ++j) {
        const float g = ra[j] + tot[j];
        ra[j] = g;
        if (Op::NORMS) na2 += g * g;
        if constexpr (Op::CLIPDOT) na2 += op.gA(a, D - 1, j) * g;
      }
      if (NC > 0) {
        float* rc = op.rowC(a, D - 1);
#pragma unroll
        for (int j = 0; j < NC; ++j) {
          const float g = rc[j] + tot[NA + j];
          rc[j] = g;
          if (Op::NORMS) nc2 += g * g;
          if constexpr (Op::CLIPDOT) nc2 += op.gC(a, D - 1, j) * g;
        }
      }
    }
    op.metrics(a, tot + NV);
  }
  if constexpr (Op::CLIPDOT) {   // <G_k, adjoint> of the block -> the clip-VJP coefficients
    na2 = wsum_dpp(na2);
    nc2 = wsum_dpp(nc2);
    __syncthreads();
    if (lane == 0) { red[wv][0] = na2; red[wv][1] = nc2; }
    __syncthreads();
    if (tid == 0) {
      float x = 0.0f, y = 0.0f;
      for (int w = 0; w < 8; ++w) { x += red[w][0]; y += red[w][1]; }
      clip_coef(a, x, y, op.gstat, op.lr_a, op.lr_c, op.max_norm, op.coef);
    }
  }
  if (Op::NORMS) {   // global norms of the (complete) gradient tables: every nonzero row was written above
    na2 = wsum_dpp(na2);
    nc2 = wsum_dpp(nc2);
    __syncthreads();
    if (lane == 0) { red[wv][0] = na2; red[wv][1] = nc2; }
    __syncthreads();
    if (Op::APPLY) {
      if constexpr (Op::APPLY) {
        float x = 0.0f, y = 0.0f;
        for (int w = 0; w < 8; ++w) { x += red[w][0]; y += red[w][1]; }
        const float gna = sqrtf(x), gnc = sqrtf(y);
        const bool clip_a = !(gna < op.max_norm), clip_c = !(gnc < op.max_norm);
        auto upd = [&](float p0, float g, bool clip, float gn, float lr) {
          const float gg = clip ? (g / gn) * op.max_norm : g;
          return p0 + (-(lr * gg));
        };
        // theta_k / phi_k (srcv, loaded above) -> theta_w / phi_w (the same tables in place, or theta_{k+1})
        auto apply_row = [&](size_t r, const float* src, const float* g) {
          float* ta = op.theta_w + ((size_t)a * D + r) * NA;
          float* tc = op.phi_w + ((size_t)a * D + r) * NC;
#pragma unroll
          for (int j = 0; j < NA; ++j) ta[j] = upd(src[j], g[j], clip_a, gna, op.lr_a);
#pragma unroll
          for (int j = 0; j < NC; ++j) tc[j] = upd(src[NA + j], g[NA + j], clip_c, gnc, op.lr_c);
        };
        if (applied) {
#pragma unroll
          for (int e = 0; e < CH; ++e)
            if ((endm >> e) & 1u) apply_row(kc[e] >> 12, srcv[e], vec + (size_t)(kc[e] & SMASK) * NVP);
          if (tid == 0 && !has_last) {
            float g[NV];
#pragma unroll
            for (int j = 0; j < NV; ++j) g[j] = 0.0f + tot[j];
            apply_row((size_t)(D - 1), srcv[CH], g);
          }
        }
        if (tid == 0) {
          op.finish(a, x, y);   // reads step[a]: before the increment
          op.metrics(a, tot + NV);
          if (applied) op.step_w[a] += 1;
        }
      }
    } else if (tid == 0) {
      float x = 0.0f, y = 0.0f;
      for (int w = 0; w < 8; ++w) { x += red[w][0]; y += red[w][1]; }
      op.finish(a, x, y);
    }
  }
  ROWS_STAMP(5);
  if constexpr (entropy_after<Op>::value) {
    __syncthreads();   // the rewritten rows (and red's last readers) before the entropies read them
    static_assert(NVP == 13, "entropy_metric_block keeps 13 terms per sample in the row-vector area");
    entropy_metric_block(a, tid, W, T, D, op.theta_w, op.phi_w, op.tidx, op.ttime, op.met,
                         reinterpret_cast<float (*)[4]>(&red[0][0]), vec);
  }
  ROWS_STAMP(6);
}

template <class Op>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) k_rows_sorted(Op op) {
  // the reverse agent loop runs beside eval_agent's VALU-bound key chain (meta.py eval_keys_early): with a higher
  // wave priority these latency-bound blocks take the issue slots first and the key chain fills the gaps
  if (ROWS_PRIO > 0) __builtin_amdgcn_s_setprio(ROWS_PRIO);
  rows_sorted_body<Op, false>(op);
}

#ifndef ROWS2_WPE
#define ROWS2_WPE 4
#endif
// Two ops over the same samples in one block: the second reuses the first's sort (and reads what the first wrote:
// its rows and, through global memory, anything its thread 0 wrote -- the barrier orders them within the block).
template <class Op1, class Op2>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(ROWS2_WPE))) k_rows_sorted2(Op1 op1, Op2 op2) {
  if (ROWS_PRIO > 0) __builtin_amdgcn_s_setprio(ROWS_PRIO);
  rows_sorted_body<Op1, false, 1>(op1);
  __syncthreads();
  rows_sorted_body<Op2, true, 2>(op2);
}

// launch the sorted variant when one agent's samples fit (T*W <= SORT_MAX_TW, D < 2^19); false otherwise
template <class Op>
static bool launch_sorted(const Op& op, int N, hipStream_t stream) {
  const int TW = op.T * op.W;
  if (TW > SORT_MAX_TW || TW <= 0 || op.D >= (1 << 20)) return false;
  const size_t bytes = 2048 * 4 + (size_t)TW * (Op::NA + Op::NC) * 4;
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rows_sorted<Op>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 120 * 1024) != hipSuccess)
      return false;
    attr_set = true;
  }
  hipLaunchKernelGGL(k_rows_sorted<Op>, dim3(N), dim3(512), bytes, stream, op);
  return true;
}

template <class Op1, class Op2>
static bool launch_sorted2(const Op1& op1, const Op2& op2, int N, hipStream_t stream) {
  static_assert(Op1::NA + Op1::NC == Op2::NA + Op2::NC, "launch_sorted2: the ops' row vectors differ in size");
  const int TW = op1.T * op1.W;
  if (TW > SORT_MAX_TW || TW <= 0 || op1.D >= (1 << 20)) return false;
  const size_t bytes = 2048 * 4 + (size_t)TW * (Op1::NA + Op1::NC) * 4;
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rows_sorted2<Op1, Op2>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 120 * 1024) != hipSuccess)
      return false;
    attr_set = true;
  }
  hipLaunchKernelGGL((k_rows_sorted2<Op1, Op2>), dim3(N), dim3(512), bytes, stream, op1, op2);
  return true;
}

static inline unsigned nb256(long n) { return (unsigned)((n + 255) / 256); }
static inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

extern "C" {

int toued_meta_keys(const uint32_t* agent_keys, int N, int K, uint32_t* roll_keys, uint32_t* eval_keys,
                    uint32_t* ea_reset, uint32_t* ea_roll, hipStream_t stream) {
  TOUED_REQUIRE(N >= 1 && K >= 0, "toued_meta_keys: N=%d K=%d", N, K);
  hipLaunchKernelGGL(k_meta_keys, dim3((N + 63) / 64), dim3(64), 0, stream, agent_keys, N, K, roll_keys, eval_keys,
                     ea_reset, ea_roll);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_lpg_inputs(int N, int W, int T, int D, int F, const float* theta, const float* phi, const int* tidx,
                     const int* ttime, const uint8_t* tact, const float* trew, const uint8_t* tdone, const float* eta_e1w,
                     const float* eta_e1b, const float* eta_e2w, const float* eta_e2b, const int* step,
                     const int* levels, float* X, long xs_f, long xs_col, long eta_stride, hipStream_t stream) {
  TOUED_REQUIRE(F == 5 || F == 7, "toued_lpg_inputs: F=%d", F);
  const long n = (long)N * T * W;
  if (n == 0) return 0;
#define L_(U, FF) hipLaunchKernelGGL((k_lpg_inputs<U, FF>), dim3(nb256(n)), dim3(256), 0, stream, N, W, T, D, theta, \
                                     phi, tidx, ttime, tact, trew, tdone, eta_e1w, eta_e1b, eta_e2w, eta_e2b, step,   \
                                     levels, X, xs_f, xs_col, eta_stride)
  if (W % 64 == 0) { if (F == 5) L_(true, 5); else L_(true, 7); }
  else { if (F == 5) L_(false, 5); else L_(false, 7); }
#undef L_
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_lpg_inputs_rows(int N, int W, int T, int D, int F, const float* theta, const float* phi, const int* tidx,
                          const int* ttime, const uint8_t* tact, const float* trew, const uint8_t* tdone,
                          const float* eta_e1w, const float* eta_e1b, const float* eta_e2w, const float* eta_e2b,
                          const int* step, const int* levels, float* X, long xs_f, long xs_col, long eta_stride,
                          hipStream_t stream) {
  TOUED_REQUIRE(F == 5 || F == 7, "toued_lpg_inputs_rows: F=%d", F);
  TOUED_REQUIRE(W % 64 == 0, "toued_lpg_inputs_rows: W=%d must be a multiple of 64", W);
  if ((long)N * W * T == 0) return 0;
  const unsigned nb = (unsigned)((N * W) / 64);
  if (F == 5)
    hipLaunchKernelGGL(k_lpg_inputs_rows<5>, dim3(nb), dim3(64), 0, stream, N, W, T, D, theta, phi, tidx, ttime, tact,
                       trew, tdone, eta_e1w, eta_e1b, eta_e2w, eta_e2b, step, levels, X, xs_f, xs_col, eta_stride);
  else
    hipLaunchKernelGGL(k_lpg_inputs_rows<7>, dim3(nb), dim3(64), 0, stream, N, W, T, D, theta, phi, tidx, ttime, tact,
                       trew, tdone, eta_e1w, eta_e1b, eta_e2w, eta_e2b, step, levels, X, xs_f, xs_col, eta_stride);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_agent_grad(int N, int W, int T, int D, const float* theta, const float* phi, const int* tidx,
                     const int* ttime, const uint8_t* tact, const float* trew, const uint8_t* tdone,
                     const float* pi_hat, const float* y_hat, float alpha_y, float* Gth, float* Gph, float* met,
                     const int* step, const int* levels, float* gstat, hipStream_t stream) {
  TOUED_REQUIRE(step && levels && gstat, "toued_agent_grad: step, levels and gstat are required");
  if (N == 0) return 0;
  const long n = (long)N * T * W;
  if (n > 0) {
    GradOp op{theta, phi, tidx, ttime, tact, trew, tdone, pi_hat, y_hat, alpha_y, Gth, Gph, met, step, levels, gstat,
              N, W, T, D};
    if (launch_sorted(op, N, stream)) { TOUED_CHECK_LAUNCH(); return 0; }
    if (W % 64 == 0)
      hipLaunchKernelGGL(k_agent_grad<true>, dim3(nb256(n)), dim3(256), 0, stream, N, W, T, D, theta, phi, tidx, ttime,
                         tact, trew, tdone, pi_hat, y_hat, alpha_y, Gth, Gph, met);
    else
      hipLaunchKernelGGL(k_agent_grad<false>, dim3(nb256(n)), dim3(256), 0, stream, N, W, T, D, theta, phi, tidx,
                         ttime, tact, trew, tdone, pi_hat, y_hat, alpha_y, Gth, Gph, met);
  }
  hipLaunchKernelGGL(k_agent_norms, dim3(N), dim3(256), 0, stream, N, D, Gth, Gph, step, levels, gstat);
  TOUED_CHECK_LAUNCH();
  return 0;
}

// 1 when toued_agent_update supports these sizes (one agent's samples fit the sorted kernel)
int toued_agent_update_fits(int W, int T, int D) { return W > 0 && T > 0 && T * W <= SORT_MAX_TW && D < (1 << 20) ? 1 : 0; }

// toued_agent_grad + toued_agent_apply for an agent chain that never reads the gradient tables: clip + SGD in place
// on theta [N][D][5] / phi [N][D][8] (bit-identical to grad into zeroed tables + apply into fresh tables), step
// advanced when applied, met accumulated, gstat written
int toued_agent_update(int N, int W, int T, int D, float* theta, float* phi, const int* tidx, const int* ttime,
                       const uint8_t* tact, const float* trew, const uint8_t* tdone, const float* pi_hat,
                       const float* y_hat, float alpha_y, float lr_a, float lr_c, float max_norm, float* met, int* step,
                       const int* levels, float* gstat, hipStream_t stream) {
  TOUED_REQUIRE(step && levels && gstat && met, "toued_agent_update: met, step, levels and gstat are required");
  TOUED_REQUIRE(toued_agent_update_fits(W, T, D), "toued_agent_update: W=%d T=%d D=%d unsupported (T*W <= %d)", W, T, D,
                SORT_MAX_TW);
  if (N == 0) return 0;
  GradApplyOp op;
  static_cast<GradOp&>(op) = GradOp{theta, phi, tidx, ttime, tact, trew, tdone, pi_hat, y_hat, alpha_y, nullptr, nullptr,
                                    met, step, levels, gstat, N, W, T, D};
  op.theta_w = theta;
  op.phi_w = phi;
  op.lr_a = lr_a;
  op.lr_c = lr_c;
  op.max_norm = max_norm;
  op.step_w = step;
  TOUED_REQUIRE(launch_sorted(op, N, stream), "toued_agent_update: cannot launch the sorted kernel");
  TOUED_CHECK_LAUNCH();
  return 0;
}

// The meta-gradient's inner update k: toued_agent_grad + toued_agent_apply without the dense passes.  theta1 / phi1
// must already hold copies of theta / phi (theta_k); the touched rows of theta1 / phi1 are rewritten by clip + SGD
// (bit-identical to toued_agent_apply), the touched gradient rows go to Gth / Gph (bit-identical to toued_agent_grad
// there; the other rows are not written and must not be read: toued_entropy_clip and toued_hvp read touched rows
// only).  step advanced when applied, met accumulated, gstat written.
static int agent_step(int N, int W, int T, int D, const float* theta, const float* phi, float* theta1, float* phi1,
                      const int* tidx, const int* ttime, const uint8_t* tact, const float* trew, const uint8_t* tdone,
                      const float* pi_hat, const float* y_hat, float alpha_y, float lr_a, float lr_c, float max_norm,
                      float* Gth, float* Gph, float* met, int* step, const int* levels, float* gstat, bool with_entropy,
                      hipStream_t stream) {
  TOUED_REQUIRE(step && levels && gstat && met && Gth && Gph && theta1 && phi1,
                "toued_agent_step: every output is required");
  TOUED_REQUIRE(toued_agent_update_fits(W, T, D), "toued_agent_step: W=%d T=%d D=%d unsupported (T*W <= %d)", W, T, D,
                SORT_MAX_TW);
  TOUED_REQUIRE(theta1 != theta && phi1 != phi, "toued_agent_step: theta1 / phi1 must be separate tables");
  if (N == 0) return 0;
  GradStepOp op;
  static_cast<GradOp&>(op) = GradOp{theta, phi, tidx, ttime, tact, trew, tdone, pi_hat, y_hat, alpha_y, Gth, Gph,
                                    met, step, levels, gstat, N, W, T, D};
  op.theta_w = theta1;
  op.phi_w = phi1;
  op.lr_a = lr_a;
  op.lr_c = lr_c;
  op.max_norm = max_norm;
  op.step_w = step;
  if (with_entropy) {
    GradStepEntOp eop;
    static_cast<GradStepOp&>(eop) = op;
    TOUED_REQUIRE(launch_sorted(eop, N, stream), "toued_agent_step_entropy: cannot launch the sorted kernel");
  } else {
    TOUED_REQUIRE(launch_sorted(op, N, stream), "toued_agent_step: cannot launch the sorted kernel");
  }
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_agent_step(int N, int W, int T, int D, const float* theta, const float* phi, float* theta1, float* phi1,
                     const int* tidx, const int* ttime, const uint8_t* tact, const float* trew, const uint8_t* tdone,
                     const float* pi_hat, const float* y_hat, float alpha_y, float lr_a, float lr_c, float max_norm,
                     float* Gth, float* Gph, float* met, int* step, const int* levels, float* gstat, hipStream_t stream) {
  return agent_step(N, W, T, D, theta, phi, theta1, phi1, tidx, ttime, tact, trew, tdone, pi_hat, y_hat, alpha_y, lr_a,
                    lr_c, max_norm, Gth, Gph, met, step, levels, gstat, false, stream);
}

// toued_agent_step followed by toued_entropy's metric mode on theta1 / phi1 (met slots 3, 4), in the same launch
int toued_agent_step_entropy(int N, int W, int T, int D, const float* theta, const float* phi, float* theta1,
                             float* phi1, const int* tidx, const int* ttime, const uint8_t* tact, const float* trew,
                             const uint8_t* tdone, const float* pi_hat, const float* y_hat, float alpha_y, float lr_a,
                             float lr_c, float max_norm, float* Gth, float* Gph, float* met, int* step,
                             const int* levels, float* gstat, hipStream_t stream) {
  return agent_step(N, W, T, D, theta, phi, theta1, phi1, tidx, ttime, tact, trew, tdone, pi_hat, y_hat, alpha_y, lr_a,
                    lr_c, max_norm, Gth, Gph, met, step, levels, gstat, true, stream);
}

// toued_entropy's gradient mode followed by toued_clip_dot over the touched rows, in one kernel (the reverse pass of toued_agent_step's
// update k: Gth / Gph hold that update's touched rows, which are the rows this trajectory's entropy gradient writes)
int toued_meta_metrics(int N, int K, const float* met, float inv_wt, const float* loss_out, float pec, float pl2,
                       float tec, float tl2, float* out, hipStream_t stream) {
  if (N == 0) return 0;
  TOUED_REQUIRE(K >= 1, "toued_meta_metrics: K=%d", K);
  hipLaunchKernelGGL(k_meta_metrics, dim3((N + 255) / 256), dim3(256), 0, stream, N, K, met, inv_wt, loss_out, pec, pl2,
                     tec, tl2, out);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_entropy_clip(int N, int W, int T, int D, const float* theta, const float* phi, const int* tidx,
                       const int* ttime, float coef_a, float coef_c, float* adj_th, float* adj_ph, const float* Gth,
                       const float* Gph, const float* gstat, float lr_a, float lr_c, float max_norm, float* coef,
                       hipStream_t stream) {
  TOUED_REQUIRE(toued_agent_update_fits(W, T, D), "toued_entropy_clip: W=%d T=%d D=%d unsupported", W, T, D);
  if (N == 0) return 0;
  EntropyClipOp op;
  static_cast<EntropyBwdOp&>(op) = EntropyBwdOp{theta, phi, tidx, ttime, coef_a, coef_c, adj_th, adj_ph, N, W, T, D};
  op.Gth = Gth;
  op.Gph = Gph;
  op.gstat = gstat;
  op.lr_a = lr_a;
  op.lr_c = lr_c;
  op.max_norm = max_norm;
  op.coef = coef;
  TOUED_REQUIRE(launch_sorted(op, N, stream), "toued_entropy_clip: cannot launch the sorted kernel");
  TOUED_CHECK_LAUNCH();
  return 0;
}

// The reverse pass's step k as one launch: toued_entropy_clip on (theta1, phi1) = theta_{k+1} / phi_{k+1}, then
// toued_hvp on (theta, phi) = theta_k / phi_k reading the adjoint and coef the first part wrote, in place on adj_th /
// adj_ph; the rollout's samples are sorted once.  Same operations as the two launches (bit-identical).
int toued_entropy_clip_hvp(int N, int W, int T, int D, int K, const float* theta1, const float* phi1,
                           const float* theta, const float* phi, const int* tidx, const int* ttime, const uint8_t* tact,
                           const float* pi_hat, const float* y_hat, float coef_a, float coef_c, float* adj_th,
                           float* adj_ph, const float* Gth, const float* Gph, const float* gstat, float lr_a,
                           float lr_c, float max_norm, float* coef, float alpha_y, float b2, float b3, float* d_pi_hat,
                           float* d_y_hat, hipStream_t stream) {
  TOUED_REQUIRE(toued_agent_update_fits(W, T, D), "toued_entropy_clip_hvp: W=%d T=%d D=%d unsupported", W, T, D);
  if (N == 0) return 0;
  EntropyClipOp ec;
  static_cast<EntropyBwdOp&>(ec) = EntropyBwdOp{theta1, phi1, tidx, ttime, coef_a, coef_c, adj_th, adj_ph, N, W, T, D};
  ec.Gth = Gth;
  ec.Gph = Gph;
  ec.gstat = gstat;
  ec.lr_a = lr_a;
  ec.lr_c = lr_c;
  ec.max_norm = max_norm;
  ec.coef = coef;
  const HvpOp hv{theta, phi, tidx, ttime, tact, pi_hat, y_hat, Gth, Gph, adj_th, adj_ph, coef, lr_a, lr_c, alpha_y,
                 b2, b3, adj_th, adj_ph, d_pi_hat, d_y_hat, N, W, T, D, K};
  TOUED_REQUIRE(launch_sorted2(ec, hv, N, stream), "toued_entropy_clip_hvp: cannot launch the sorted kernel");
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_agent_apply(int N, int D, const float* th0, const float* ph0, const float* Gth, const float* Gph,
                      float lr_a, float lr_c, float max_norm, int* step, float* th1, float* ph1, const float* gstat,
                      hipStream_t stream) {
  if (N == 0 || D == 0) return 0;
  const bool v4 = aligned16(th0) && aligned16(ph0) && aligned16(Gth) && aligned16(Gph) && aligned16(th1) &&
                  aligned16(ph1);
  // critic table (8 D floats): ~2 vectors per thread at the chosen width; the actor table's blocks beyond its
  // size exit at once
  const long nvec = v4 ? (long)D * 2 + 1 : (long)D * 8;
  const unsigned gx = (unsigned)std::max(1L, std::min(64L, (nvec + 511) / 512));
  hipLaunchKernelGGL(k_agent_apply, dim3(gx, N, 2), dim3(256), 0, stream, N, D, th0, ph0, Gth, Gph, lr_a, lr_c,
                     max_norm, step, th1, ph1, gstat, v4 ? 1 : 0);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_entropy(int N, int W, int T, int D, const float* theta, const float* phi, const int* tidx, const int* ttime,
                  float* met, float coef_a, float coef_c, float* adj_th, float* adj_ph, hipStream_t stream) {
  const long n = (long)N * T * W;
  if (n == 0) return 0;
  if (adj_th && !met) {
    EntropyBwdOp op{theta, phi, tidx, ttime, coef_a, coef_c, adj_th, adj_ph, N, W, T, D};
    if (launch_sorted(op, N, stream)) { TOUED_CHECK_LAUNCH(); return 0; }
  }
  if (met && !adj_th) {   // metrics only: deterministic per-agent reduction
    hipLaunchKernelGGL(k_entropy_metric, dim3(N), dim3(256), 0, stream, W, T, D, theta, phi, tidx, ttime, met);
    TOUED_CHECK_LAUNCH();
    return 0;
  }
  if (W % 64 == 0)
    hipLaunchKernelGGL(k_entropy<true>, dim3(nb256(n)), dim3(256), 0, stream, N, W, T, D, theta, phi, tidx, ttime,
                       met, coef_a, coef_c, adj_th, adj_ph);
  else
    hipLaunchKernelGGL(k_entropy<false>, dim3(nb256(n)), dim3(256), 0, stream, N, W, T, D, theta, phi, tidx, ttime,
                       met, coef_a, coef_c, adj_th, adj_ph);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_eval_loss(int N, int W, int T, int D, const float* theta, const float* vcrit, const int* tidx,
                    const int* ttime, const uint8_t* tact, const float* trew, const uint8_t* tdone, float gamma,
                    float lam, float* adv_scratch, float* abar, float* out, hipStream_t stream) {
  if (N == 0) return 0;
  hipLaunchKernelGGL(k_eval_loss, dim3(N), dim3(64), 0, stream, N, W, T, D, theta, vcrit, tidx, ttime, tact, trew,
                     tdone, gamma, lam, adv_scratch, abar, out);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_lpgloss_grad(int N, int W, int T, int D, const float* theta, const int* tidx, const int* ttime,
                       const uint8_t* tact, const float* abar, float* adj_th, hipStream_t stream) {
  const long n = (long)N * T * W;
  if (n == 0) return 0;
  {
    LpgLossOp op{theta, tidx, ttime, tact, abar, adj_th, N, W, T, D};
    if (launch_sorted(op, N, stream)) { TOUED_CHECK_LAUNCH(); return 0; }
  }
  if (W % 64 == 0)
    hipLaunchKernelGGL(k_lpgloss_grad<true>, dim3(nb256(n)), dim3(256), 0, stream, N, W, T, D, theta, tidx, ttime,
                       tact, abar, adj_th);
  else
    hipLaunchKernelGGL(k_lpgloss_grad<false>, dim3(nb256(n)), dim3(256), 0, stream, N, W, T, D, theta, tidx, ttime,
                       tact, abar, adj_th);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_clip_dot(int N, int D, const float* Gth, const float* Gph, const float* adj_th, const float* adj_ph,
                   const float* gstat, float lr_a, float lr_c, float max_norm, float* coef, hipStream_t stream) {
  if (N == 0) return 0;
  const bool v4 = aligned16(Gth) && aligned16(Gph) && aligned16(adj_th) && aligned16(adj_ph);
  hipLaunchKernelGGL(k_clip_dot, dim3(N), dim3(1024), 0, stream, N, D, Gth, Gph, adj_th, adj_ph, gstat, lr_a, lr_c,
                     max_norm, coef, v4 ? 1 : 0);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_hvp(int N, int W, int T, int D, int K, const float* theta, const float* phi, const int* tidx,
              const int* ttime, const uint8_t* tact, const float* pi_hat, const float* y_hat, const float* Gth,
              const float* Gph, const float* adj_th_in, const float* adj_ph_in, const float* coef, float lr_a,
              float lr_c, float alpha_y, float b2, float b3, float* adj_th_out, float* adj_ph_out, float* d_pi_hat,
              float* d_y_hat, hipStream_t stream) {
  const long n = (long)N * T * W;
  if (n == 0) return 0;
  {
    HvpOp op{theta, phi, tidx, ttime, tact, pi_hat, y_hat, Gth, Gph, adj_th_in, adj_ph_in, coef, lr_a, lr_c, alpha_y,
             b2, b3, adj_th_out, adj_ph_out, d_pi_hat, d_y_hat, N, W, T, D, K};
    if (launch_sorted(op, N, stream)) { TOUED_CHECK_LAUNCH(); return 0; }
  }
  if (W % 64 == 0)
    hipLaunchKernelGGL(k_hvp<true>, dim3(nb256(n)), dim3(256), 0, stream, N, W, T, D, K, theta, phi, tidx, ttime, tact,
                       pi_hat, y_hat, Gth, Gph, adj_th_in, adj_ph_in, coef, lr_a, lr_c, alpha_y, b2, b3, adj_th_out,
                       adj_ph_out, d_pi_hat, d_y_hat);
  else
    hipLaunchKernelGGL(k_hvp<false>, dim3(nb256(n)), dim3(256), 0, stream, N, W, T, D, K, theta, phi, tidx, ttime,
                       tact, pi_hat, y_hat, Gth, Gph, adj_th_in, adj_ph_in, coef, lr_a, lr_c, alpha_y, b2, b3,
                       adj_th_out, adj_ph_out, d_pi_hat, d_y_hat);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_embed_bwd(int N, int W, int T, int D, int K, const float* phi_hist, long phi_stride, int phi_slot0,
                    const int* tidx_hist,
                    long tidx_stride, const int* ttime_hist, const uint8_t* tdone_hist, long tstep_stride,
                    const float* dX3, const float* dX4, long dx_stride_k, const float* e1w, const float* e1b,
                    const float* e2w, float* partial, int n_blocks, hipStream_t stream) {
  if ((long)K * N * T * W == 0) return 0;
  TOUED_REQUIRE((long)K * N * (T + 1) * W < (1L << 31), "toued_embed_bwd: K*N*(T+1)*W = %ld samples exceed 2^31",
                (long)K * N * (T + 1) * W);
  TOUED_REQUIRE(phi_slot0 >= 0 && phi_slot0 <= K, "toued_embed_bwd: phi_slot0=%d outside the K+1=%d slots", phi_slot0,
                K + 1);
#define L_(KER) hipLaunchKernelGGL(KER, dim3(n_blocks), dim3(256), 0, stream, N, W, T, D, K, phi_hist, phi_stride,     \
                                   phi_slot0,                                                                       \
                                   tidx_hist, tidx_stride, ttime_hist, tdone_hist, tstep_stride, dX3, dX4, dx_stride_k, \
                                   e1w, e1b, e2w, partial)
  if (EMBED_V == 3) {
    if (W % 64 == 0) L_(k_embed_bwd3<true>); else L_(k_embed_bwd3<false>);
  } else {
    if (W % 64 == 0) L_(k_embed_bwd<true>); else L_(k_embed_bwd<false>);
  }
#undef L_
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_init_tables(const uint32_t* keys, int n, int cols, int D, float lo, float hi, float stddev, float* out,
                      hipStream_t stream) {
  const long tot = (long)n * D * cols;
  if (tot == 0) return 0;
  hipLaunchKernelGGL(k_init_tables, dim3(nb256((long)D * cols), n), dim3(256), 0, stream, keys, n, cols, D, lo, hi,
                     stddev, out, nullptr);
  TOUED_CHECK_LAUNCH();
  return 0;
}

// the same, writing only the tables i with mask[i] != 0 (in place: the level sampler's where(terminated, new, old))
int toued_init_tables_masked(const uint32_t* keys, int n, int cols, int D, float lo, float hi, float stddev,
                             float* out, const uint8_t* mask, hipStream_t stream) {
  TOUED_REQUIRE(mask != nullptr, "toued_init_tables_masked: mask required");
  const long tot = (long)n * D * cols;
  if (tot == 0) return 0;
  hipLaunchKernelGGL(k_init_tables_blk, dim3(n), dim3(256), 0, stream, keys, n, cols, D, lo, hi, stddev, out, mask);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_gather_add(float* out, const float* src, const int* src_idx, const int* dst_idx, int n, hipStream_t stream) {
  TOUED_REQUIRE(n >= 0, "toued_gather_add: n=%d", n);
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_gather_add, dim3((n + 255) / 256), dim3(256), 0, stream, out, src, src_idx, dst_idx, n);
  TOUED_CHECK_LAUNCH();
  return 0;
}

#ifdef ROWS_STAMPS
int toued_dbg_rows_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_rows_stamps), sizeof(g_rows_stamps)) == hipSuccess ? 0 : 1;
}
int toued_dbg_rows_span(unsigned long long* host) {   // [3][8][1024][4]: start, end, XCC_ID, HW_ID
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_rows_span), sizeof(g_rows_span)) == hipSuccess ? 0 : 1;
}
#endif

int toued_sum_rows_add(const float* part, int rows, int cols, float* out, hipStream_t stream) {
  TOUED_REQUIRE(rows >= 0 && cols >= 0, "toued_sum_rows_add: rows=%d cols=%d", rows, cols);
  if (cols == 0) return 0;
  hipLaunchKernelGGL(k_sum_rows_add, dim3(cols), dim3(256), 0, stream, part, rows, cols, out);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_adam(int P, float* eta, const float* grad, float* m, float* v, float n_mean, float lr, double b1, double b2,
               float eps, int count, hipStream_t stream) {
  TOUED_REQUIRE(count >= 1 && n_mean > 0.0f, "toued_adam: count=%d n_mean=%g", count, (double)n_mean);
  if (P == 0) return 0;
  // jax weak-typed python floats: decay -> f32(b), (1 - decay) -> f32(1.0 - b) rounded from double;
  // decay**count in f32 (int32 count), then 1 - that in f32
  const float b1f = (float)b1, b2f = (float)b2;
  const float bc1 = 1.0f - powf(b1f, (float)count), bc2 = 1.0f - powf(b2f, (float)count);
  hipLaunchKernelGGL(k_adam, dim3(nb256(P)), dim3(256), 0, stream, P, eta, grad, m, v, n_mean, lr, b1f,
                     (float)(1.0 - b1), b2f, (float)(1.0 - b2), eps, bc1, bc2);
  TOUED_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
