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
//   k_a2c_update the whole update in one block per agent, deterministic: per-sample row vectors in LDS,
//                sorted by (row, sample), segment sums in sample order, norms, clip and SGD on the touched rows
//                (W*T <= 2048; grad + apply, which scatter with float atomics, are the fallback above that)
//
// Trajectory layout as the rollout kernel writes it: idx/time [N][T+1][W], act/done/rew [N][T][W].
#include "env_dev.h"
#include "wave_dev.h"

#include <cstdlib>
#include <cstring>

#define EPSF 1e-8f

#ifdef A2C_STAMPS_FINE
// finer stamps inside the V gather + GAE phase (tools/a2c_stamps.py --fine): every update overwrites them
__device__ unsigned long long g_a2c_fine[512 * 8];
#define A2C_FINE(ph)                                                                                   \
  do {                                                                                                 \
    if (blockIdx.x < 512 && threadIdx.x == 0) g_a2c_fine[blockIdx.x * 8 + (ph)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define A2C_FINE(ph) do {} while (0)
#endif

namespace {

TOUED_DEV float wave_sum(float v) { return wsum_dpp(v); }

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

// Block-wide sums of N values at once (256-thread blocks, red >= 4 N floats): one barrier pair instead of N; the
// same summation order as N block_sum calls.
template <int N>
TOUED_DEV void block_sum_n(float (&v)[N], float* red) {
#pragma unroll
  for (int j = 0; j < N; ++j) v[j] = wave_sum(v[j]);
  const int wv = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int j = 0; j < N; ++j) red[wv * N + j] = v[j];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < N; ++j) {
    float s = 0.0f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i * N + j];
    v[j] = s;
  }
}

// Staged trajectory of one agent in LDS and the quantities every sample's gradient needs.
struct A2CStage {
  float* vt;    // [T+1][W] V(obs)
  float* cc;    // [T+1][W] 0.001 * time
  int* ix;      // [T+1][W] obs row
  float* rw;    // [T][W] reward
  float* nd;    // [T][W] 1 - done
  float* adv;   // [W*T] GAE advantages, worker-major
  float* dv;    // [W*T] target - V
  float* abar;  // [W] mean_t normalised advantage
  uint8_t* act; // [T][W] action
  __host__ __device__ static size_t floats(int W, int T) {
    return 3 * (size_t)(T + 1) * W + 4 * (size_t)W * T + W + ((size_t)W * T + 3) / 4;
  }
  TOUED_DEV void carve(float* base, int W, int T) {
    const int NO = (T + 1) * W, NS = T * W;
    vt = base;
    cc = vt + NO;
    ix = reinterpret_cast<int*>(cc + NO);
    rw = reinterpret_cast<float*>(ix + NO);
    nd = rw + NS;
    adv = nd + NS;
    dv = adv + NS;
    abar = dv + NS;
    act = reinterpret_cast<uint8_t*>(abar + W);
  }
};

// S.vt[j] = V(obs j) + c_j V[D-1] for the NO staged observations, from S.ix / S.cc: each thread's up to VB gathers are
// issued before the first is waited on.  Ends without a barrier; the caller syncs.
TOUED_DEV void gather_values(const A2CStage& S, const float* __restrict__ v, int D, int NO) {
  constexpr int VB = 8;
  const int tid = threadIdx.x, nt = blockDim.x;
  const float vlast = v[D - 1];
  for (int j0 = tid; j0 < NO; j0 += VB * nt) {
    float g[VB];
#pragma unroll
    for (int q = 0; q < VB; ++q) {
      const int j = j0 + q * nt;
      g[q] = j < NO ? v[S.ix[j]] : 0.0f;
    }
#pragma unroll
    for (int q = 0; q < VB; ++q) {
      const int j = j0 + q * nt;
      if (j < NO) S.vt[j] = g[q] + S.cc[j] * vlast;
    }
  }
}

// Latency structure: the agent's whole trajectory (obs rows and times, actions, rewards, dones) is staged into LDS
// with coalesced loads, V(obs) gathered for every observation at once, and only then the per-worker GAE scans run
// out of LDS -- a handful of dependent memory round trips per update instead of two per time step.  Ends with a
// barrier.
TOUED_DEV void a2c_load(const A2CStage& S, int a, int W, int T, int D, const float* __restrict__ v,
                        const int* __restrict__ tidx, const int* __restrict__ ttime, const uint8_t* __restrict__ tact,
                        const float* __restrict__ trew, const uint8_t* __restrict__ tdone) {
  const int NO = (T + 1) * W, NS = T * W, tid = threadIdx.x;
  const float vlast = v[D - 1];
  const size_t tb = (size_t)a * (T + 1) * W;
  const size_t sb = (size_t)a * T * W;
  for (int i = tid; i < NO; i += blockDim.x) {
    const int idx = tidx[tb + i];
    const float c = (float)ttime[tb + i] * 0.001f;
    S.ix[i] = idx;
    S.cc[i] = c;
    S.vt[i] = v[idx] + c * vlast;
  }
  for (int i = tid; i < NS; i += blockDim.x) {
    S.rw[i] = trew[sb + i];
    S.nd[i] = tdone[sb + i] ? 0.0f : 1.0f;
    if (tact) S.act[i] = tact[sb + i];
  }
  __syncthreads();
}

// GAE on the staged trajectory.  Returns the critic loss mean((target - V)^2) (a2c.py:29-37); fills adv/dv/abar
// (a2c.py:43 normalisation, the [T,T] broadcast's mean_t factor).  Ends with a barrier.
// one worker's reverse GAE scan over the staged trajectory; the restrict-qualified views let the unrolled loop issue
// a chunk's LDS loads ahead of the previous steps' adv / dv stores (with plain pointers into the one LDS stage each
// step waited a load round trip: 4.0 k cycles per 20-step scan, profiles/r04/a2c_stamps_fine_r04h.log)
TOUED_DEV void gae_scan(const float* __restrict__ vt, const float* __restrict__ nd, const float* __restrict__ rw,
                        float* __restrict__ adv, float* __restrict__ dv, int W, int T, int w, float gamma, float lam,
                        float& s_adv, float& cl) {
  float vn = vt[T * W + w];
  float g = 0.0f;
#pragma unroll 10
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
}

TOUED_DEV float a2c_gae(const A2CStage& S, int W, int T, float gamma, float lam, float* red) {
  const int tid = threadIdx.x;
  const float n = (float)(W * T);
  if (W <= 64) {
    // every worker in wave 0: the scan, the advantage mean, the critic loss, the variance (two-pass over each
    // worker's own advantages) and abar without a block reduction -- wave sums only, one barrier at the end (the
    // block path's three reductions cost ~1.4 k cycles each, profiles/r04/a2c_stamps_fine_r04h.log).  The mean and
    // the critic loss are the block path's values bit for bit (its other waves add zeros); the variance is summed
    // per worker instead of strided over the block.
    if (tid < 64) {
      float sa = 0.0f, cl = 0.0f;
      if (tid < W) gae_scan(S.vt, S.nd, S.rw, S.adv, S.dv, W, T, tid, gamma, lam, sa, cl);
      A2C_FINE(2);
      const float mean = wsum_dpp(sa) / n;
      const float closs = wsum_dpp(tid < W ? cl / (float)T : 0.0f) / (float)W;
      A2C_FINE(3);
      float sv = 0.0f;
      if (tid < W) {
#pragma unroll 4
        for (int t = 0; t < T; ++t) {
          const float d = S.adv[tid * T + t] - mean;
          sv += d * d;
        }
      }
      const float inv_sd = 1.0f / (sqrtf(wsum_dpp(sv) / n) + EPSF);
      A2C_FINE(4);
      if (tid < W) {
        float ab = 0.0f;
#pragma unroll 4
        for (int t = 0; t < T; ++t) ab += (S.adv[tid * T + t] - mean) * inv_sd;
        S.abar[tid] = ab / (float)T;
      }
      if (tid == 0) red[0] = closs;
    }
    __syncthreads();
    return red[0];
  }
  // per-worker GAE (reverse scan over T, util/metrics.py:17-38)
  float s_adv = 0.0f, s_cl = 0.0f;
  for (int w = tid; w < W; w += blockDim.x) {
    float cl = 0.0f;
    gae_scan(S.vt, S.nd, S.rw, S.adv, S.dv, W, T, w, gamma, lam, s_adv, cl);
    s_cl += cl / (float)T;
  }
  A2C_FINE(2);
  float ms[2] = {s_adv, s_cl};
  block_sum_n<2>(ms, red);
  A2C_FINE(3);
  const float mean = ms[0] / n;
  const float closs = ms[1] / (float)W;
  float s_var = 0.0f;
  for (int i = tid; i < W * T; i += blockDim.x) {
    const float d = S.adv[i] - mean;
    s_var += d * d;
  }
  const float inv_sd = 1.0f / (sqrtf(block_sum(s_var, red) / n) + EPSF);
  A2C_FINE(4);
  for (int w = tid; w < W; w += blockDim.x) {
    float ab = 0.0f;
#pragma unroll 4
    for (int t = 0; t < T; ++t) ab += (S.adv[w * T + t] - mean) * inv_sd;
    S.abar[w] = ab / (float)T;
  }
  __syncthreads();
  return closs;
}

// Sample i = t*W + w of the staged agent: actor row cotangent d[5] (policy term through the [T,T] broadcast plus
// the entropy bonus of pi + 1e-8, a2c.py:52-63), critic row cotangent (returned), the row, the time coefficient
// and this sample's actor-loss term.
// The gradient maths run on the hardware transcendentals (v_exp_f32 / v_log_f32 / v_rcp_f32 without the library's
// denormal range scaling: every argument here is a normal number or an exp underflow) and explicit FMAs: about a
// third fewer VALU per sample, within the update's float tolerance (tests/test_gpu_plr.py, 1e-4 of the float64 step).
// The FMAs are written out, not left to contraction, which depends on the surrounding code: the chain kernel and the
// one-update kernel inline this into different contexts and must stay bit-identical.  The rollouts, which steer
// sampling, keep their exact portable maths.
TOUED_DEV float hexp(float x) { return __builtin_amdgcn_exp2f(x * 1.44269504088896341f); }
TOUED_DEV float hlog(float x) { return __builtin_amdgcn_logf(x) * 0.693147180559945309f; }

TOUED_DEV float a2c_sample(const A2CStage& S, int i, int W, int T, const float* thr, const float* lastA, float ent_coef,
                           float inv_n, float* d, float& c, float& al) {
  const int t = i / W, w = i - t * W;
  c = S.cc[i];
  const int act = S.act[i];
  float l[5], p[5], m = -__builtin_inff();
#pragma unroll
  for (int j = 0; j < 5; ++j) { l[j] = fmaf(c, lastA[j], thr[j]); m = fmaxf(m, l[j]); }
  float z = 0.0f;
#pragma unroll
  for (int j = 0; j < 5; ++j) { p[j] = hexp(l[j] - m); z += p[j]; }
  const float iz = __builtin_amdgcn_rcpf(z);
  float pa = 0.0f, h = 0.0f, gl[5], pg = 0.0f;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    p[j] *= iz;
    pa = (j == act) ? p[j] : pa;
    const float lg = hlog(p[j] + EPSF);
    h = fmaf(-(p[j] + EPSF), lg, h);
    gl[j] = -(lg + 1.0f);
    pg = fmaf(p[j], gl[j], pg);
  }
  const float ab = S.abar[w];
  const float rho = pa * __builtin_amdgcn_rcpf(pa + EPSF);
  const float kr = -ab * inv_n * rho;
  const float ke = -ent_coef * inv_n;
#pragma unroll
  for (int j = 0; j < 5; ++j) d[j] = fmaf(kr, (j == act ? 1.0f : 0.0f) - p[j], ke * p[j] * (gl[j] - pg));
  al = fmaf(-hlog(pa + EPSF), ab, -ent_coef * h);
  return -2.0f * S.dv[w * T + t] * inv_n;
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

// loss_out[a] += {actor_loss, critic_loss} (accumulated over updates; the caller zeroes it).  Fallback for
// W*T > 2048: the per-sample rows are scattered with float atomics (summation order not fixed).
__global__ void __launch_bounds__(256) k_a2c_grad(int W, int T, int D, const float* __restrict__ theta,
                                                  const float* __restrict__ vcrit, const int* __restrict__ tidx,
                                                  const int* __restrict__ ttime, const uint8_t* __restrict__ tact,
                                                  const float* __restrict__ trew, const uint8_t* __restrict__ tdone,
                                                  float gamma, float lam, float ent_coef, float* __restrict__ Ga,
                                                  float* __restrict__ Gv, float* __restrict__ loss_out) {
  extern __shared__ float lds[];
  __shared__ float red[8];
  A2CStage S;
  S.carve(lds, W, T);
  const int a = blockIdx.x, tid = threadIdx.x;
  a2c_load(S, a, W, T, D, vcrit + (size_t)a * D, tidx, ttime, tact, trew, tdone);
  const float closs = a2c_gae(S, W, T, gamma, lam, red);
  const float* th = theta + (size_t)a * D * 5;
  float* ga = Ga + (size_t)a * D * 5;
  float* gv = Gv + (size_t)a * D;
  float lastA[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) lastA[j] = th[(size_t)(D - 1) * 5 + j];
  const float inv_n = 1.0f / (float)(W * T);
  float accA[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f}, accV = 0.0f, s_al = 0.0f;
  for (int i = tid; i < W * T; i += blockDim.x) {
    float d[5], c, al, thr[5];
    const int idx = S.ix[i];
#pragma unroll
    for (int j = 0; j < 5; ++j) thr[j] = th[(size_t)idx * 5 + j];
    const float dvv = a2c_sample(S, i, W, T, thr, lastA, ent_coef, inv_n, d, c, al);
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      atomicAdd(&ga[(size_t)idx * 5 + j], d[j]);
      accA[j] += c * d[j];
    }
    atomicAdd(&gv[idx], dvv);
    accV += c * dvv;
    s_al += al;
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
  // optax's t / g_norm * max_norm as one scale per table (v_rcp_f32: within the update's float tolerance)
  const float sc_a = max_norm * __builtin_amdgcn_rcpf(gna), sc_c = max_norm * __builtin_amdgcn_rcpf(gnc);
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

// ---------------------------------------------------------------------------- deterministic fused update
// One block (256 threads) per agent, W*T <= 2048 samples.  The reference's gradient is obs^T . dlogits over the
// agent's [W, T] batch (XLA, deterministic); here every sample's 6-float row cotangent (5 actor + 1 critic) is
// written to LDS, the keys (row << 11 | sample) are bitonic-sorted in registers (wave_dev.h), and each row's
// segment is summed by a segmented scan over the chunks (a fixed combination tree) -- no atomics, so a replay gives
// bit-identical tables.  The row sums stay in LDS (in the vector slot of the segment's last sample) until the two
// global norms are known; then clip + SGD rewrite only the rows that have samples (an untouched row's update
// th + -(lr * 0) is the identity).  The time row D-1 (every sample contributes c * v) is a block reduction.  LDS
// does not depend on D: staged trajectory + 2048 keys + W*T*6 floats (~77 KB at W=64, T=20), so two agents share
// a CU.
#define A2C_SORT_MAX 2048
#define A2C_NV 6

#ifdef A2C_STAMPS
// timing instrumentation (tools/a2c_stamps.py, built by tools/build_variant.py a2c.hip A2C_STAMPS=1): thread 0 of
// workgroups < 512 records s_memtime at 7 points of the (last) launch (k_a2c_chain: of its last update, plus the end of
// the env phase in slot 7)
__device__ unsigned long long g_a2c_stamps[512 * 8];
#define A2C_STAMP(ph)                                                                                  \
  do {                                                                                                 \
    if (blockIdx.x < 512 && tid == 0) g_a2c_stamps[blockIdx.x * 8 + (ph)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define A2C_STAMP(ph) do {} while (0)
#endif

// LDS scalars of one fused update
struct A2CShared {
  float red[4 * (A2C_NV + 1)];
  float tot[A2C_NV];
  int has_last;
  int scan_a[4];              // the segmented scan's per-wave totals
  float scan_b[4][A2C_NV];
  int dflag[64];              // toued_a2c_chain_self: step t's keys of the update being drawn are in LDS (its number + 1)
};

// The fused update on a staged trajectory after its GAE (closs = the critic loss): per-sample row vectors, the sort,
// segmented sums, norms, clip + SGD of the touched rows, the step counter and the losses.  sh.has_last must be 0 on
// entry (the caller clears it before a barrier).  CRITIC_ONLY: the meta-gradient value critic's own update
// (meta/train.py:61-81 with the reference's discarded `.replace` fixed, --fix_value_critic): the same critic loss
// and SGD, no actor, no lifetime discard, `step` is the value critic's TrainState step.
template <bool CRITIC_ONLY>
TOUED_DEV void a2c_update_body(const A2CStage& S, uint32_t* key, float* vec, A2CShared& sh, float closs, int a, int W,
                               int T, int D, float* __restrict__ theta, float* __restrict__ vcrit, float ent_coef,
                               float lr_a, float lr_c, float max_norm, int* __restrict__ step,
                               const int* __restrict__ levels, float* __restrict__ loss_out) {
  constexpr int NV = A2C_NV, CH = A2C_SORT_MAX / 256;
  constexpr uint32_t NONE = 0xFFFFFFFFu, SMASK = 2047u;
  const int tid = threadIdx.x, TW = W * T;
  float* red = sh.red;
  float* tot = sh.tot;
  int& has_last = sh.has_last;
  float* v = vcrit + (size_t)a * D;
  float* th = CRITIC_ONLY ? nullptr : theta + (size_t)a * D * 5;
  // 1) per-sample row vectors -> LDS, sort keys, time-row partial sums, actor loss.  Thread t's samples
  //    sl = t + 256 h: their actor rows are gathered up front (eight independent loads in flight, not one per sample)
  const int lane = tid & 63, wv = tid >> 6;
  float lastA[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
  if (!CRITIC_ONLY) {
#pragma unroll
    for (int j = 0; j < 5; ++j) lastA[j] = th[(size_t)(D - 1) * 5 + j];
  }
  const float inv_n = 1.0f / (float)TW;
  // actor rows through a buffer descriptor over the whole table array (host-checked < 4 GiB): a 16-byte and a
  // 4-byte load per 20-byte row instead of five dword gathers
  const __amdgpu_buffer_rsrc_t rs_th = theta_rsrc(CRITIC_ONLY ? vcrit : theta);
  const unsigned th_off = (unsigned)((size_t)a * D * 20);
  int sidx[CH];
  float trow[CH][5];
#pragma unroll
  for (int h = 0; h < CH; ++h) {
    const int sl = tid + 256 * h;
    sidx[h] = sl < TW ? S.ix[sl] : 0;
#pragma unroll
    for (int j = 0; j < 5; ++j) trow[h][j] = 0.0f;
    if (!CRITIC_ONLY && sl < TW) load_row5(rs_th, th_off + (unsigned)sidx[h] * 20u, trow[h]);
  }
  float acc[NV + 1] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};   // time-row partials [NV], actor loss
#pragma unroll
  for (int h = 0; h < CH; ++h) {
    const int sl = tid + 256 * h;
    uint32_t kk = NONE;
    if (sl < TW) {
      float d[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f}, c, al = 0.0f, dvv;
      const int idx = sidx[h];
      if (CRITIC_ONLY) {
        const int t = sl / W, w = sl - t * W;
        c = S.cc[sl];
        dvv = -2.0f * S.dv[w * T + t] * inv_n;
      } else {
        dvv = a2c_sample(S, sl, W, T, trow[h], lastA, ent_coef, inv_n, d, c, al);
      }
      kk = ((uint32_t)idx << 11) | (uint32_t)sl;
#pragma unroll
      for (int j = 0; j < 5; ++j) { vec[sl * NV + j] = d[j]; acc[j] += c * d[j]; }
      vec[sl * NV + 5] = dvv;
      acc[5] += c * dvv;
      acc[NV] += al;
      if (idx == D - 1) has_last = 1;
    }
    key[sl] = kk;
  }
  block_sum_n<NV + 1>(acc, red);
  if (tid == 0) {
#pragma unroll
    for (int j = 0; j < NV; ++j) tot[j] = acc[j];
  }
  const float al = acc[NV] * inv_n;
  A2C_STAMP(2);
  // 2) sort by (row, sample)
  sort2048_reg<256>(key, tid);
  A2C_STAMP(3);
  // 3) segmented row sums, deterministic (a fixed combination tree).  Thread t owns the sorted entries
  //    [CH t, CH t + CH) as runs of equal rows.  The part of a segment lying in earlier chunks (the carry) reaches the
  //    chunk where the segment ends through a segmented scan over the 256 chunks: carry_t = a_t carry_{t-1} + b_t,
  //    b_t = the sum of chunk t's last run, a_t = 1 iff chunk t is one run continuing chunk t-1's segment.  Each
  //    segment's sum goes to the vector slot of its LAST entry; that entry's thread applies it.
  auto rowof = [](uint32_t k) { return k == NONE ? NONE : (k >> 11); };
  uint32_t kc[CH];
  {
    const uint4* kv = reinterpret_cast<const uint4*>(key) + 2 * tid;
    const uint4 x0 = kv[0], x1 = kv[1];
    kc[0] = x0.x; kc[1] = x0.y; kc[2] = x0.z; kc[3] = x0.w;
    kc[4] = x1.x; kc[5] = x1.y; kc[6] = x1.z; kc[7] = x1.w;
  }
  const uint32_t prow = tid == 0 ? NONE : rowof(key[CH * tid - 1]);
  const uint32_t nrow = tid == 255 ? NONE : rowof(key[CH * tid + CH]);
  uint32_t endm = 0u;   // bit e: a segment ends at entry e
#pragma unroll
  for (int e = 0; e < CH; ++e) {
    const uint32_t r = rowof(kc[e]);
    const uint32_t rn = e < CH - 1 ? rowof(kc[e + 1]) : nrow;
    if (r != NONE && rn != r) endm |= 1u << e;
  }
  // pass 1: the last run's sum b_t and a_t
  float sb[NV] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
  const uint32_t r0 = rowof(kc[0]);
  int sa = (r0 != NONE && prow == r0) ? 1 : 0;
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
        const float* ve = vec + (size_t)(kc[e] & SMASK) * NV;
#pragma unroll
        for (int j = 0; j < NV; ++j) sb[j] += ve[j];
      }
    }
  }
  // inclusive scan of (a, b) within the wave, then across the four waves
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
    sh.scan_a[wv] = sa;
#pragma unroll
    for (int j = 0; j < NV; ++j) sh.scan_b[wv][j] = sb[j];
  }
  __syncthreads();
  float pb[NV] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};   // carry at the end of wave wv - 1
  for (int w2 = 0; w2 < wv; ++w2) {
    const bool cont = w2 > 0 && sh.scan_a[w2];
#pragma unroll
    for (int j = 0; j < NV; ++j) pb[j] = cont ? pb[j] + sh.scan_b[w2][j] : sh.scan_b[w2][j];
  }
  float cin[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const float x = (wv > 0 && sa) ? pb[j] + sb[j] : sb[j];   // carry at the end of this chunk
    cin[j] = __shfl_up(x, 1, 64);
    if (lane == 0) cin[j] = pb[j];                          // (wave 0, lane 0: no carry, r0 != prow)
  }
  // pass 2: runs in entry order, the first one continuing the carry; sums at segment ends
  float na2 = 0.0f, nc2 = 0.0f;
  {
    const bool cont = r0 != NONE && prow == r0;
    float run[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) run[j] = cont ? cin[j] : 0.0f;
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
        float* ve = vec + (size_t)(kc[e] & SMASK) * NV;
#pragma unroll
        for (int j = 0; j < NV; ++j) run[j] += ve[j];
        if ((endm >> e) & 1u) {
          if ((int)r == D - 1) {
#pragma unroll
            for (int j = 0; j < NV; ++j) run[j] += tot[j];
          }
#pragma unroll
          for (int j = 0; j < NV; ++j) ve[j] = run[j];
#pragma unroll
          for (int j = 0; j < 5; ++j) na2 += run[j] * run[j];
          nc2 += run[5] * run[5];
        }
      }
    }
  }
  if (tid == 0 && !has_last) {
#pragma unroll
    for (int j = 0; j < 5; ++j) na2 += tot[j] * tot[j];
    nc2 += tot[5] * tot[5];
  }
  A2C_STAMP(4);
  // 4) clip_by_global_norm + SGD (models/optim.py:5-11), discarded past the lifetime (a2c.py:71-75).  The rows of
  //    this thread's segments are gathered before the norm reduction, so its barriers cover their latency.
  const int st = step[a];
  const bool applied = CRITIC_ONLY || (st + 1) <= levels[(size_t)a * LEVEL_WORDS + L_LIFETIME];
  float rth[CH][5], rv[CH];
#pragma unroll
  for (int e = 0; e < CH; ++e) {
    const bool on = applied && ((endm >> e) & 1u);
    const size_t r = on ? (size_t)(kc[e] >> 11) : 0;
#pragma unroll
    for (int j = 0; j < 5; ++j) rth[e][j] = 0.0f;
    if (!CRITIC_ONLY && on) load_row5(rs_th, th_off + (unsigned)r * 20u, rth[e]);
    rv[e] = on ? v[r] : 0.0f;
  }
  float nn[2] = {na2, nc2};
  block_sum_n<2>(nn, red);
  const float gna = sqrtf(nn[0]), gnc = sqrtf(nn[1]);
  const bool clip_a = !(gna < max_norm), clip_c = !(gnc < max_norm);
  // optax's t / g_norm * max_norm as one scale per table (v_rcp_f32: within the update's float tolerance)
  const float sc_a = max_norm * __builtin_amdgcn_rcpf(gna), sc_c = max_norm * __builtin_amdgcn_rcpf(gnc);
  A2C_STAMP(5);
  if (applied) {
#pragma unroll
    for (int e = 0; e < CH; ++e) {
      if ((endm >> e) & 1u) {
        const size_t r = kc[e] >> 11;
        const float* g = vec + (size_t)(kc[e] & SMASK) * NV;
        if (!CRITIC_ONLY) {
#pragma unroll
          for (int j = 0; j < 5; ++j) {
            const float gg = clip_a ? g[j] * sc_a : g[j];
            th[r * 5 + j] = rth[e][j] + (-(lr_a * gg));
          }
        }
        const float gg = clip_c ? g[5] * sc_c : g[5];
        v[r] = rv[e] + (-(lr_c * gg));
      }
    }
    if (tid == 0 && !has_last) {
      const size_t r = (size_t)(D - 1);
      if (!CRITIC_ONLY) {
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          const float gg = clip_a ? tot[j] * sc_a : tot[j];
          th[r * 5 + j] = th[r * 5 + j] + (-(lr_a * gg));
        }
      }
      const float gg = clip_c ? tot[5] * sc_c : tot[5];
      v[r] = v[r] + (-(lr_c * gg));
    }
  }
  if (tid == 0) {
    step[a] = applied ? st + 1 : st;
    loss_out[a * 2 + 0] += al;
    loss_out[a * 2 + 1] += closs;
  }
  A2C_STAMP(6);
}

template <bool CRITIC_ONLY>
__global__ void __launch_bounds__(256) k_a2c_update(int W, int T, int D, float* __restrict__ theta,
                                                    float* __restrict__ vcrit, const int* __restrict__ tidx,
                                                    const int* __restrict__ ttime, const uint8_t* __restrict__ tact,
                                                    const float* __restrict__ trew, const uint8_t* __restrict__ tdone,
                                                    float gamma, float lam, float ent_coef, float lr_a, float lr_c,
                                                    float max_norm, int* __restrict__ step,
                                                    const int* __restrict__ levels, float* __restrict__ loss_out) {
  extern __shared__ float lds[];
  __shared__ A2CShared sh;
  const int a = blockIdx.x, tid = threadIdx.x;
  A2CStage S;
  S.carve(lds, W, T);
  uint32_t* key = reinterpret_cast<uint32_t*>(lds + A2CStage::floats(W, T));   // [2048]
  float* vec = reinterpret_cast<float*>(key + A2C_SORT_MAX);                    // [W*T][6]
  if (tid == 0) sh.has_last = 0;
  A2C_STAMP(0);
  a2c_load(S, a, W, T, D, vcrit + (size_t)a * D, tidx, ttime, CRITIC_ONLY ? nullptr : tact, trew, tdone);
  const float closs = a2c_gae(S, W, T, gamma, lam, sh.red);
  A2C_STAMP(1);
  a2c_update_body<CRITIC_ONLY>(S, key, vec, sh, closs, a, W, T, D, theta, vcrit, ent_coef, lr_a, lr_c, max_norm, step,
                               levels, loss_out);
}

// ---------------------------------------------------------------------------- the A2C chain in one kernel
// train_a2c_agent's scan (a2c.py:79-125) for one antagonist per 256-thread workgroup, U updates in one launch: per
// update the env chain of the W workers (threads 0..W-1, state in registers across updates, on the precomputed
// state-independent draws of toued_rollout_draws: [T][U x n] uint32x4, update u's worker i at column u*n + i)
// writes the trajectory straight into the LDS stage, then the fused update (the same code as k_a2c_update) runs on
// it and rewrites the touched rows of the agent's actor/critic tables.  The tables stay in global memory (an
// obs_dim = 3201 table pair is 77 KB; two workgroups share a CU's LDS), read back by the next rollout after the
// workgroup barrier.  Bit-identical to toued_rollout_env + toued_a2c_update per update
// (tests/test_gpu_plr.py::test_a2c_chain_matches_launch_per_update).
// SELF (toued_a2c_chain_self, W <= 64): the chain makes its own draws.  The env chain runs in wave 0 and waves 1-3
// are idle there, so during update u they make update u + 1's (the key chain split_at(key_{u+1}, W, w) then two
// splits per step, k_eval_keys' chain, each wave redundantly, and every third step's step_draws) into a per-agent
// double buffer dscr [N][2][T][W] (global, L2-resident); update 0's are made by all four waves before the loop.
// The same draws as toued_rollout_draws over the same keys, so the same trajectories.
template <int NMAX, bool CAND, bool SELF>
__global__ void __launch_bounds__(256) k_a2c_chain(EnvSpec sp, const int* __restrict__ levels, int W, int T, int D,
                                                   int U, float* __restrict__ theta, float* __restrict__ vcrit,
                                                   int* __restrict__ state, const uint4* __restrict__ draws,
                                                   long dstride, const uint32_t* __restrict__ ukeys,
                                                   uint4* __restrict__ dscr, float gamma, float lam, float ent_coef,
                                                   float lr_a, float lr_c, float max_norm, int* __restrict__ step,
                                                   float* __restrict__ loss_out, unsigned* __restrict__ err,
                                                   int test_skip_publish) {
  extern __shared__ float lds[];
  __shared__ A2CShared sh;
#ifndef A2C_PRIO
#define A2C_PRIO 3
#endif
  // the chain is latency-bound and the next chunk's draws (VALU-bound threefry) run beside it on the same SIMDs:
  // its waves take the issue slots first
  __builtin_amdgcn_s_setprio(A2C_PRIO);
  const int a = blockIdx.x, tid = threadIdx.x, n = (int)gridDim.x * W;
  A2CStage S;
  S.carve(lds, W, T);
  uint32_t* key = reinterpret_cast<uint32_t*>(lds + A2CStage::floats(W, T));   // [2048]
  float* vec = reinterpret_cast<float*>(key + A2C_SORT_MAX);                    // [W*T][6]
  const float* tab = theta + (size_t)a * D * 5;
  const float* v = vcrit + (size_t)a * D;
  // env workers: all W in wave 0 (default), or spread over the four waves (A2C_ENV_SPREAD=1, W % 4 == 0: W/4 lanes of
  // each wave, so each wave's row gather touches W/4 cache lines instead of W).  The spread paid before the level's
  // transition table (NPT); since, one wave per agent costs a quarter of the issue slots and the chain runs faster
  // (profiles/r04/a2c_env_spread_r04z.txt: 93.2 vs 95.2 k cycles per update, 1.37 vs 1.50 ms per 32-update launch)
#ifndef A2C_ENV_SPREAD
#define A2C_ENV_SPREAD 0
#endif
  const bool spread = !SELF && A2C_ENV_SPREAD && W % 4 == 0;   // (SELF: the env chain in wave 0 always)
  const int w = spread ? (tid >> 6) * (W / 4) + (tid & 63) : tid;
  const bool env = spread ? (tid & 63) < W / 4 : tid < W;
  const int i = a * W + w;
#ifndef A2C_NPT
#define A2C_NPT 1
#endif
  constexpr bool NPT = A2C_NPT && !CAND;   // the level's transition table in LDS (TrainWorker)
  TrainWorker<NMAX, CAND, NPT> wk;
  if (env) wk.init(sp, levels, a, theta, D, state, n, i);
  if constexpr (NPT) {   // the level's transition table after the update's LDS (toued_a2c_chain sizes it)
    uint16_t* npt = reinterpret_cast<uint16_t*>(vec + (size_t)W * T * A2C_NV);
    if (env) wk.build_npt(npt, w, W);
    wk.npt = npt;
    __syncthreads();
  }
  const int wv = tid >> 6, ln = tid & 63;
  // SELF: update uu's draws of steps t = part (mod nparts) for worker ln into buffer slot `slot`
  auto make_draws = [&](int uu, int slot, int part, int nparts) {
    if (ln >= W) return;
    const uint32_t* kp = ukeys + ((size_t)uu * gridDim.x + a) * 2;
    const int* levp = levels + (size_t)a * LEVEL_WORDS;
    uint2 r = split_at(make_uint2(kp[0], kp[1]), (uint32_t)W, (uint32_t)ln);
    draw4* out = reinterpret_cast<draw4*>(dscr) + (size_t)(a * 2 + slot) * T * W + ln;
    for (int t = 0; t < T; ++t) {
      uint2 sub, sub_env;
      split2(r, r, sub);
      split2(r, r, sub_env);
      if (t % nparts == part) out[(size_t)t * W] = step_draws<NMAX>(levp, sub, sub_env);
    }
  };
  // SELF, during update u's env chain: wave 1 runs update uu = u + 1's key chain into LDS (the update's per-sample
  // vectors, free until the update body), step by step behind a flag; waves 2 and 3 make the draws of alternate steps
  // from it.  Flags hold uu + 1 (updates only grow, so a stale flag never matches); a wait that never ends stops
  // after ~2^20 sleeps instead of hanging and sets TOUED_DEVERR_A2C_DRAW_WAIT in the device error word `err`, which
  // the host turns into an error (toued_device_error_check): the draws it then makes are from stale keys.
  // test_skip_publish = 1 (tests only, TOUED_TEST_A2C_SKIP_PUBLISH): the key wave never publishes step 0 of update 1.
  uint4* kl = reinterpret_cast<uint4*>(vec);   // [T][W] (sub, sub_env)
#ifndef A2C_SELF_PRIO
#define A2C_SELF_PRIO 0
#endif
  auto make_draws_split = [&](int uu, int slot) {
    // the draw waves below the env chain's priority: their threefry fills the issue slots its latency leaves
    __builtin_amdgcn_s_setprio(A2C_SELF_PRIO);
    if (wv == 1) {
      const uint32_t* kp = ukeys + ((size_t)uu * gridDim.x + a) * 2;
      uint2 r = split_at(make_uint2(kp[0], kp[1]), (uint32_t)W, (uint32_t)ln);
      for (int t = 0; t < T; ++t) {
        uint2 sub, sub_env;
        split2(r, r, sub);
        split2(r, r, sub_env);
        if (ln < W) kl[t * W + ln] = make_uint4(sub.x, sub.y, sub_env.x, sub_env.y);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (ln == 0 && !(test_skip_publish && uu == 1 && t == 0))
          __hip_atomic_store(&sh.dflag[t], uu + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    } else {
      const int* levp = levels + (size_t)a * LEVEL_WORDS;
      draw4* out = reinterpret_cast<draw4*>(dscr) + (size_t)(a * 2 + slot) * T * W + ln;
      for (int t = wv - 2; t < T; t += 2) {
        bool seen = false;
        for (int it = 0; it < (1 << 20) && !seen; ++it) {
          seen = __hip_atomic_load(&sh.dflag[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == uu + 1;
          if (!seen) __builtin_amdgcn_s_sleep(1);
        }
        // a vector atomic from one lane (err is a plain device word; never a scalar-cache write)
        if (!seen && ln == 0 && err) atomicOr(err, TOUED_DEVERR_A2C_DRAW_WAIT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (ln < W) {
          const uint4 k4 = kl[t * W + ln];
          out[(size_t)t * W] = step_draws<NMAX>(levp, make_uint2(k4.x, k4.y), make_uint2(k4.z, k4.w));
        }
      }
    }
    __builtin_amdgcn_s_setprio(A2C_PRIO);
  };
  if (SELF) {
    for (int t = tid; t < 64; t += 256) sh.dflag[t] = 0;
    make_draws(0, 0, wv, 4);
    __syncthreads();
  }
  for (int u = 0; u < U; ++u) {
    if (tid == 0) sh.has_last = 0;
    if (u == U - 1) A2C_STAMP(0);
    if (env) {
      wk.load_rows(tab, D);
      const long ds = SELF ? (long)W : dstride;
      const draw4* dr = SELF ? reinterpret_cast<const draw4*>(dscr) + (size_t)(a * 2 + (u & 1)) * T * W + w
                             : reinterpret_cast<const draw4*>(draws) + (size_t)u * n + i;
      draw4 dr0 = {0u, 0u, 0u, 0u};
      if (T > 0) dr0 = dr[0];
      draw4 dr1 = dr0;
      if (T > 1) dr1 = dr[ds];
      for (int t = 0; t < T; ++t) {
        const draw4 d = dr0;
        dr0 = dr1;
        if (t + 2 < T) dr1 = dr[(size_t)(t + 2) * ds];
        int oi, ot, action;
        float rew;
        bool done;
        wk.step(sp, tab, d, oi, ot, action, rew, done);
        S.ix[t * W + w] = oi;
        S.cc[t * W + w] = (float)ot * 0.001f;
        S.act[t * W + w] = (uint8_t)action;
        S.rw[t * W + w] = rew;
        S.nd[t * W + w] = done ? 0.0f : 1.0f;
      }
      S.ix[T * W + w] = wk.idx;
      S.cc[T * W + w] = (float)wk.s.time * 0.001f;
    } else if (SELF && wv >= 1 && u + 1 < U) {
#ifndef A2C_SELF_SPLIT
#define A2C_SELF_SPLIT 1
#endif
      if (A2C_SELF_SPLIT)
        make_draws_split(u + 1, (u + 1) & 1);   // beside wave 0's env chain
      else
        make_draws(u + 1, (u + 1) & 1, wv - 1, 3);
    }
    if (u == U - 1) A2C_STAMP(7);
    __syncthreads();
    A2C_FINE(0);
    // V(obs) for every observation (a2c_load's gather) as its own phase: loading each step's V inside the env chain
    // instead (behind the row gather, stored a step later) made the chain 48 -> 69 k cycles per update -- a second
    // 64-lane gather per step doubles the chain's cache-line lookups (profiles/r04/a2c_stamps_fine_r04i.log)
    gather_values(S, v, D, (T + 1) * W);
    __syncthreads();
    A2C_FINE(1);
    const float closs = a2c_gae(S, W, T, gamma, lam, sh.red);
    A2C_FINE(5);
    if (u == U - 1) A2C_STAMP(1);
    a2c_update_body<false>(S, key, vec, sh, closs, a, W, T, D, theta, vcrit, ent_coef, lr_a, lr_c, max_norm, step,
                           levels, loss_out);
    __syncthreads();   // the rewritten rows and the step counter before the next rollout reads them
  }
  if (env) store_state<NMAX>(state, n, i, wk.s);
}

static size_t a2c_update_lds(int W, int T) {
  return (A2CStage::floats(W, T) + A2C_SORT_MAX + (size_t)W * T * A2C_NV) * sizeof(float);
}

// util/metrics.py:17-38 gae() over n = N * W independent workers: one lane per worker runs the reverse scan over T
// (the recurrence carries one float; T = 20 dependent FMAs per lane), reading value [N][T+1][W], reward and done
// [N][T][W] and writing adv / target [N][T][W] -- each (t, agent) row of W workers is one coalesced 4 W-byte access
// per wave.  The reference's operation order, in f32 with no contraction: value_diff = (gamma v[t+1]) (1 - d) - v[t];
// delta = r + value_diff; gae = delta + ((gamma lambda) (1 - d)) gae; target = gae + v[t].  17 B per (worker, t).
__global__ void __launch_bounds__(256) k_gae(int n, int W, int T, const float* __restrict__ value,
                                              const float* __restrict__ reward, const uint8_t* __restrict__ done,
                                              float gamma, float gl, float* __restrict__ adv,
                                              float* __restrict__ target) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int a = i / W, w = i - a * W;
  const long vb = (long)a * (T + 1) * W + w, sb = (long)a * T * W + w;
  float vn = __builtin_nontemporal_load(value + vb + (long)T * W);
  float g = 0.0f;
#pragma unroll 4
  for (int t = T - 1; t >= 0; --t) {
    const float v = __builtin_nontemporal_load(value + vb + (long)t * W);
    const float nd = __builtin_nontemporal_load(done + sb + (long)t * W) ? 0.0f : 1.0f;
    const float r = __builtin_nontemporal_load(reward + sb + (long)t * W);
    const float delta = r + (gamma * vn * nd - v);
    g = delta + gl * nd * g;
    __builtin_nontemporal_store(g, adv + sb + (long)t * W);
    __builtin_nontemporal_store(g + v, target + sb + (long)t * W);
    vn = v;
  }
}

// The (row, sample) sort of the sorted-segment kernels on its own, for its parity test: block b sorts keys[b][2048]
// with NT threads (256: the A2C kernels, 512: agent.hip's k_rows_sorted)
template <int NT>
__global__ void __launch_bounds__(NT) k_sort_keys2048(const uint32_t* __restrict__ keys, uint32_t* __restrict__ out) {
  __shared__ uint32_t key[2048];
  const size_t b = (size_t)blockIdx.x * 2048;
  for (int i = threadIdx.x; i < 2048; i += NT) key[i] = keys[b + i];
  sort2048_reg<NT>(key, threadIdx.x);
  for (int i = threadIdx.x; i < 2048; i += NT) out[b + i] = key[i];
}

extern "C" {

int toued_gae(int N, int W, int T, const float* value, const float* reward, const uint8_t* done, float gamma,
              float gamma_lambda, float* adv, float* target, hipStream_t stream) {
  TOUED_REQUIRE(N >= 0 && W >= 1 && T >= 1 && (long)N * W < (1L << 31), "toued_gae: N=%d W=%d T=%d", N, W, T);
  const int n = N * W;
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_gae, dim3((n + 255) / 256), dim3(256), 0, stream, n, W, T, value, reward, done, gamma,
                     gamma_lambda, adv, target);
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_sort_keys2048(const uint32_t* keys, uint32_t* out, int nblocks, int threads, hipStream_t stream) {
  TOUED_REQUIRE(nblocks >= 0 && (threads == 256 || threads == 512), "toued_sort_keys2048: nblocks=%d threads=%d",
                nblocks, threads);
  if (nblocks == 0) return 0;
  TOUED_REQUIRE(keys && out, "toued_sort_keys2048: null buffer");
  if (threads == 256)
    hipLaunchKernelGGL(k_sort_keys2048<256>, dim3(nblocks), dim3(256), 0, stream, keys, out);
  else
    hipLaunchKernelGGL(k_sort_keys2048<512>, dim3(nblocks), dim3(512), 0, stream, keys, out);
  TOUED_CHECK_LAUNCH();
  return 0;
}

#ifdef A2C_STAMPS_FINE
int toued_dbg_a2c_fine(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_a2c_fine), sizeof(g_a2c_fine)) == hipSuccess ? 0 : 1;
}
#endif
#ifdef A2C_STAMPS
int toued_dbg_a2c_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_a2c_stamps), sizeof(g_a2c_stamps)) == hipSuccess ? 0 : 1;
}
#endif

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
  const size_t lds = A2CStage::floats(W, T) * sizeof(float);
  TOUED_REQUIRE(lds <= 64 * 1024, "toued_a2c_grad: W*T too large for LDS");
  if (N == 0) return 0;
  hipLaunchKernelGGL(k_a2c_grad, dim3(N), dim3(256), lds, stream, W, T, D, theta, vcrit, tidx, ttime, tact, trew,
                     tdone, gamma, lam, ent_coef, Ga, Gv, loss_out);
  TOUED_CHECK_LAUNCH();
  return 0;
}

// 1 when the deterministic fused A2C update supports these sizes (W*T <= 2048, rows < 2^21; else use
// toued_a2c_grad + toued_a2c_apply)
int toued_a2c_update_fits(int W, int T, int D) {
  return W > 0 && T > 0 && D > 1 && W * T <= A2C_SORT_MAX && D < (1 << 21) && a2c_update_lds(W, T) <= 150 * 1024
             ? 1 : 0;
}

int toued_a2c_update(int N, int W, int T, int D, float* theta, float* vcrit, const int* tidx, const int* ttime,
                     const uint8_t* tact, const float* trew, const uint8_t* tdone, float gamma, float lam,
                     float ent_coef, float lr_a, float lr_c, float max_norm, int* step, const int* levels,
                     float* loss_out, hipStream_t stream) {
  TOUED_REQUIRE(toued_a2c_update_fits(W, T, D), "toued_a2c_update: D=%d W=%d T=%d unsupported (W*T <= %d; use "
                "grad + apply)", D, W, T, A2C_SORT_MAX);
  TOUED_REQUIRE((double)N * D * 20.0 < 4294967295.0, "toued_a2c_update: actor tables (%d x %d rows) exceed 4 GiB", N, D);
  const size_t lds = a2c_update_lds(W, T);
  if (N == 0) return 0;
  static bool attr_set = false;
  if (!attr_set) {
    TOUED_REQUIRE(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_a2c_update<false>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024) == hipSuccess,
                  "toued_a2c_update: cannot raise the dynamic LDS limit");
    attr_set = true;
  }
  hipLaunchKernelGGL(k_a2c_update<false>, dim3(N), dim3(256), lds, stream, W, T, D, theta, vcrit, tidx, ttime, tact,
                     trew, tdone, gamma, lam, ent_coef, lr_a, lr_c, max_norm, step, levels, loss_out);
  TOUED_CHECK_LAUNCH();
  return 0;
}

// 1 when toued_a2c_chain supports these sizes: the fused update's and W <= 256 workers (one per thread)
int toued_a2c_chain_fits(int W, int T, int D) { return W <= 256 && toued_a2c_update_fits(W, T, D) ? 1 : 0; }
// 1 when toued_a2c_chain_self does: the env chain in one wave (W <= 64) and one draw flag per step (T <= 64)
int toued_a2c_chain_self_fits(int W, int T, int D) {
  return W >= 1 && W <= 64 && T >= 1 && T <= 64 && toued_a2c_chain_fits(W, T, D) ? 1 : 0;
}

// U A2C updates (rollout + fused update each) of N antagonists in one launch: theta [N][D][5], vcrit [N][D], step
// [N], state [S_FIELDS][N*W] updated in place, loss_out [N][2] accumulated; draws = toued_rollout_draws' output for
// U batches ([T][dstride] uint32x4, update u's worker i at column u*N*W + i)
int toued_a2c_chain(EnvSpec sp, const int* levels, int N, int W, int T, int D, int U, float* theta, float* vcrit,
                    int* state, const uint32_t* draws, long dstride, float gamma, float lam, float ent_coef, float lr_a,
                    float lr_c, float max_norm, int* step, float* loss_out, hipStream_t stream) {
  TOUED_REQUIRE(sp.tabular && sp.n_max >= 1 && sp.n_max <= 5 && sp.max_grid >= 1 && sp.max_grid * sp.max_grid <= 256,
                "toued_a2c_chain: tabular env spec required");
  TOUED_REQUIRE(N >= 0 && U >= 0 && toued_a2c_chain_fits(W, T, D), "toued_a2c_chain: N=%d U=%d W=%d T=%d D=%d unsupported",
                N, U, W, T, D);
  TOUED_REQUIRE(D == sp.max_grid * sp.max_grid * (1 << sp.n_max) + 1, "toued_a2c_chain: D=%d != obs_dim", D);
  TOUED_REQUIRE((double)N * D * 20.0 < 4294967295.0, "toued_a2c_chain: actor tables (%d x %d rows) exceed 4 GiB", N, D);
  TOUED_REQUIRE(dstride >= (long)U * N * W, "toued_a2c_chain: draw stride %ld < %ld", dstride, (long)U * N * W);
  if (N == 0 || U == 0) return 0;
  // the env chain's row gathers: the chosen row after the choice (default: 68k vs 94k cycles per 20-step chain,
  // profiles/r03/a2c_stamps_rows.log) or the five candidate rows ahead of it (TOUED_TRAIN_ROWS=cand; bit-identical)
  static const bool cand = getenv("TOUED_TRAIN_ROWS") && strcmp(getenv("TOUED_TRAIN_ROWS"), "cand") == 0;
  // + the transition table of the default (non-candidate) worker: G2 x 5 u16
  const size_t lds = a2c_update_lds(W, T) + (cand ? 0 : ((size_t)sp.max_grid * sp.max_grid * 5 * 2 + 3) / 4 * 4);
  static bool attr_set[2][6] = {};
#define TOUED_A2C_CHAIN_LAUNCH(NM, CD)                                                                               \
  {                                                                                                                   \
    if (!attr_set[CD][NM]) {                                                                                          \
      TOUED_REQUIRE(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_a2c_chain<NM, CD, false>),                   \
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024) == hipSuccess,        \
                    "toued_a2c_chain: cannot raise the dynamic LDS limit");                                           \
      attr_set[CD][NM] = true;                                                                                        \
    }                                                                                                                 \
    hipLaunchKernelGGL((k_a2c_chain<NM, CD, false>), dim3(N), dim3(256), lds, stream, sp, levels, W, T, D, U, theta,  \
                       vcrit, state, reinterpret_cast<const uint4*>(draws), dstride, nullptr, nullptr, gamma, lam,    \
                       ent_coef, lr_a, lr_c, max_norm, step, loss_out, nullptr, 0);                                   \
  }
#define TOUED_A2C_CHAIN_CASE(NM)                                                                                     \
  case NM:                                                                                                            \
    if (cand) TOUED_A2C_CHAIN_LAUNCH(NM, true) else TOUED_A2C_CHAIN_LAUNCH(NM, false)                                \
    break;
  switch (sp.n_max) {
    TOUED_A2C_CHAIN_CASE(1)
    TOUED_A2C_CHAIN_CASE(2)
    TOUED_A2C_CHAIN_CASE(3)
    TOUED_A2C_CHAIN_CASE(4)
    TOUED_A2C_CHAIN_CASE(5)
    default: break;
  }
#undef TOUED_A2C_CHAIN_LAUNCH
#undef TOUED_A2C_CHAIN_CASE
  TOUED_CHECK_LAUNCH();
  return 0;
}

// The same chain making its own draws from the U update keys (keys [U][N][2], toued_key_chain's output):
// scratch = u32 [N][2][T][W][4].  W <= 64 (the env chain in one wave).  Bit-identical to toued_rollout_draws +
// toued_a2c_chain over the same keys.
int toued_a2c_chain_self(EnvSpec sp, const int* levels, int N, int W, int T, int D, int U, float* theta, float* vcrit,
                         int* state, const uint32_t* keys, uint32_t* scratch, float gamma, float lam, float ent_coef,
                         float lr_a, float lr_c, float max_norm, int* step, float* loss_out, hipStream_t stream) {
  TOUED_REQUIRE(sp.tabular && sp.n_max >= 1 && sp.n_max <= 5 && sp.max_grid >= 1 && sp.max_grid * sp.max_grid <= 256,
                "toued_a2c_chain_self: tabular env spec required");
  TOUED_REQUIRE(N >= 0 && U >= 0 && toued_a2c_chain_self_fits(W, T, D),
                "toued_a2c_chain_self: N=%d U=%d W=%d T=%d D=%d unsupported", N, U, W, T, D);
  TOUED_REQUIRE(D == sp.max_grid * sp.max_grid * (1 << sp.n_max) + 1, "toued_a2c_chain_self: D=%d != obs_dim", D);
  TOUED_REQUIRE((double)N * D * 20.0 < 4294967295.0, "toued_a2c_chain_self: actor tables (%d x %d rows) exceed 4 GiB",
                N, D);
  TOUED_REQUIRE(keys && scratch, "toued_a2c_chain_self: null keys / scratch");
  unsigned* err = toued::dev_err_word();
  TOUED_REQUIRE(err, "toued_a2c_chain_self: call toued_device_error_check once first (it allocates the device error "
                "word, outside any graph capture)");
  if (N == 0 || U == 0) return 0;
  const int skip_pub = getenv("TOUED_TEST_A2C_SKIP_PUBLISH") && atoi(getenv("TOUED_TEST_A2C_SKIP_PUBLISH"));
  const size_t lds = a2c_update_lds(W, T) + ((size_t)sp.max_grid * sp.max_grid * 5 * 2 + 3) / 4 * 4;
  static bool attr_set[6] = {};
#define TOUED_A2C_SELF_CASE(NM)                                                                                      \
  case NM:                                                                                                            \
    if (!attr_set[NM]) {                                                                                              \
      TOUED_REQUIRE(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_a2c_chain<NM, false, true>),                 \
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024) == hipSuccess,        \
                    "toued_a2c_chain_self: cannot raise the dynamic LDS limit");                                      \
      attr_set[NM] = true;                                                                                            \
    }                                                                                                                 \
    hipLaunchKernelGGL((k_a2c_chain<NM, false, true>), dim3(N), dim3(256), lds, stream, sp, levels, W, T, D, U, theta, \
                       vcrit, state, nullptr, 0L, keys, reinterpret_cast<uint4*>(scratch), gamma, lam, ent_coef,      \
                       lr_a, lr_c, max_norm, step, loss_out, err, skip_pub);                                          \
    break;
  switch (sp.n_max) {
    TOUED_A2C_SELF_CASE(1)
    TOUED_A2C_SELF_CASE(2)
    TOUED_A2C_SELF_CASE(3)
    TOUED_A2C_SELF_CASE(4)
    TOUED_A2C_SELF_CASE(5)
    default: break;
  }
#undef TOUED_A2C_SELF_CASE
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_value_critic_update(int N, int W, int T, int D, float* vcrit, const int* tidx, const int* ttime,
                              const float* trew, const uint8_t* tdone, float gamma, float lam, float lr,
                              float max_norm, int* vstep, float* loss_out, hipStream_t stream) {
  TOUED_REQUIRE(toued_a2c_update_fits(W, T, D), "toued_value_critic_update: D=%d W=%d T=%d unsupported (W*T <= %d)",
                D, W, T, A2C_SORT_MAX);
  if (N == 0) return 0;
  const size_t lds = a2c_update_lds(W, T);
  static bool attr_set = false;
  if (!attr_set) {
    TOUED_REQUIRE(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_a2c_update<true>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024) == hipSuccess,
                  "toued_value_critic_update: cannot raise the dynamic LDS limit");
    attr_set = true;
  }
  hipLaunchKernelGGL(k_a2c_update<true>, dim3(N), dim3(256), lds, stream, W, T, D, nullptr, vcrit, tidx, ttime,
                     nullptr, trew, tdone, gamma, lam, 0.0f, 0.0f, lr, max_norm, vstep, nullptr, loss_out);
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
