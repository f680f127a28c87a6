// C++/OpenMP CPU restatement of the rollout hot path -- TEST INFRASTRUCTURE / CPU BASELINE ONLY.
//
// The second CPU baseline of BASELINE.md §2 ("a C++/OpenMP (g++ -O3) build of the same step, rollout and
// GAE code, using compact observations"): the GridWorld step and auto-reset, the batched rollout with the
// linear-softmax tabular actor, and GAE, as plain scalar host code, one OpenMP thread per env worker block.
// It follows the numpy oracle line by line (oracle/gridworld.py, oracle/rollout.py, oracle/jaxrand.py,
// oracle/pmath.py), which in turn cite the reference:
//   environments/gridworld/gridworld.py:72-211  step_env / _get_next_pos / _get_valid_obj_idxs / reset_env
//   gymnax 0.0.6 Environment.step               key, key_reset = split(key); select(done, reset, step)
//   environments/rollout.py:38-102              batch_reset / batch_rollout / policy_step
//   models/agent.py:7-17                        softmax(obs @ W) with the one-hot obs in compact form
//   util/metrics.py:17-38                       gae
// and jax 0.4.13's threefry2x32 PRNG.  tests/test_oracle_cpu.py checks it bit-exact against the numpy oracle.
// Levels come in the packed int32[64] layout of oracle/levels.pack_levels; the env state is the SoA
// int32[12][n] layout of the device (fields time, pos, exists bitmask, early_term, obj_poss[8]).
// Built by oracle/cpu/__init__.py (g++ -O3 -fopenmp -ffp-contract=off); never linked by the product.
#include <math.h>
#include <cmath>
#include <stdint.h>
#include <string.h>
#include <omp.h>
#include <algorithm>
#include <vector>

namespace {

enum { L_MAX_STEPS = 0, L_GRID = 1, L_START = 2, L_NOBJS = 3, L_RANDRESP = 4, L_OBJ_IDS = 8, L_STATIC = 16,
       L_REW = 24, L_PTERM = 32, L_PRESP = 40, L_WALLS = 48, LW = 80 };
enum { S_TIME = 0, S_POS = 1, S_EXISTS = 2, S_TERM = 3, S_OBJ = 4 };

struct Key { uint32_t a, b; };

inline uint32_t rotl(uint32_t v, int r) { return (v << r) | (v >> (32 - r)); }

// threefry2x32 with 20 rounds (Random123; jax/_src/prng.py)
inline void threefry(Key k, uint32_t x0, uint32_t x1, uint32_t& y0, uint32_t& y1) {
  const uint32_t ks[3] = {k.a, k.b, k.a ^ k.b ^ 0x1BD11BDAu};
  static const int R[2][4] = {{13, 15, 26, 6}, {17, 29, 16, 24}};
  x0 += ks[0];
  x1 += ks[1];
  for (int i = 0; i < 5; ++i) {
    for (int j = 0; j < 4; ++j) {
      x0 += x1;
      x1 = rotl(x1, R[i & 1][j]);
      x1 ^= x0;
    }
    x0 += ks[(i + 1) % 3];
    x1 += ks[(i + 2) % 3] + (uint32_t)(i + 1);
  }
  y0 = x0;
  y1 = x1;
}

// element j of threefry_2x32(key, iota(count)) (odd counts padded with one zero counter)
inline uint32_t bits_at(Key k, uint32_t count, uint32_t j) {
  const uint32_t h = (count + 1) / 2;
  const uint32_t b = j < h ? j : j - h;
  const uint32_t hi = b + h;
  uint32_t y0, y1;
  threefry(k, b, hi < count ? hi : 0u, y0, y1);
  return j < h ? y0 : y1;
}

inline Key split_at(Key k, uint32_t num, uint32_t i) { return {bits_at(k, 2 * num, 2 * i), bits_at(k, 2 * num, 2 * i + 1)}; }

inline float unit_of(uint32_t bits) {
  uint32_t u = (bits >> 9) | 0x3F800000u;
  float f;
  memcpy(&f, &u, 4);
  return f - 1.0f;
}

inline float uniform_of(uint32_t bits, float lo, float hi) {
  const float v = unit_of(bits) * (hi - lo) + lo;
  return v > lo ? v : lo;
}

inline float as_f(int v) { float f; memcpy(&f, &v, 4); return f; }
inline float pow2i(int k) { uint32_t u = (uint32_t)(k + 127) << 23; float f; memcpy(&f, &u, 4); return f; }

// oracle/pmath.py exp: Cody-Waite reduction, degree-7 Taylor polynomial, two-step scaling
float pexp(float x) {
  if (x != x) return x;
  if (x > 88.72283905206835f) return INFINITY;
  if (x < -103.972084f) return 0.0f;
  const float k = rintf(x * 1.44269504088896341f);
  float r = x - k * 0.693145751953125f;
  r = r - k * 1.428606765330187045e-06f;
  const float C[8] = {1.0f, 1.0f, 0.5f, (float)(1.0 / 6.0), (float)(1.0 / 24.0), (float)(1.0 / 120.0),
                      (float)(1.0 / 720.0), (float)(1.0 / 5040.0)};
  float p = C[7];
  for (int i = 6; i >= 0; --i) p = p * r + C[i];
  int ki = std::min(200, std::max(-200, (int)k));
  const int k1 = (int)floor(ki / 2.0), k2 = ki - k1;
  return (p * pow2i(std::min(127, std::max(-126, k1)))) * pow2i(std::min(127, std::max(-126, k2)));
}

// oracle/pmath.py log (musl logf reduction)
float plog(float x) {
  if (x != x) return x;
  if (x == 0.0f) return -INFINITY;
  if (x < 0.0f) return NAN;
  if (isinf(x)) return x;
  const bool sub = x < 1.17549435e-38f;
  const float xs = sub ? x * 8388608.0f : x;
  uint32_t bits;
  memcpy(&bits, &xs, 4);
  int e = (int)((bits >> 23) & 0xFFu) - 127;
  if (sub) e -= 23;
  uint32_t mb = (bits & 0x7FFFFFu) | 0x3F800000u;
  float m;
  memcpy(&m, &mb, 4);
  if (m > 1.41421356237f) { m = m * 0.5f; e += 1; }
  const float f = m - 1.0f;
  const float s = f / (2.0f + f);
  const float z = s * s, w = z * z;
  const float t1 = w * (0.40000972152f + w * 0.24279078841f);
  const float t2 = z * (0.66666662693f + w * 0.28498786688f);
  const float R = t2 + t1;
  const float hfsq = 0.5f * f * f;
  const float dk = (float)e;
  return dk * 0.693145751953125f - ((hfsq - (s * (hfsq + R) + dk * 1.428606765330187045e-06f)) - f);
}

struct Spec { int max_grid, n_max, n_types, tabular; };

struct State { int time, pos, exists, early_term; int obj[8]; };

inline bool wall(const int* lev, int c) { return ((uint32_t)lev[L_WALLS + (c >> 5)] >> (c & 31)) & 1u; }

// gridworld.py:138-146
int next_pos(const int* lev, int pos, int a) {
  const int g = lev[L_GRID];
  const int top = pos < g, bottom = pos >= g * (g - 1), left = pos % g == 0, right = pos % g == g - 1;
  const int step = (a == 0) * (1 - top) * -g + (a == 1) * (1 - bottom) * g + (a == 2) * (1 - left) * -1 +
                   (a == 3) * (1 - right) * 1;
  const int nxt = pos + step;
  return wall(lev, nxt) ? pos : nxt;
}

// gridworld.py:149-155 (cells equal to a value of the bool walls array are excluded: SURVEY B.5), plus the
// caller's extra exclusions
std::vector<char> valid_cells(const Spec& sp, const int* lev, int pos, const int* excl, int nexcl) {
  const int G2 = sp.max_grid * sp.max_grid, g = lev[L_GRID];
  bool has_t = false, has_f = false;
  for (int c = 0; c < G2; ++c) (wall(lev, c) ? has_t : has_f) = true;
  std::vector<char> v(G2);
  for (int c = 0; c < G2; ++c) {
    bool ok = c != pos && c < g * g && !((c == 0 && has_f) || (c == 1 && has_t));
    for (int i = 0; i < nexcl; ++i) ok = ok && c != excl[i];
    v[c] = ok;
  }
  return v;
}

// choice(key, G2, (n,), replace=False, p=valid/count): stable argsort of -gumbel - log(p)
void choice_noreplace(Key key, const std::vector<char>& valid, int n, int* out) {
  const int G2 = (int)valid.size();
  int cnt = 0;
  for (char c : valid) cnt += c;
  const float pv = 1.0f / (float)cnt;
  std::vector<std::pair<float, int>> g(G2);
  for (int c = 0; c < G2; ++c) {
    const float u = uniform_of(bits_at(key, (uint32_t)G2, (uint32_t)c), 1.17549435e-38f, 1.0f);
    const float gm = -plog(-plog(u));
    const float lp = valid[c] ? plog(pv) : -INFINITY;
    g[c] = {-gm - lp, c};
  }
  std::stable_sort(g.begin(), g.end(), [](const std::pair<float, int>& x, const std::pair<float, int>& y) {
    return x.first < y.first;
  });
  for (int i = 0; i < n; ++i) out[i] = g[i].second;
}

// gridworld.py:157-182
void reset_env(const Spec& sp, const int* lev, Key key, State& s) {
  const int G2 = sp.max_grid * sp.max_grid, n = sp.n_max;
  s.time = 0;
  s.pos = lev[L_START];
  s.early_term = 0;
  s.exists = 0;
  for (int i = 0; i < n; ++i) {
    s.obj[i] = lev[L_STATIC + i];
    if (i < lev[L_NOBJS]) s.exists |= 1 << i;
  }
  if (!sp.tabular && lev[L_RANDRESP]) {
    const Key obj_key = split_at(key, 2, 0);
    int pick[8];
    choice_noreplace(obj_key, valid_cells(sp, lev, s.pos, nullptr, 0), n, pick);
    for (int i = 0; i < n; ++i) s.obj[i] = pick[i];
  }
  for (int i = 0; i < n; ++i) s.obj[i] += lev[L_OBJ_IDS + i] * G2;
}

// gridworld.py:72-136 + the gymnax auto-reset; every key derived as the reference does
void env_step(const Spec& sp, const int* lev, Key key, State& s, int action, float& reward, bool& done) {
  const int G2 = sp.max_grid * sp.max_grid, n = sp.n_max;
  const Key key_s = split_at(key, 2, 0), key_r = split_at(key, 2, 1);
  const Key term_key = split_at(key_s, 3, 0), respawn_key = split_at(key_s, 3, 1), obj_key = split_at(key_s, 3, 2);
  const int pos = next_pos(lev, s.pos, action);
  int old[8], collected = 0, respawn = 0;
  for (int i = 0; i < n; ++i) {
    old[i] = s.obj[i] - lev[L_OBJ_IDS + i] * G2;
    if (((s.exists >> i) & 1) && old[i] == pos) collected |= 1 << i;
    if (unit_of(bits_at(respawn_key, (uint32_t)n, (uint32_t)i)) < as_f(lev[L_PRESP + i])) respawn |= 1 << i;
  }
  int exists = s.exists | respawn;
  int newpos[8];
  for (int i = 0; i < n; ++i) newpos[i] = old[i];
  if (!sp.tabular && lev[L_RANDRESP]) {
    int pick[8];
    choice_noreplace(obj_key, valid_cells(sp, lev, pos, old, n), n, pick);
    for (int i = 0; i < n; ++i)
      if (!((s.exists >> i) & 1) && ((respawn >> i) & 1)) newpos[i] = pick[i];
  }
  const int used = (1 << lev[L_NOBJS]) - 1;
  exists = exists & ~collected & used;
  float p_t = 0.0f, rew = 0.0f;
  for (int i = 0; i < n; ++i) {
    const float ci = ((collected >> i) & 1) ? 1.0f : 0.0f;
    p_t = p_t + as_f(lev[L_PTERM + i]) * ci;
    rew = rew + as_f(lev[L_REW + i]) * ci;
  }
  rew = rew + 0.0f;
  const bool term = unit_of(bits_at(term_key, 1, 0)) < p_t || s.early_term;
  const int time = s.time + 1;
  done = time >= lev[L_MAX_STEPS] || term;
  reward = rew;
  if (done) {
    reset_env(sp, lev, key_r, s);
  } else {
    s.time = time;
    s.pos = pos;
    s.exists = exists;
    s.early_term = term;
    for (int i = 0; i < n; ++i) s.obj[i] = newpos[i] + lev[L_OBJ_IDS + i] * G2;
  }
}

// softmax(W[idx] + (f32(t) * 0.001) W[D-1]) (oracle/rollout.py softmax: max-shift, portable exp, sequential sum)
void probs5(const float* tab, int D, int idx, int t, float* p) {
  const float c = (float)t * 0.001f;
  float l[5], m = -INFINITY, e[5], s;
  for (int j = 0; j < 5; ++j) { l[j] = tab[(size_t)idx * 5 + j] + c * tab[(size_t)(D - 1) * 5 + j]; m = std::max(m, l[j]); }
  for (int j = 0; j < 5; ++j) e[j] = pexp(l[j] - m);
  s = e[0];
  for (int j = 1; j < 5; ++j) s = s + e[j];
  for (int j = 0; j < 5; ++j) p[j] = e[j] / s;
}

// choice(key, 5, p=p) with jnp.cumsum's associative-scan order
int choice5(Key key, const float* p) {
  const float c0 = p[0], c1 = p[0] + p[1], c2 = c1 + p[2], c3 = c1 + (p[2] + p[3]), c4 = c3 + p[4];
  const float r = c4 * (1.0f - unit_of(bits_at(key, 1, 0)));
  return (c0 < r) + (c1 < r) + (c2 < r) + (c3 < r) + (c4 < r);
}

}  // namespace

extern "C" {

int toued_cpu_threads(void) { return omp_get_max_threads(); }

// RolloutWrapper.batch_rollout for N agents x W workers (rollout.py:45-102); state SoA [12][N*W] in place.
int toued_cpu_rollout(int max_grid, int n_max, int n_types, int tabular, const int* levels, const float* theta, int D,
                      const uint32_t* agent_keys, int* state, int T, int W, int N, int* traj_idx, int* traj_time,
                      uint8_t* traj_action, float* traj_reward, uint8_t* traj_done, float* cum_return) {
  const Spec sp{max_grid, n_max, n_types, tabular};
  const int n = N * W;
#pragma omp parallel for schedule(static)
  for (int i = 0; i < n; ++i) {
    const int a = i / W, w = i - a * W;
    const int* lev = levels + (size_t)a * LW;
    const float* tab = theta + (size_t)a * D * 5;
    State s;
    s.time = state[S_TIME * n + i];
    s.pos = state[S_POS * n + i];
    s.exists = state[S_EXISTS * n + i];
    s.early_term = state[S_TERM * n + i];
    for (int k = 0; k < n_max; ++k) s.obj[k] = state[(S_OBJ + k) * n + i];
    Key rng = split_at({agent_keys[2 * a], agent_keys[2 * a + 1]}, (uint32_t)W, (uint32_t)w);
    float cum = 0.0f, valid = 1.0f;
    const size_t bo = (size_t)a * (T + 1) * W + w, bt = (size_t)a * T * W + w;
    for (int t = 0; t < T; ++t) {
      const int idx = s.pos + max_grid * max_grid * s.exists, tm = s.time;
      const Key sub_a = split_at(rng, 2, 1);
      rng = split_at(rng, 2, 0);
      float p[5];
      probs5(tab, D, idx, tm, p);
      const int act = choice5(sub_a, p);
      const Key sub_e = split_at(rng, 2, 1);
      rng = split_at(rng, 2, 0);
      float r;
      bool d;
      env_step(sp, lev, sub_e, s, act, r, d);
      cum = cum + r * valid;
      valid = valid * (d ? 0.0f : 1.0f);
      if (traj_idx) {
        traj_idx[bo + (size_t)t * W] = idx;
        traj_time[bo + (size_t)t * W] = tm;
        traj_action[bt + (size_t)t * W] = (uint8_t)act;
        traj_reward[bt + (size_t)t * W] = r;
        traj_done[bt + (size_t)t * W] = d;
      }
    }
    if (traj_idx) {
      traj_idx[bo + (size_t)T * W] = s.pos + max_grid * max_grid * s.exists;
      traj_time[bo + (size_t)T * W] = s.time;
    }
    state[S_TIME * n + i] = s.time;
    state[S_POS * n + i] = s.pos;
    state[S_EXISTS * n + i] = s.exists;
    state[S_TERM * n + i] = s.early_term;
    for (int k = 0; k < n_max; ++k) state[(S_OBJ + k) * n + i] = s.obj[k];
    if (cum_return) cum_return[i] = cum;
  }
  return 0;
}

// gae (util/metrics.py:17-38) per worker over a rollout in the layout above, V = vcrit[a][idx] + c vcrit[a][D-1]
// (the linear value critic on the compact obs): adv, target [N][W][T].
int toued_cpu_gae(const float* vcrit, int D, const int* traj_idx, const int* traj_time, const float* traj_reward,
                  const uint8_t* traj_done, int T, int W, int N, float gamma, float lam, float* adv, float* target) {
#pragma omp parallel for schedule(static)
  for (int i = 0; i < N * W; ++i) {
    const int a = i / W, w = i - a * W;
    const float* v = vcrit + (size_t)a * D;
    const size_t bo = (size_t)a * (T + 1) * W + w, bt = (size_t)a * T * W + w;
    auto V = [&](int t) { return v[traj_idx[bo + (size_t)t * W]] + (float)traj_time[bo + (size_t)t * W] * 0.001f * v[D - 1]; };
    float g = 0.0f, vn = V(T);
    for (int t = T - 1; t >= 0; --t) {
      const float vv = V(t), nd = traj_done[bt + (size_t)t * W] ? 0.0f : 1.0f;
      const float delta = traj_reward[bt + (size_t)t * W] + (gamma * vn * nd - vv);
      g = delta + gamma * lam * nd * g;
      adv[(size_t)i * T + t] = g;
      target[(size_t)i * T + t] = g + vv;
      vn = vv;
    }
  }
  return 0;
}

// a2c_agent_train_step (agents/a2c.py:19-76) for N agents over one rollout in the layout above, as oracle/a2c.py
// restates it, with closed-form gradients of the linear tables (one OpenMP thread per agent):
//   critic: V = vcrit[idx] + 0.001 t vcrit[D-1]; GAE per worker; loss mean_w mean_t (target - V)^2
//           -> dL/dV_{w,t} = -2 (target - V) / (W T) for t < T (the bootstrap V_T is stop-gradient);
//   actor:  per worker -mean_t log(pi_a + 1e-8) * mean_t adv_n (the [T] x [T,1] broadcast) minus
//           entropy_coeff * (-mean_t sum_b q_b log q_b), q = pi + 1e-8, adv_n normalised over the agent's [W, T];
//           d/dl_c through the softmax: p_c (g_c - sum_b g_b p_b) with g_b the loss's derivative w.r.t. p_b;
//   optax clip_by_global_norm (each table's own norm) -> SGD; the update is discarded past the lifetime
//   (a2c.py:82-86).  theta [N][D][5], vcrit [N][D], step [N] updated in place; loss [N][2] (actor, critic).
int toued_cpu_a2c_update(float* theta, float* vcrit, int* step, const int* levels, int D, const int* traj_idx,
                         const int* traj_time, const uint8_t* traj_action, const float* traj_reward,
                         const uint8_t* traj_done, int T, int W, int N, float gamma, float lam, float entropy_coeff,
                         float actor_lr, float critic_lr, float max_norm, float* loss) {
  const float EPS = 1e-8f;
#pragma omp parallel for schedule(dynamic)
  for (int a = 0; a < N; ++a) {
    float* th = theta + (size_t)a * D * 5;
    float* vc = vcrit + (size_t)a * D;
    std::vector<float> ga((size_t)D * 5, 0.0f), gc(D, 0.0f), adv((size_t)W * T), tgt((size_t)W * T), vv((size_t)W * T);
    double asum = 0.0, closs = 0.0;
    for (int w = 0; w < W; ++w) {
      const size_t bo = (size_t)a * (T + 1) * W + w, bt = (size_t)a * T * W + w;
      auto V = [&](int t) { return vc[traj_idx[bo + (size_t)t * W]] + (float)traj_time[bo + (size_t)t * W] * 0.001f * vc[D - 1]; };
      float g = 0.0f, vn = V(T);
      for (int t = T - 1; t >= 0; --t) {
        const float v = V(t), nd = traj_done[bt + (size_t)t * W] ? 0.0f : 1.0f;
        const float delta = traj_reward[bt + (size_t)t * W] + (gamma * vn * nd - v);
        g = delta + gamma * lam * nd * g;
        adv[(size_t)w * T + t] = g;
        tgt[(size_t)w * T + t] = g + v;
        vv[(size_t)w * T + t] = v;
        vn = v;
      }
    }
    const double inv = 1.0 / ((double)W * T);
    for (size_t i = 0; i < (size_t)W * T; ++i) asum += adv[i];
    const double mean = asum * inv;
    double var = 0.0;
    for (size_t i = 0; i < (size_t)W * T; ++i) var += (adv[i] - mean) * (adv[i] - mean);
    const float sd = (float)std::sqrt(var * inv) + EPS;
    double aloss = 0.0;
    for (int w = 0; w < W; ++w) {
      const size_t bo = (size_t)a * (T + 1) * W + w, bt = (size_t)a * T * W + w;
      double abar = 0.0, lsum = 0.0, ent = 0.0;
      for (int t = 0; t < T; ++t) abar += ((double)adv[(size_t)w * T + t] - mean) / sd;
      abar /= T;
      for (int t = 0; t < T; ++t) {
        const int idx = traj_idx[bo + (size_t)t * W], tm = traj_time[bo + (size_t)t * W];
        const int act = traj_action[bt + (size_t)t * W];
        const float c = (float)tm * 0.001f;
        // critic
        const float dv = -2.0f * (tgt[(size_t)w * T + t] - vv[(size_t)w * T + t]) * (float)inv;
        closs += (double)(tgt[(size_t)w * T + t] - vv[(size_t)w * T + t]) * (tgt[(size_t)w * T + t] - vv[(size_t)w * T + t]);
        gc[idx] += dv;
        gc[D - 1] += dv * c;
        // actor
        float l[5], p[5], m = -INFINITY, s = 0.0f;
        for (int j = 0; j < 5; ++j) { l[j] = th[(size_t)idx * 5 + j] + c * th[(size_t)(D - 1) * 5 + j]; m = std::max(m, l[j]); }
        for (int j = 0; j < 5; ++j) { p[j] = std::exp(l[j] - m); s += p[j]; }
        float gp[5], dot = 0.0f;
        for (int j = 0; j < 5; ++j) {
          p[j] /= s;
          const float q = p[j] + EPS, lq = std::log(q);
          ent -= (double)q * lq;
          gp[j] = entropy_coeff * (lq + 1.0f) * (float)inv;
        }
        lsum += std::log(p[act] + EPS);
        gp[act] += -(float)abar / (T * (p[act] + EPS)) / W;
        for (int j = 0; j < 5; ++j) dot += gp[j] * p[j];
        for (int j = 0; j < 5; ++j) {
          const float gl = p[j] * (gp[j] - dot);
          ga[(size_t)idx * 5 + j] += gl;
          ga[(size_t)(D - 1) * 5 + j] += gl * c;
        }
      }
      aloss += -(lsum / T) * abar - entropy_coeff * (ent / T);
    }
    if (loss) {
      loss[2 * a] = (float)(aloss / W);
      loss[2 * a + 1] = (float)(closs * inv);
    }
    const int lifetime = levels[(size_t)a * LW + 5];
    if (step[a] + 1 > lifetime) continue;            // discarded update (a2c.py:82-86)
    double na = 0.0, nc = 0.0;
    for (float g : ga) na += (double)g * g;
    for (float g : gc) nc += (double)g * g;
    // optax: where(norm < max_norm, g, g / norm * max_norm)
    const float fa = (float)std::sqrt(na), fc = (float)std::sqrt(nc);
    for (size_t i = 0; i < ga.size(); ++i) th[i] -= actor_lr * (fa < max_norm ? ga[i] : ga[i] / fa * max_norm);
    for (int i = 0; i < D; ++i) vc[i] -= critic_lr * (fc < max_norm ? gc[i] : gc[i] / fc * max_norm);
    step[a] += 1;
  }
  return 0;
}

}  // extern "C"
