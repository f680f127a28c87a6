// GridWorld env step/reset and the fused persistent rollout — HIP for gfx950.
//
// Restates environments/gridworld/gridworld.py:72-211 (step_env/reset_env/
// get_obs), the gymnax 0.0.6 auto-reset wrapper (Environment.step), and
// environments/rollout.py:38-102 (batch_reset / batch_rollout / policy_step)
// with the linear-softmax tabular actor of models/agent.py:7-17.
//
// Mapping: one lane = one env worker.  With W % 64 == 0 every wavefront holds
// the workers of a single agent, so the level record and the actor's
// time-feature row are wave-uniform (readfirstlane -> scalar loads).  The env
// state lives in VGPRs for the whole T-step scan; the trajectory is written
// lane-contiguously ([agent][t][worker]) so every store is coalesced.
#include "common.h"

namespace {

struct EnvState {
  int time, pos, exists, early_term;
  int obj[TOUED_MAX_OBJS];
};

TOUED_DEV int lev_i(const int* lev, int w) { return lev[w]; }
TOUED_DEV float lev_f(const int* lev, int w) { return __int_as_float(lev[w]); }
TOUED_DEV uint32_t wall_word(const int* lev, int w) { return (uint32_t)lev[L_WALLS + w]; }

// The level record held in registers (the tabular rollouts): words [0, L_WALLS + 8) loaded once per lane before
// the step loop, so no step waits on a level load (the step maths reads them under data-dependent branches, where
// the compiler cannot hoist loads).  Every index is a compile-time constant after unrolling except the wall word,
// which is selected from registers.
struct LevR {
  int v[L_WALLS + 8];
};
TOUED_DEV LevR lev_regs(const int* lev) {
  LevR r;
#pragma unroll
  for (int i = 0; i < L_WALLS + 8; ++i) r.v[i] = lev[i];
  return r;
}
TOUED_DEV int lev_i(const LevR& l, int w) { return l.v[w]; }
TOUED_DEV float lev_f(const LevR& l, int w) { return __int_as_float(l.v[w]); }
TOUED_DEV uint32_t wall_word(const LevR& l, int w) {
  // masks, not selects: a select between two array elements is folded into a load from a selected address,
  // which would move the whole record to scratch
  uint32_t x = 0u;
#pragma unroll
  for (int i = 0; i < 8; ++i) x |= (uint32_t)l.v[L_WALLS + i] & (0u - (uint32_t)(w == i));
  return x;
}

template <typename LV>
TOUED_DEV bool wall_at(const LV& lev, int cell) {
  return (wall_word(lev, cell >> 5) >> (cell & 31)) & 1u;
}

// _get_next_pos, gridworld.py:138-146
template <typename LV>
TOUED_DEV int next_pos(const LV& lev, int pos, int action) {
  const int g = lev_i(lev, L_GRID);
  const int top = pos < g, bottom = pos >= g * (g - 1);
  const int left = (pos % g) == 0, right = (pos % g) == g - 1;
  const int step = (action == 0) * (1 - top) * -g + (action == 1) * (1 - bottom) * g +
                   (action == 2) * (1 - left) * -1 + (action == 3) * (1 - right) * 1;
  const int nxt = pos + step;
  return wall_at(lev, nxt) ? pos : nxt;
}

// the same on the level's wall bitmask held in registers (wl = lev[L_WALLS .. +7])
// One actor-table row (5 floats, 20-byte rows: 4-byte aligned) as a 16-byte and a 4-byte buffer load instead of five
// dword gathers: per row one cache-line lookup per instruction instead of five (the candidate-row gathers of the
// rollouts are bound by those lookups: 64 lanes, 64 different rows).  `off` = byte offset of the row in `theta`.
typedef unsigned row_u32x4 __attribute__((ext_vector_type(4)));
TOUED_DEV void load_row5(__amdgpu_buffer_rsrc_t rs, unsigned off, float (&r)[5]) {
  const row_u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0);
  r[0] = __uint_as_float(x.x); r[1] = __uint_as_float(x.y); r[2] = __uint_as_float(x.z); r[3] = __uint_as_float(x.w);
  r[4] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (int)off + 16, 0, 0));
}
TOUED_DEV __amdgpu_buffer_rsrc_t theta_rsrc(const float* theta) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(theta), 0, -1 /* 4 GiB: host-checked */, 0x00020000);
}

TOUED_DEV int next_pos_r(int g, const uint32_t (&wl)[8], int pos, int action) {
  const int top = pos < g, bottom = pos >= g * (g - 1);
  const int left = (pos % g) == 0, right = (pos % g) == g - 1;
  const int step = (action == 0) * (1 - top) * -g + (action == 1) * (1 - bottom) * g +
                   (action == 2) * (1 - left) * -1 + (action == 3) * (1 - right) * 1;
  const int nxt = pos + step;
  const int w = nxt >> 5;
  uint32_t x = 0u;
#pragma unroll
  for (int i = 0; i < 8; ++i) x |= wl[i] & (0u - (uint32_t)(w == i));
  return ((x >> (nxt & 31)) & 1u) ? pos : nxt;
}

// Gumbel top-k choice over the max_grid^2 cells (jax.random.choice replace=False, p given):
// g_c = -gumbel(key)_c - log(p_c), stable ascending argsort, first NMAX indices.
// valid(c) decides p_c = valid/count.  Streaming insertion keeps (value, index) lexicographic order.
template <int NMAX, typename ValidFn>
TOUED_DEV void gumbel_topk(uint2 key, int g2, ValidFn valid, int* out) {
  int cnt = 0;
  for (int c = 0; c < g2; ++c) cnt += valid(c) ? 1 : 0;
  const float pv = __fdiv_rn(1.0f, (float)cnt);
  const float lp_valid = plog(pv);
  float bv[NMAX];
  int bi[NMAX];
#pragma unroll
  for (int j = 0; j < NMAX; ++j) { bv[j] = __builtin_inff(); bi[j] = 0x7fffffff; }
  const float tiny = 1.17549435e-38f;
  for (int c = 0; c < g2; ++c) {
    const float u = uniform_from_bits(random_bits_at(key, (uint32_t)g2, (uint32_t)c), tiny, 1.0f);
    const float gmb = -plog(-plog(u));
    const float g = valid(c) ? __fsub_rn(-gmb, lp_valid) : __builtin_inff();
    // insert (g, c) if it precedes the current last entry
    if (g < bv[NMAX - 1] || (g == bv[NMAX - 1] && c < bi[NMAX - 1])) {
      float cv = g;
      int ci = c;
#pragma unroll
      for (int j = 0; j < NMAX; ++j) {
        const bool before = (cv < bv[j]) || (cv == bv[j] && ci < bi[j]);
        if (before) {
          const float tv = bv[j]; const int ti = bi[j];
          bv[j] = cv; bi[j] = ci; cv = tv; ci = ti;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NMAX; ++j) out[j] = bi[j];
}

// _get_valid_obj_idxs, gridworld.py:149-155, with the isin(idx, bool walls) quirk
struct ValidCells {
  int pos; int g2grid; bool has_false, has_true; int excl[TOUED_MAX_OBJS]; int n_excl;
  TOUED_DEV bool operator()(int c) const {
    bool v = (c != pos) && (c < g2grid);
    v = v && !((c == 0 && has_false) || (c == 1 && has_true));
    for (int i = 0; i < n_excl; ++i) v = v && (c != excl[i]);
    return v;
  }
};

template <typename LV>
TOUED_DEV ValidCells make_valid(const LV& lev, int G2, int pos) {
  ValidCells vc;
  vc.pos = pos;
  const int g = lev_i(lev, L_GRID);
  vc.g2grid = g * g;
  bool any_t = false, any_f = false;
  for (int w = 0; w < 8; ++w) {
    const int lo = w * 32;
    if (lo >= G2) break;
    const int nb = (G2 - lo) < 32 ? (G2 - lo) : 32;
    const uint32_t mask = nb == 32 ? 0xffffffffu : ((1u << nb) - 1u);
    const uint32_t bits = wall_word(lev, w) & mask;
    any_t |= bits != 0u;
    any_f |= bits != mask;
  }
  vc.has_true = any_t; vc.has_false = any_f; vc.n_excl = 0;
  return vc;
}

// reset_env, gridworld.py:157-182
template <int NMAX, bool TAB, typename LV>
TOUED_DEV void reset_env(const EnvSpec& sp, const LV& lev, uint2 key, EnvState& s) {
  const int G2 = sp.max_grid * sp.max_grid;
  s.time = 0;
  s.pos = lev_i(lev, L_START);
  s.early_term = 0;
  const int nobj = lev_i(lev, L_NOBJS);
  s.exists = 0;
#pragma unroll
  for (int i = 0; i < NMAX; ++i) {
    s.obj[i] = lev_i(lev, L_STATIC + i);
    if (i < nobj) s.exists |= 1 << i;
  }
  if (!TAB) {
    if (lev_i(lev, L_RANDRESP)) {
      uint2 obj_key, pos_key;
      split2(key, obj_key, pos_key);
      ValidCells vc = make_valid(lev, G2, s.pos);
      int pick[NMAX];
      gumbel_topk<NMAX>(obj_key, G2, vc, pick);
#pragma unroll
      for (int i = 0; i < NMAX; ++i) s.obj[i] = pick[i];
    }
  }
#pragma unroll
  for (int i = 0; i < NMAX; ++i) s.obj[i] += lev_i(lev, L_OBJ_IDS + i) * G2;
}

// respawn = bernoulli(respawn_key, p_respawn[obj_ids]) over NMAX draws (gridworld.py:99-101) for the objects in
// `miss`; respawn_key = (c2.x, c0.y).  Block b covers draws b and b + nb; only blocks holding a missing object's
// draw are evaluated (the others cannot change the OR into `exists`).
template <int NMAX, typename LV>
TOUED_DEV int respawn_draws(const LV& lev, int miss, uint2 respawn_key) {
  int respawn = 0;
  if (miss == 0) return 0;
  constexpr uint32_t nb = (NMAX + 1) / 2;
#pragma unroll
  for (uint32_t b = 0; b < nb; ++b) {
    const uint32_t hi = b + nb;
    const bool want = ((miss >> b) & 1) || (hi < (uint32_t)NMAX && ((miss >> hi) & 1));
    if (!want) continue;
    const uint2 y = threefry(respawn_key.x, respawn_key.y, b, hi < (uint32_t)NMAX ? hi : 0u);
    const float u0 = bits_to_unit(y.x);
    if (u0 < lev_f(lev, L_PRESP + b)) respawn |= 1 << b;
    if (hi < (uint32_t)NMAX) {
      const float u1 = bits_to_unit(y.y);
      if (u1 < lev_f(lev, L_PRESP + hi)) respawn |= 1 << hi;
    }
  }
  return respawn;
}

// the objects a tabular step_env can respawn: missing ones among the level's n_objs
template <int NMAX, typename LV>
TOUED_DEV int missing_objs(const LV& lev, int exists) {
  const int nobj = lev_i(lev, L_NOBJS);
  const int used = nobj >= 32 ? -1 : ((1 << nobj) - 1);
  return ~exists & used & ((1 << NMAX) - 1);
}

// gymnax Environment.step -> step_env (gridworld.py:72-136) + auto-reset select (RESET = false: the caller
// discards the state after a done, so the reset and its key are skipped).
// PRE: the state-independent blocks d0, d1 (split(key)) and c0 (first block of split(key_s, 3)) come
// precomputed in pre[0..2] (the rollout computes them a step ahead, beside the actor-row gather).
// resp_pre >= 0 (TAB with PRE only): the step's respawn mask, already drawn by the caller (respawn_draws);
// pos_pre >= 0: next_pos(s.pos, action), already computed by the caller.
template <int NMAX, bool TAB, bool RESET = true, bool PRE = false, typename LV>
TOUED_DEV void env_step(const EnvSpec& sp, const LV& lev, uint2 key, EnvState& s, int action,
                        float& reward, bool& done, const uint2* pre = nullptr, int resp_pre = -1,
                        int pos_pre = -1) {
  const int G2 = sp.max_grid * sp.max_grid;
  const int pos = pos_pre >= 0 ? pos_pre : next_pos(lev, s.pos, action);
  int old[NMAX];
  int collected = 0;
#pragma unroll
  for (int i = 0; i < NMAX; ++i) {
    old[i] = s.obj[i] - lev_i(lev, L_OBJ_IDS + i) * G2;
    if (((s.exists >> i) & 1) && old[i] == pos) collected |= 1 << i;
  }
  const int nobj = lev_i(lev, L_NOBJS);
  const int used = nobj >= 32 ? -1 : ((1 << nobj) - 1);
  // The step's keys: (key_s, key_r) = split(key); (term, respawn, obj) = split(key_s, 3).  Only the
  // threefry blocks whose outcome can change the result are evaluated (identical results, fewer calls):
  //  * respawn draw i matters only while object i is missing (it is OR-ed into `exists`; with random
  //    respawn it also picks the missing object's cell);
  //  * the termination draw matters only when something was collected (p_t = 0 otherwise);
  //  * key_r only on done.
  // split(key): blocks d0 = (0,2), d1 = (1,3): key_s = (d0.x, d1.x), key_r = (d0.y, d1.y).
  // split(key_s, 3): blocks c0 = (0,3), c1 = (1,4), c2 = (2,5): term = (c0.x, c1.x), respawn = (c2.x, c0.y),
  // obj = (c1.y, c2.y).
  const int miss = ~s.exists & (TAB ? used : -1) & ((1 << NMAX) - 1);
  const bool need_term = collected != 0;
  const bool have_resp = TAB && PRE && resp_pre >= 0;
  bool have_d = false, have_c1 = false;
  uint2 d0 = make_uint2(0u, 0u), d1 = d0, c0 = d0, c1 = d0, c2 = d0;
  if (PRE) {
    d0 = pre[0];
    d1 = pre[1];
    c0 = pre[2];
    have_d = true;
    if (miss != 0 && !have_resp) c2 = threefry(d0.x, d1.x, 2u, 5u);
    if (need_term) { c1 = threefry(d0.x, d1.x, 1u, 4u); have_c1 = true; }
  } else if (need_term || miss != 0) {
    d0 = threefry(key.x, key.y, 0u, 2u);
    d1 = threefry(key.x, key.y, 1u, 3u);
    have_d = true;
    c0 = threefry(d0.x, d1.x, 0u, 3u);
    if (miss != 0) c2 = threefry(d0.x, d1.x, 2u, 5u);
    if (need_term) { c1 = threefry(d0.x, d1.x, 1u, 4u); have_c1 = true; }
  }
  const int respawn = have_resp ? resp_pre : respawn_draws<NMAX>(lev, miss, make_uint2(c2.x, c0.y));
  int exists = s.exists | respawn;
  int newpos[NMAX];
#pragma unroll
  for (int i = 0; i < NMAX; ++i) newpos[i] = old[i];
  if (!TAB) {
    const int use_new = (~s.exists) & respawn & ((1 << NMAX) - 1);
    if (lev_i(lev, L_RANDRESP) && use_new) {
      if (!have_c1) c1 = threefry(d0.x, d1.x, 1u, 4u);
      const uint2 obj_key = make_uint2(c1.y, c2.y);
      ValidCells vc = make_valid(lev, G2, pos);
#pragma unroll
      for (int i = 0; i < NMAX; ++i) vc.excl[i] = old[i];
      vc.n_excl = NMAX;
      int pick[NMAX];
      gumbel_topk<NMAX>(obj_key, G2, vc, pick);
#pragma unroll
      for (int i = 0; i < NMAX; ++i) if ((use_new >> i) & 1) newpos[i] = pick[i];
    }
  }
  exists = exists & ~collected & used;

  float p_t = 0.0f, rew = 0.0f;
#pragma unroll
  for (int i = 0; i < NMAX; ++i) {
    const float ci = ((collected >> i) & 1) ? 1.0f : 0.0f;
    p_t = __fadd_rn(p_t, __fmul_rn(lev_f(lev, L_PTERM + i), ci));
    if ((collected >> i) & 1) rew = __fadd_rn(rew, lev_f(lev, L_REW + i));
  }
  bool hit = false;
  if (need_term) hit = bits_to_unit(threefry(c0.x, c1.x, 0u, 0u).x) < p_t;   // bits1(term_key)
  const int term = hit || s.early_term;
  const int time = s.time + 1;
  done = (time >= lev_i(lev, L_MAX_STEPS)) || term;
  reward = rew;
  if (done) {
    if (!RESET) return;
    if (!have_d) {
      d0 = threefry(key.x, key.y, 0u, 2u);
      d1 = threefry(key.x, key.y, 1u, 3u);
    }
    reset_env<NMAX, TAB>(sp, lev, make_uint2(d0.y, d1.y), s);
  } else {
    s.time = time;
    s.pos = pos;
    s.exists = exists;
    s.early_term = term;
#pragma unroll
    for (int i = 0; i < NMAX; ++i) s.obj[i] = newpos[i] + lev_i(lev, L_OBJ_IDS + i) * G2;
  }
}

template <int NMAX>
TOUED_DEV void load_state(const int* st, int n, int i, EnvState& s) {
  s.time = st[S_TIME * n + i];
  s.pos = st[S_POS * n + i];
  s.exists = st[S_EXISTS * n + i];
  s.early_term = st[S_TERM * n + i];
#pragma unroll
  for (int k = 0; k < NMAX; ++k) s.obj[k] = st[(S_OBJ + k) * n + i];
}

template <int NMAX>
TOUED_DEV void store_state(int* st, int n, int i, const EnvState& s) {
  st[S_TIME * n + i] = s.time;
  st[S_POS * n + i] = s.pos;
  st[S_EXISTS * n + i] = s.exists;
  st[S_TERM * n + i] = s.early_term;
#pragma unroll
  for (int k = 0; k < NMAX; ++k) st[(S_OBJ + k) * n + i] = s.obj[k];
}

TOUED_DEV int tab_index(const EnvSpec& sp, const EnvState& s) {
  return s.pos + sp.max_grid * sp.max_grid * s.exists;
}

// ---------------------------------------------------------------- kernels
// gymnax reset for n independent (key, level) pairs; worker i uses level i / W.
template <int NMAX, bool TAB>
__global__ void __launch_bounds__(256) k_gw_reset(EnvSpec sp, const int* __restrict__ levels, int W,
                                                  const uint32_t* __restrict__ keys, int* __restrict__ state,
                                                  int* __restrict__ obs_idx, int* __restrict__ obs_time, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int* lev = levels + (size_t)(i / W) * LEVEL_WORDS;
  EnvState s;
  reset_env<NMAX, TAB>(sp, lev, make_uint2(keys[2 * i], keys[2 * i + 1]), s);
  store_state<NMAX>(state, n, i, s);
  obs_idx[i] = tab_index(sp, s);
  obs_time[i] = s.time;
}

template <int NMAX, bool TAB>
__global__ void __launch_bounds__(256) k_gw_step(EnvSpec sp, const int* __restrict__ levels, int W,
                                                 const uint32_t* __restrict__ keys, int* __restrict__ state,
                                                 const int* __restrict__ actions, int* __restrict__ obs_idx,
                                                 int* __restrict__ obs_time, float* __restrict__ reward,
                                                 uint8_t* __restrict__ done, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int* lev = levels + (size_t)(i / W) * LEVEL_WORDS;
  EnvState s;
  load_state<NMAX>(state, n, i, s);
  float r; bool d;
  env_step<NMAX, TAB>(sp, lev, make_uint2(keys[2 * i], keys[2 * i + 1]), s, actions[i], r, d);
  store_state<NMAX>(state, n, i, s);
  obs_idx[i] = tab_index(sp, s);
  obs_time[i] = s.time;
  reward[i] = r;
  done[i] = d ? 1 : 0;
}

// RolloutWrapper.batch_reset: worker keys = split(agent_key, W)[w].
template <int NMAX, bool TAB>
__global__ void __launch_bounds__(256) k_batch_reset(EnvSpec sp, const int* __restrict__ levels,
                                                     const uint32_t* __restrict__ agent_keys, int W,
                                                     int* __restrict__ state, int* __restrict__ obs_idx,
                                                     int* __restrict__ obs_time, int n,
                                                     const uint8_t* __restrict__ mask) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int a = i / W, w = i - a * W;
  if (mask && !mask[a]) return;
  const int* lev = levels + (size_t)a * LEVEL_WORDS;
  const uint2 key = split_at(make_uint2(agent_keys[2 * a], agent_keys[2 * a + 1]), (uint32_t)W, (uint32_t)w);
  EnvState s;
  reset_env<NMAX, TAB>(sp, lev, key, s);
  store_state<NMAX>(state, n, i, s);
  obs_idx[i] = tab_index(sp, s);
  obs_time[i] = s.time;
}

// Linear softmax actor on a compact tabular obs: logits = W[idx] + (f32(t)*0.001)*W[D-1].
TOUED_DEV void actor_probs5(const float* __restrict__ tab, const float* last, int idx, int t, float* p) {
  const float c = __fmul_rn((float)t, 0.001f);
  float l[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) l[j] = __fadd_rn(tab[(size_t)idx * 5 + j], __fmul_rn(c, last[j]));
  float m = l[0];
#pragma unroll
  for (int j = 1; j < 5; ++j) m = fmaxf(m, l[j]);
  float e[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) e[j] = pexp(__fsub_rn(l[j], m));
  float s = e[0];
#pragma unroll
  for (int j = 1; j < 5; ++j) s = __fadd_rn(s, e[j]);
#pragma unroll
  for (int j = 0; j < 5; ++j) p[j] = __fdiv_rn(e[j], s);
}

// actor_probs5 on an already gathered table row
TOUED_DEV void actor_probs5_row(const float* row, const float* last, int t, float* p) {
  const float c = __fmul_rn((float)t, 0.001f);
  float l[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) l[j] = __fadd_rn(row[j], __fmul_rn(c, last[j]));
  float m = l[0];
#pragma unroll
  for (int j = 1; j < 5; ++j) m = fmaxf(m, l[j]);
  float e[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) e[j] = pexp(__fsub_rn(l[j], m));
  float s = e[0];
#pragma unroll
  for (int j = 1; j < 5; ++j) s = __fadd_rn(s, e[j]);
#pragma unroll
  for (int j = 0; j < 5; ++j) p[j] = __fdiv_rn(e[j], s);
}

// choice5 with the key's bits1 already drawn
TOUED_DEV int choice5_bits(uint32_t bits, const float* p) {
  const float c0 = p[0];
  const float c1 = __fadd_rn(p[0], p[1]);
  const float c2 = __fadd_rn(c1, p[2]);
  const float c3 = __fadd_rn(c1, __fadd_rn(p[2], p[3]));
  const float c4 = __fadd_rn(c3, p[4]);
  const float u = bits_to_unit(bits);
  const float r = __fmul_rn(c4, __fsub_rn(1.0f, u));
  return (c0 < r) + (c1 < r) + (c2 < r) + (c3 < r) + (c4 < r);
}

// jax.random.choice(key, 5, p=p): searchsorted(cumsum_assoc(p), c4*(1-u), 'left')
TOUED_DEV int choice5(uint2 key, const float* p) {
  const float c0 = p[0];
  const float c1 = __fadd_rn(p[0], p[1]);
  const float c2 = __fadd_rn(c1, p[2]);
  const float c3 = __fadd_rn(c1, __fadd_rn(p[2], p[3]));
  const float c4 = __fadd_rn(c3, p[4]);
  const float u = bits_to_unit(bits1(key));
  const float r = __fmul_rn(c4, __fsub_rn(1.0f, u));
  return (c0 < r) + (c1 < r) + (c2 < r) + (c3 < r) + (c4 < r);
}

// Fused rollout: T policy steps per worker, state in registers.
// traj_idx/time: [N][T+1][W]; action/done u8 [N][T][W]; reward f32 [N][T][W].
template <int NMAX, bool TAB, bool UNIFORM>
__global__ void __launch_bounds__(256) k_rollout(EnvSpec sp, const int* __restrict__ levels,
                                                 const float* __restrict__ theta, int D,
                                                 const uint32_t* __restrict__ agent_keys, int* __restrict__ state,
                                                 int T, int W, int n, int* __restrict__ traj_idx,
                                                 int* __restrict__ traj_time, uint8_t* __restrict__ traj_action,
                                                 float* __restrict__ traj_reward, uint8_t* __restrict__ traj_done,
                                                 float* __restrict__ cum_return) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int a = i / W;
  if (UNIFORM) a = __builtin_amdgcn_readfirstlane(a);
  const int w = i - a * W;
  const LevR lev = lev_regs(levels + (size_t)a * LEVEL_WORDS);
  const float* tab = theta + (size_t)a * D * 5;
  const __amdgpu_buffer_rsrc_t rs_t = theta_rsrc(theta);
  const unsigned tab_off = (unsigned)((size_t)a * D * 20);
  float last[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) last[j] = tab[(size_t)(D - 1) * 5 + j];
  uint2 rng = split_at(make_uint2(agent_keys[2 * a], agent_keys[2 * a + 1]), (uint32_t)W, (uint32_t)w);
  EnvState s;
  load_state<NMAX>(state, n, i, s);
  float cum = 0.0f, valid = 1.0f;
  const size_t base_o = (size_t)a * (T + 1) * W + w;
  const size_t base_t = (size_t)a * T * W + w;
  // Every threefry block that does not depend on the env state is computed one step ahead, between the issue of
  // the step's actor-row gather and its use: (rng, sub) = split(rng) [action key], the choice bits,
  // (rng, sub) = split(rng) [env key], and the env key's d0, d1, c0 (env_step<.., PRE>).  The rollout is a
  // chain of dependent steps per wave, so this independent work fills the gather's latency.
  struct StepKeys { uint2 rng, sub_env; uint32_t cbits; uint2 pre[3]; };
  auto keys_of = [&](uint2 r) {
    StepKeys k;
    uint2 sub;
    split2(r, r, sub);
    k.cbits = bits1(sub);
    split2(r, r, k.sub_env);
    k.rng = r;
    k.pre[0] = threefry(k.sub_env.x, k.sub_env.y, 0u, 2u);
    k.pre[1] = threefry(k.sub_env.x, k.sub_env.y, 1u, 3u);
    k.pre[2] = threefry(k.pre[0].x, k.pre[1].x, 0u, 3u);
    return k;
  };
  StepKeys kc = keys_of(rng);
  // Candidate-row prefetch (tabular): given the state and the step's keys, the next observation of a step that
  // does not end the episode is a function of the action alone -- position next_pos(pos, a), objects
  // (exists | respawn) & ~collected(a) & used, with the respawn draws state-independent blocks -- so the five
  // possible next actor rows are gathered at the start of the step and the taken one is selected afterwards.
  // The gather then overlaps the whole step instead of sitting on the chain.  A miss (the episode ended and the
  // auto-reset moved the agent) re-gathers; the selection never changes a value.
  int idx = tab_index(sp, s);
  float row[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) row[j] = tab[(size_t)idx * 5 + j];
  const int G2 = sp.max_grid * sp.max_grid;
  const int nobj = lev_i(lev, L_NOBJS);
  const int used = nobj >= 32 ? -1 : ((1 << nobj) - 1);
  int objpos[NMAX];
#pragma unroll
  for (int o = 0; o < NMAX; ++o) objpos[o] = s.obj[o] - lev_i(lev, L_OBJ_IDS + o) * G2;   // static in TAB
  const int grid = lev_i(lev, L_GRID);
  uint32_t wl[8];   // the wall bitmask in registers: no dependent level load on the step chain
#pragma unroll
  for (int i = 0; i < 8; ++i) wl[i] = (uint32_t)lev_i(lev, L_WALLS + i);
  for (int t = 0; t < T; ++t) {
    const int tm = s.time;
    int cidx[5], cpos[5];
    float crow[5][5];
    int resp = -1;
    if (TAB) {
      const int miss = missing_objs<NMAX>(lev, s.exists);
      resp = miss ? respawn_draws<NMAX>(lev, miss, make_uint2(threefry(kc.pre[0].x, kc.pre[1].x, 2u, 5u).x,
                                                               kc.pre[2].y))
                  : 0;
#pragma unroll
      for (int a = 0; a < 5; ++a) {
        const int p = next_pos_r(grid, wl, s.pos, a);
        cpos[a] = p;
        int col = 0;
#pragma unroll
        for (int o = 0; o < NMAX; ++o)
          if (((s.exists >> o) & 1) && objpos[o] == p) col |= 1 << o;
        cidx[a] = p + G2 * ((s.exists | resp) & ~col & used);
        load_row5(rs_t, tab_off + (unsigned)cidx[a] * 20u, crow[a]);
      }
    }
    const StepKeys kn = keys_of(kc.rng);      // next step's keys while the gathers are in flight
    float p[5];
    actor_probs5_row(row, last, tm, p);
    const int action = choice5_bits(kc.cbits, p);
    float r; bool d;
    int npos = -1;
    if (TAB) {
#pragma unroll
      for (int a = 0; a < 5; ++a) npos = a == action ? cpos[a] : npos;
    }
    if (traj_idx)
      env_step<NMAX, TAB, true, true>(sp, lev, kc.sub_env, s, action, r, d, kc.pre, resp, npos);
    else
      env_step<NMAX, TAB, false, true>(sp, lev, kc.sub_env, s, action, r, d, kc.pre, resp, npos);   // returns-only
    cum = __fadd_rn(cum, __fmul_rn(r, valid));
    valid = __fmul_rn(valid, d ? 0.0f : 1.0f);
    // returns-only mode (eval_agent): nothing after the first episode can change cum_return
    if (!traj_idx && valid == 0.0f) break;
    if (traj_idx) {   // eval_agent only needs the return (agents/agents.py:98-106)
      traj_idx[base_o + (size_t)t * W] = idx;
      traj_time[base_o + (size_t)t * W] = tm;
      traj_action[base_t + (size_t)t * W] = (uint8_t)action;
      traj_reward[base_t + (size_t)t * W] = r;
      traj_done[base_t + (size_t)t * W] = d ? 1 : 0;
    }
    const int nidx = tab_index(sp, s);
    bool hit = false;
    if (TAB) {
#pragma unroll
      for (int a = 0; a < 5; ++a)
        if (a == action) {
          hit = cidx[a] == nidx;
#pragma unroll
          for (int j = 0; j < 5; ++j) row[j] = crow[a][j];
        }
    }
    if (!hit) {
#pragma unroll
      for (int j = 0; j < 5; ++j) row[j] = tab[(size_t)nidx * 5 + j];
    }
    idx = nidx;
    kc = kn;
  }
  if (traj_idx) {
    traj_idx[base_o + (size_t)T * W] = tab_index(sp, s);
    traj_time[base_o + (size_t)T * W] = s.time;
  }
  if (traj_idx) store_state<NMAX>(state, n, i, s);   // returns-only mode leaves the state untouched
  if (cum_return) cum_return[i] = cum;
}

// ---------------------------------------------------------------- eval_agent returns in three launches
// eval_agent (agents/agents.py:98-106) rolls every agent's 4 workers for the eval length (2000 steps on the tabular
// levels) and keeps only the return.  Per step a worker spends ~10 threefry blocks on draws that do not depend on the
// env state, and that chain, not the env, set the single-kernel rollout's step time.  Split by dependence:
//   k_eval_keys    the per-worker key chain ((rng, sub) = split(rng), (rng, sub_env) = split(rng) per step:
//                  two dependent splits) -> chain[t][i] = (sub, sub_env);
//   k_eval_draws   one thread per (step, worker): the choice bits bits1(sub), the termination uniform's bits
//                  bits1(term_key) and the respawn bernoullis of ALL objects -> draws[t][i] (state-independent: the
//                  step uses resp & missing, and the termination draw only when something was collected);
//   k_eval_returns the env chain on those draws (the tabular step_env algebra, returns-only: no auto-reset),
//                  the draws loaded two steps ahead and the next actor row by candidate prefetch.
// Bit-identical to k_rollout's returns-only mode (tests/test_gpu_env.py::test_eval_returns_three_launches).
__global__ void __launch_bounds__(256) k_eval_keys(const uint32_t* __restrict__ agent_keys, int W, int T, int n,
                                                   uint4* __restrict__ chain) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int a = i / W, w = i - a * W;
  uint2 r = split_at(make_uint2(agent_keys[2 * a], agent_keys[2 * a + 1]), (uint32_t)W, (uint32_t)w);
  for (int t = 0; t < T; ++t) {
    uint2 sub, sub_env;
    split2(r, r, sub);
    split2(r, r, sub_env);
    chain[(size_t)t * n + i] = make_uint4(sub.x, sub.y, sub_env.x, sub_env.y);
  }
}

template <int NMAX>
__global__ void __launch_bounds__(256) k_eval_draws(const int* __restrict__ levels, int W, int n, long total,
                                                    const uint4* __restrict__ chain, uint4* __restrict__ draws) {
  const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= total) return;
  const int i = (int)(j % n);
  const int* lev = levels + (size_t)(i / W) * LEVEL_WORDS;
  const uint4 c = chain[j];
  const uint32_t cbits = bits1(make_uint2(c.x, c.y));
  // split(sub_env) blocks d0, d1; split(key_s, 3) blocks c0, c1, c2 (env_step's naming)
  const uint2 d0 = threefry(c.z, c.w, 0u, 2u), d1 = threefry(c.z, c.w, 1u, 3u);
  const uint2 c0 = threefry(d0.x, d1.x, 0u, 3u), c1 = threefry(d0.x, d1.x, 1u, 4u), c2 = threefry(d0.x, d1.x, 2u, 5u);
  const int resp = respawn_draws<NMAX>(lev, (1 << NMAX) - 1, make_uint2(c2.x, c0.y));
  const uint32_t tbits = threefry(c0.x, c1.x, 0u, 0u).x;
  draws[j] = make_uint4(cbits, tbits, (uint32_t)resp, 0u);
}

template <int NMAX>
__global__ void __launch_bounds__(256) k_eval_returns(EnvSpec sp, const int* __restrict__ levels,
                                                      const float* __restrict__ theta, int D,
                                                      const int* __restrict__ state, int T, int W, int n,
                                                      const uint4* __restrict__ draws, float* __restrict__ cum_return) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int a = i / W;
  const LevR lev = lev_regs(levels + (size_t)a * LEVEL_WORDS);
  const float* tab = theta + (size_t)a * D * 5;
  const __amdgpu_buffer_rsrc_t rs_t = theta_rsrc(theta);
  const unsigned tab_off = (unsigned)((size_t)a * D * 20);
  float last[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) last[j] = tab[(size_t)(D - 1) * 5 + j];
  EnvState s;
  load_state<NMAX>(state, n, i, s);
  const int G2 = sp.max_grid * sp.max_grid;
  const int nobj = lev_i(lev, L_NOBJS);
  const int used = nobj >= 32 ? -1 : ((1 << nobj) - 1);
  const int max_steps = lev_i(lev, L_MAX_STEPS);
  const int grid = lev_i(lev, L_GRID);
  uint32_t wl[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) wl[k] = wall_word(lev, k);
  int objpos[NMAX];
#pragma unroll
  for (int o = 0; o < NMAX; ++o) objpos[o] = s.obj[o] - lev_i(lev, L_OBJ_IDS + o) * G2;   // static in TAB
  float row[5];
  {
    const int idx = tab_index(sp, s);
#pragma unroll
    for (int j = 0; j < 5; ++j) row[j] = tab[(size_t)idx * 5 + j];
  }
  float cum = 0.0f;
  uint4 dr0 = T > 0 ? draws[i] : make_uint4(0u, 0u, 0u, 0u);
  uint4 dr1 = T > 1 ? draws[(size_t)n + i] : dr0;
  for (int t = 0; t < T; ++t) {
    const uint4 dr = dr0;
    dr0 = dr1;
    if (t + 2 < T) dr1 = draws[(size_t)(t + 2) * n + i];
    // next state of each action while the episode goes on: position, objects left
    int cpos[5], cex[5];
    float crow[5][5];
#pragma unroll
    for (int act = 0; act < 5; ++act) {
      const int p = next_pos_r(grid, wl, s.pos, act);
      int col = 0;
#pragma unroll
      for (int o = 0; o < NMAX; ++o)
        if (((s.exists >> o) & 1) && objpos[o] == p) col |= 1 << o;
      cpos[act] = p;
      cex[act] = col;
      const int ci = p + G2 * ((s.exists | (int)dr.z) & ~col & used);
      load_row5(rs_t, tab_off + (unsigned)ci * 20u, crow[act]);
    }
    float p[5];
    actor_probs5_row(row, last, s.time, p);
    const int action = choice5_bits(dr.x, p);
    int pos = 0, collected = 0;
#pragma unroll
    for (int act = 0; act < 5; ++act)
      if (act == action) {
        pos = cpos[act];
        collected = cex[act];
#pragma unroll
        for (int j = 0; j < 5; ++j) row[j] = crow[act][j];
      }
    // step_env (gridworld.py:72-136), tabular: the same operation order as env_step
    float p_t = 0.0f, rew = 0.0f;
#pragma unroll
    for (int o = 0; o < NMAX; ++o) {
      const float co = ((collected >> o) & 1) ? 1.0f : 0.0f;
      p_t = __fadd_rn(p_t, __fmul_rn(lev_f(lev, L_PTERM + o), co));
      if ((collected >> o) & 1) rew = __fadd_rn(rew, lev_f(lev, L_REW + o));
    }
    const bool hit = collected != 0 && bits_to_unit(dr.y) < p_t;
    const int term = hit || s.early_term;
    const int time = s.time + 1;
    cum = __fadd_rn(cum, rew);   // valid = 1 until the first done, after which the worker stops
    if ((time >= max_steps) || term) break;
    s.time = time;
    s.pos = pos;
    s.exists = (s.exists | (int)dr.z) & ~collected & used;
    s.early_term = term;
  }
  cum_return[i] = cum;
}

}  // namespace

// ---------------------------------------------------------------- dispatch
#define TOUED_DISPATCH_NMAX(NM, TAB, ...)                    \
  switch (NM) {                                              \
    case 1: { constexpr int NMAX = 1; __VA_ARGS__; } break;  \
    case 2: { constexpr int NMAX = 2; __VA_ARGS__; } break;  \
    case 3: { constexpr int NMAX = 3; __VA_ARGS__; } break;  \
    case 4: { constexpr int NMAX = 4; __VA_ARGS__; } break;  \
    case 5: { constexpr int NMAX = 5; __VA_ARGS__; } break;  \
    default: break;                                          \
  }

#define TOUED_DISPATCH(sp, ...)                                                  \
  if ((sp).tabular) {                                                            \
    constexpr bool TAB = true;                                                   \
    TOUED_DISPATCH_NMAX((sp).n_max, TAB, __VA_ARGS__)                            \
  } else {                                                                       \
    constexpr bool TAB = false;                                                  \
    TOUED_DISPATCH_NMAX((sp).n_max, TAB, __VA_ARGS__)                            \
  }

static int check_spec(const EnvSpec& sp) {
  TOUED_REQUIRE(sp.n_max >= 1 && sp.n_max <= 5, "env spec: max_n_objs=%d unsupported (1..5)", sp.n_max);
  TOUED_REQUIRE(sp.max_grid >= 1 && sp.max_grid * sp.max_grid <= 256, "env spec: max_grid_size=%d unsupported",
                sp.max_grid);
  TOUED_REQUIRE(sp.n_types >= 1 && sp.n_types <= 8, "env spec: max_n_obj_types=%d unsupported", sp.n_types);
  return 0;
}

static inline int nblk(long n) { return (int)((n + 255) / 256); }

extern "C" {

int toued_gw_reset(EnvSpec sp, const int* levels, int W, const uint32_t* keys, int* state, int* obs_idx,
                   int* obs_time, int n, hipStream_t stream) {
  if (int e = check_spec(sp)) return e;
  TOUED_REQUIRE(n >= 0 && W >= 1, "toued_gw_reset: bad sizes n=%d W=%d", n, W);
  if (n == 0) return 0;
  TOUED_DISPATCH(sp, hipLaunchKernelGGL((k_gw_reset<NMAX, TAB>), dim3(nblk(n)), dim3(256), 0, stream, sp, levels,
                                        W, keys, state, obs_idx, obs_time, n));
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_gw_step(EnvSpec sp, const int* levels, int W, const uint32_t* keys, int* state, const int* actions,
                  int* obs_idx, int* obs_time, float* reward, uint8_t* done, int n, hipStream_t stream) {
  if (int e = check_spec(sp)) return e;
  TOUED_REQUIRE(n >= 0 && W >= 1, "toued_gw_step: bad sizes n=%d W=%d", n, W);
  if (n == 0) return 0;
  TOUED_DISPATCH(sp, hipLaunchKernelGGL((k_gw_step<NMAX, TAB>), dim3(nblk(n)), dim3(256), 0, stream, sp, levels, W,
                                        keys, state, actions, obs_idx, obs_time, reward, done, n));
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_batch_reset(EnvSpec sp, const int* levels, const uint32_t* agent_keys, int n_agents, int W, int* state,
                      int* obs_idx, int* obs_time, hipStream_t stream) {
  if (int e = check_spec(sp)) return e;
  TOUED_REQUIRE(n_agents >= 0 && W >= 1, "toued_batch_reset: bad sizes N=%d W=%d", n_agents, W);
  const int n = n_agents * W;
  if (n == 0) return 0;
  TOUED_DISPATCH(sp, hipLaunchKernelGGL((k_batch_reset<NMAX, TAB>), dim3(nblk(n)), dim3(256), 0, stream, sp, levels,
                                        agent_keys, W, state, obs_idx, obs_time, n, nullptr));
  TOUED_CHECK_LAUNCH();
  return 0;
}

// the same for the workers of the agents a with mask[a] != 0 only (in place into state / obs_idx / obs_time)
int toued_batch_reset_masked(EnvSpec sp, const int* levels, const uint32_t* agent_keys, int n_agents, int W, int* state,
                             int* obs_idx, int* obs_time, const uint8_t* mask, hipStream_t stream) {
  if (int e = check_spec(sp)) return e;
  TOUED_REQUIRE(n_agents >= 0 && W >= 1 && mask, "toued_batch_reset_masked: bad sizes N=%d W=%d", n_agents, W);
  const int n = n_agents * W;
  if (n == 0) return 0;
  TOUED_DISPATCH(sp, hipLaunchKernelGGL((k_batch_reset<NMAX, TAB>), dim3(nblk(n)), dim3(256), 0, stream, sp, levels,
                                        agent_keys, W, state, obs_idx, obs_time, n, mask));
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_eval_keys(const uint32_t* agent_keys, int n_agents, int W, int T, uint32_t* chain, hipStream_t stream) {
  TOUED_REQUIRE(n_agents >= 0 && W >= 1 && T >= 0, "toued_eval_keys: bad sizes N=%d W=%d T=%d", n_agents, W, T);
  const int n = n_agents * W;
  if (n == 0 || T == 0) return 0;
  hipLaunchKernelGGL(k_eval_keys, dim3(nblk(n)), dim3(256), 0, stream, agent_keys, W, T, n,
                     reinterpret_cast<uint4*>(chain));
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_eval_draws(EnvSpec sp, const int* levels, int n_agents, int W, int T, const uint32_t* chain, uint32_t* draws,
                     hipStream_t stream) {
  if (int e = check_spec(sp)) return e;
  TOUED_REQUIRE(sp.tabular, "toued_eval_draws: tabular envs only");
  TOUED_REQUIRE(n_agents >= 0 && W >= 1 && T >= 0, "toued_eval_draws: bad sizes N=%d W=%d T=%d", n_agents, W, T);
  const int n = n_agents * W;
  const long total = (long)n * T;
  if (total == 0) return 0;
  const unsigned g = (unsigned)((total + 255) / 256);
  TOUED_DISPATCH_NMAX(sp.n_max, true, hipLaunchKernelGGL(k_eval_draws<NMAX>, dim3(g), dim3(256), 0, stream, levels,
                                                        W, n, total, reinterpret_cast<const uint4*>(chain),
                                                        reinterpret_cast<uint4*>(draws)));
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_eval_returns(EnvSpec sp, const int* levels, const float* theta, int D, const int* state, int n_agents, int W,
                       int T, const uint32_t* draws, float* cum_return, hipStream_t stream) {
  if (int e = check_spec(sp)) return e;
  TOUED_REQUIRE(sp.tabular, "toued_eval_returns: the linear tabular actor needs a tabular env");
  TOUED_REQUIRE(n_agents >= 0 && W >= 1 && T >= 0, "toued_eval_returns: bad sizes N=%d W=%d T=%d", n_agents, W, T);
  TOUED_REQUIRE(D == sp.max_grid * sp.max_grid * (1 << sp.n_max) + 1, "toued_eval_returns: D=%d != obs_dim", D);
  TOUED_REQUIRE((double)n_agents * D * 20.0 < 4294967295.0, "toued_eval_returns: actor tables (%d x %d rows) exceed 4 GiB",
                n_agents, D);
  const int n = n_agents * W;
  if (n == 0) return 0;
  TOUED_DISPATCH_NMAX(sp.n_max, true, hipLaunchKernelGGL(k_eval_returns<NMAX>, dim3(nblk(n)), dim3(256), 0, stream, sp,
                                                        levels, theta, D, state, T, W, n,
                                                        reinterpret_cast<const uint4*>(draws), cum_return));
  TOUED_CHECK_LAUNCH();
  return 0;
}

int toued_rollout(EnvSpec sp, const int* levels, const float* theta, int D, const uint32_t* agent_keys, int* state,
                  int n_agents, int W, int T, int* traj_idx, int* traj_time, uint8_t* traj_action,
                  float* traj_reward, uint8_t* traj_done, float* cum_return, hipStream_t stream) {
  if (int e = check_spec(sp)) return e;
  TOUED_REQUIRE(n_agents >= 0 && W >= 1 && T >= 0, "toued_rollout: bad sizes N=%d W=%d T=%d", n_agents, W, T);
  TOUED_REQUIRE(sp.tabular, "toued_rollout: the linear tabular actor needs a tabular env");
  TOUED_REQUIRE(D == sp.max_grid * sp.max_grid * (1 << sp.n_max) + 1, "toued_rollout: D=%d != obs_dim", D);
  TOUED_REQUIRE((double)n_agents * D * 20.0 < 4294967295.0, "toued_rollout: actor tables (%d x %d rows) exceed 4 GiB",
                n_agents, D);
  TOUED_REQUIRE(traj_idx || cum_return, "toued_rollout: returns-only mode needs cum_return");
  const int n = n_agents * W;
  if (n == 0) return 0;
  if (W % 64 == 0) {
    TOUED_DISPATCH(sp, hipLaunchKernelGGL((k_rollout<NMAX, TAB, true>), dim3(nblk(n)), dim3(256), 0, stream, sp,
                                          levels, theta, D, agent_keys, state, T, W, n, traj_idx, traj_time,
                                          traj_action, traj_reward, traj_done, cum_return));
  } else {
    TOUED_DISPATCH(sp, hipLaunchKernelGGL((k_rollout<NMAX, TAB, false>), dim3(nblk(n)), dim3(256), 0, stream, sp,
                                          levels, theta, D, agent_keys, state, T, W, n, traj_idx, traj_time,
                                          traj_action, traj_reward, traj_done, cum_return));
  }
  TOUED_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
