// Tabular GridWorld device code shared by the rollout kernels (env.hip) and the A2C chain (a2c.hip):
// environments/gridworld/gridworld.py:72-211 (step_env / reset_env / get_obs), the gymnax 0.0.6 auto-reset and
// the linear-softmax tabular actor of models/agent.py:7-17.  Internal linkage: every including unit gets its own
// copy (device code only).
#pragma once
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
  for (int j = 0; j < 5; ++j) e[j] = pexp_le0(__fsub_rn(l[j], m));
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
  for (int j = 0; j < 5; ++j) e[j] = pexp_le0(__fsub_rn(l[j], m));
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

// a step's four draw words (choice bits, termination bits, respawn mask, 0) as a native vector: HIP's uint4 struct
// copies in the two-ahead prefetch rotation went through scratch
typedef unsigned draw4 __attribute__((ext_vector_type(4)));

// One env step's four draw words from its two keys (sub: the action choice, sub_env: step_env's key), as
// step_env would draw them (gridworld.py:72-136 over env_step's key splits): the choice bits, the termination
// uniform's bits and the respawn bernoullis of every object, 0.  The state-independent half of a tabular step
// (k_eval_draws and the A2C chain's own draws call this one function, so their draws are the same bits).
template <int NMAX, typename LV>
TOUED_DEV draw4 step_draws(const LV& lev, uint2 sub, uint2 sub_env) {
  const uint32_t cbits = bits1(sub);
  // split(sub_env) blocks d0, d1; split(key_s, 3) blocks c0, c1, c2 (env_step's naming)
  const uint2 d0 = threefry(sub_env.x, sub_env.y, 0u, 2u), d1 = threefry(sub_env.x, sub_env.y, 1u, 3u);
  const uint2 c0 = threefry(d0.x, d1.x, 0u, 3u), c1 = threefry(d0.x, d1.x, 1u, 4u), c2 = threefry(d0.x, d1.x, 2u, 5u);
  const int resp = respawn_draws<NMAX>(lev, (1 << NMAX) - 1, make_uint2(c2.x, c0.y));
  const uint32_t tbits = threefry(c0.x, c1.x, 0u, 0u).x;
  draw4 r = {cbits, tbits, (unsigned)resp, 0u};
  return r;
}

// One train-rollout worker on the state-independent draws of its steps (the env chain of the three-launch rollouts,
// toued_rollout_env, and of the A2C chain, toued_a2c_chain): the level record in registers, the five candidate next
// actor rows gathered before the choice (the next state of a step that does not end the episode is a function of
// the action and the step's draws), the gymnax auto-reset (reset_env<TAB> draws nothing on the tabular levels).  One
// code path for both kernels, so their trajectories are bit-identical.  CAND = false (the default of both launchers):
// no candidate gathers, the chosen next row is gathered after the step -- one dependent round trip per step beats
// five 64-lane row gathers ahead of the choice here (W = 64 workers of one agent per wave; measured).
//
// NPT (the A2C chain): the move and the object test come from a per-level transition table in LDS, [G2][5] entries
// next cell | (mask of the objects placed there) << 8, built once per launch by build_npt -- one LDS read per step
// instead of next_pos_r's boundary tests, wall-word select and the object loop (~50 VALU); the same values.
template <int NMAX, bool CAND = true, bool NPT = false>
struct TrainWorker {
  LevR lev;
  EnvState s;
  uint32_t wl[8];
  int objpos[NMAX];
  int G2, used, max_steps, grid, start, idx, ridx;
  float row[5], last[5], rrow[5];   // rrow: the auto-reset observation's row (a constant index per worker)
  __amdgpu_buffer_rsrc_t rs_t;
  unsigned tab_off;
  const uint16_t* npt;   // NPT: the transition table (LDS)

  // worker i (agent a) of a batch of n workers; the state from state [S_FIELDS][n]
  TOUED_DEV void init(const EnvSpec& sp, const int* __restrict__ levels, int a, const float* __restrict__ theta, int D,
                      const int* __restrict__ state, int n, int i) {
    lev = lev_regs(levels + (size_t)a * LEVEL_WORDS);
    rs_t = theta_rsrc(theta);
    tab_off = (unsigned)((size_t)a * D * 20);
    load_state<NMAX>(state, n, i, s);
    G2 = sp.max_grid * sp.max_grid;
    const int nobj = lev_i(lev, L_NOBJS);
    used = nobj >= 32 ? -1 : ((1 << nobj) - 1);
    max_steps = lev_i(lev, L_MAX_STEPS);
    grid = lev_i(lev, L_GRID);
    start = lev_i(lev, L_START);
#pragma unroll
    for (int k = 0; k < 8; ++k) wl[k] = wall_word(lev, k);
#pragma unroll
    for (int o = 0; o < NMAX; ++o) objpos[o] = s.obj[o] - lev_i(lev, L_OBJ_IDS + o) * G2;   // static in TAB
    idx = tab_index(sp, s);
    ridx = start + G2 * (used & ((1 << NMAX) - 1));
  }

  // NPT: entries c0, c0 + nc, ... of the transition table (all of a workgroup's workers share the level and so the
  // static object cells objpos)
  TOUED_DEV void build_npt(uint16_t* tbl, int c0, int nc) const {
    for (int c = c0; c < G2 * 5; c += nc) {
      const int p = next_pos_r(grid, wl, c / 5, c - (c / 5) * 5);
      int m = 0;
#pragma unroll
      for (int o = 0; o < NMAX; ++o)
        if (objpos[o] == p) m |= 1 << o;
      tbl[c] = (uint16_t)(p | (m << 8));
    }
  }

  // the actor rows a rollout starts from: the time row D-1, the current observation's row and the reset row
  // (re-read after every update of the table)
  TOUED_DEV void load_rows(const float* __restrict__ tab, int D) {
#pragma unroll
    for (int j = 0; j < 5; ++j) last[j] = tab[(size_t)(D - 1) * 5 + j];
#pragma unroll
    for (int j = 0; j < 5; ++j) row[j] = tab[(size_t)idx * 5 + j];
#pragma unroll
    for (int j = 0; j < 5; ++j) rrow[j] = tab[(size_t)ridx * 5 + j];
  }

  // one policy step + step_env (gridworld.py:72-136) + auto-reset on the step's draws dr: returns the observation
  // row index and time the step acted on (obs_idx/obs_time of the trajectory), its action, reward and done
  TOUED_DEV void step(const EnvSpec& sp, const float* __restrict__ tab, draw4 dr, int& o_idx, int& o_time, int& action,
                      float& rew, bool& done) {
    int cpos[5], cex[5];
    float crow[5][5];
    if (CAND) {
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
    }
    o_idx = idx;
    o_time = s.time;
    float p[5];
    actor_probs5_row(row, last, s.time, p);
    action = choice5_bits(dr.x, p);
    int pos = 0, collected = 0;
    if (CAND) {
#pragma unroll
      for (int act = 0; act < 5; ++act)
        if (act == action) {
          pos = cpos[act];
          collected = cex[act];
#pragma unroll
          for (int j = 0; j < 5; ++j) row[j] = crow[act][j];
        }
    } else if constexpr (NPT) {
      const uint32_t e = npt[s.pos * 5 + action];
      pos = (int)(e & 0xFFu);
      collected = (int)(e >> 8) & s.exists;
    } else {
      pos = next_pos_r(grid, wl, s.pos, action);
#pragma unroll
      for (int o = 0; o < NMAX; ++o)
        if (((s.exists >> o) & 1) && objpos[o] == pos) collected |= 1 << o;
    }
    // step_env (gridworld.py:72-136), tabular: env_step's operation order.  Without a collection p_t only feeds the
    // (false) hit test and rew stays 0, so the sums run under a branch most waves skip
    float p_t = 0.0f;
    rew = 0.0f;
    if (collected) {
#pragma unroll
      for (int o = 0; o < NMAX; ++o) {
        const float co = ((collected >> o) & 1) ? 1.0f : 0.0f;
        p_t = __fadd_rn(p_t, __fmul_rn(lev_f(lev, L_PTERM + o), co));
        if ((collected >> o) & 1) rew = __fadd_rn(rew, lev_f(lev, L_REW + o));
      }
    }
    const bool hit = collected != 0 && bits_to_unit(dr.y) < p_t;
    const int term = hit || s.early_term;
    const int time = s.time + 1;
    done = (time >= max_steps) || term;
    if (done) {   // gymnax auto-reset: reset_env<TAB> (gridworld.py:157-182) draws nothing on the tabular levels
      s.time = 0;
      s.pos = start;
      s.exists = used & ((1 << NMAX) - 1);
      s.early_term = 0;
      idx = ridx;   // == tab_index(sp, s)
#pragma unroll
      for (int j = 0; j < 5; ++j) row[j] = rrow[j];
    } else {
      s.time = time;
      s.pos = pos;
      s.exists = (s.exists | (int)dr.z) & ~collected & used;
      s.early_term = term;
      idx = tab_index(sp, s);   // == the candidate row's index: row already holds it
#ifdef A2C_NOGATHER
      // timing only (tools/a2c_stamps.py on an A2C_NOGATHER variant): the env chain without its row gathers
      if (!CAND) {
#pragma unroll
        for (int j = 0; j < 5; ++j) row[j] = rrow[j];
      }
#else
      if (!CAND) load_row5(rs_t, tab_off + (unsigned)idx * 20u, row);
#endif
    }
  }
};

}  // namespace
