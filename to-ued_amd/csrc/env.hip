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
#include "env_dev.h"

#include <cstdlib>
#include <cstring>

namespace {

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

// The same key chain with the two threefry blocks of each split on a lane pair (lanes 2i, 2i+1: blocks (0,2) and
// (1,3)), exchanged by a DPP quad permute: half the instructions per wave and step for 32 chains per wave.  The
// chain is issue-bound at one wave per SIMD, so eval_agent's few chains (4 per agent) finish in half the time on twice
// the SIMDs; bit-identical to k_eval_keys (the train rollouts' wide chains keep k_eval_keys).
__global__ void __launch_bounds__(1024) k_eval_keys_pairs(const uint32_t* __restrict__ agent_keys, int W, int T, int n,
                                                         uint2* __restrict__ chain) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = g >> 1;
  const uint32_t j = (uint32_t)(g & 1);
  if (i >= n) return;   // both lanes of a pair leave together: the DPP partners below are always active
  const int a = i / W, w = i - a * W;
  uint2 r = split_at(make_uint2(agent_keys[2 * a], agent_keys[2 * a + 1]), (uint32_t)W, (uint32_t)w);
  auto xor1 = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false); };
  // split(r) -> (r', sub): r' = (y0.x, y1.x), sub = (y0.y, y1.y); lane j holds y_j
  auto split_pair = [&](uint2& key, uint2& sub) {
    const uint2 y = threefry(key.x, key.y, j, j + 2u);
    const uint32_t px = xor1(y.x), py = xor1(y.y);
    key = j ? make_uint2(px, y.x) : make_uint2(y.x, px);
    sub = j ? make_uint2(py, y.y) : make_uint2(y.y, py);
  };
  for (int t = 0; t < T; ++t) {
    uint2 sub, sub_env;
    split_pair(r, sub);
    split_pair(r, sub_env);
    chain[((size_t)t * n + i) * 2 + j] = j ? sub_env : sub;   // (sub, sub_env) as one 16-byte record per chain
  }
}

// (n workers per step; worker i plays level (i / W) % na: the train rollouts' U update batches share the levels)
template <int NMAX>
__global__ void __launch_bounds__(256) k_eval_draws(const int* __restrict__ levels, int W, int na, int n, long total,
                                                    const uint4* __restrict__ chain, uint4* __restrict__ draws) {
  const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= total) return;
  const int i = (int)(j % n);
  const int* lev = levels + (size_t)((i / W) % na) * LEVEL_WORDS;
  const uint4 c = chain[j];
  const draw4 d = step_draws<NMAX>(lev, make_uint2(c.x, c.y), make_uint2(c.z, c.w));
  draws[j] = make_uint4(d.x, d.y, d.z, d.w);
}

#ifdef H3_PLACE
__device__ unsigned g_evr_place[64 * 64 * 2];   // (XCC_ID, HW_ID) of eval_returns' workgroups per launch (ring of 64)
__device__ unsigned g_evr_launch;
__global__ void k_evr_next() { if (threadIdx.x == 0) atomicAdd(&g_evr_launch, 1u); }
#endif

// TBL (W a multiple of 64: every wave plays one agent's level): the five candidate moves and their object tests come
// from a per-wave transition table in LDS, [G2][5] entries next cell | (mask of the objects placed there) << 8,
// built once per launch -- five LDS reads per step instead of five next_pos_r and object loops; the same values.
#ifndef EVAL_CHOSEN_ROW
#define EVAL_CHOSEN_ROW 1   // gather only the chosen next row after the choice (0: the five candidates a step ahead)
#endif
template <int NMAX, bool TBL>
__global__ void __launch_bounds__(256) k_eval_returns(EnvSpec sp, const int* __restrict__ levels,
                                                      const float* __restrict__ theta, int D,
                                                      const int* __restrict__ state, int T, int W, int n,
                                                      const uint4* __restrict__ draws, float* __restrict__ cum_return) {
  __shared__ uint16_t tbl[TBL ? 4 : 1][TBL ? 256 * 5 : 1];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;   // (TBL: n is a multiple of 64, so whole waves leave)
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
  uint16_t* tw = tbl[TBL ? (threadIdx.x >> 6) : 0];
  if (TBL) {
    for (int c = threadIdx.x & 63; c < G2 * 5; c += 64) {
      const int p = next_pos_r(grid, wl, c / 5, c - (c / 5) * 5);
      int m = 0;
#pragma unroll
      for (int o = 0; o < NMAX; ++o)
        if (objpos[o] == p) m |= 1 << o;
      tw[c] = (uint16_t)(p | (m << 8));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  float row[5];
  {
    const int idx = tab_index(sp, s);
#pragma unroll
    for (int j = 0; j < 5; ++j) row[j] = tab[(size_t)idx * 5 + j];
  }
  float cum = 0.0f;
  float warm = 0.0f;   // EVAL_CHOSEN_ROW 2: the cache-warming loads' sink (stored nowhere that matters)
  const draw4* dw = reinterpret_cast<const draw4*>(draws);
  draw4 dr0 = {0u, 0u, 0u, 0u};
  if (T > 0) dr0 = dw[i];
  draw4 dr1 = dr0;
  if (T > 1) dr1 = dw[(size_t)n + i];
  for (int t = 0; t < T; ++t) {
    const draw4 dr = dr0;
    dr0 = dr1;
    if (t + 2 < T) dr1 = dw[(size_t)(t + 2) * n + i];
    // next state of each action while the episode goes on: position, objects left
    int cpos[5], cex[5];
    float crow[EVAL_CHOSEN_ROW ? 1 : 5][5];
#pragma unroll
    for (int act = 0; act < 5; ++act) {
      int p, col = 0;
      if (TBL) {
        const uint32_t e = tw[s.pos * 5 + act];
        p = (int)(e & 0xFFu);
        col = (int)(e >> 8) & s.exists;
      } else {
        p = next_pos_r(grid, wl, s.pos, act);
#pragma unroll
        for (int o = 0; o < NMAX; ++o)
          if (((s.exists >> o) & 1) && objpos[o] == p) col |= 1 << o;
      }
      cpos[act] = p;
      cex[act] = col;
      if (!EVAL_CHOSEN_ROW) {
        const int ci = p + G2 * ((s.exists | (int)dr.z) & ~col & used);
        load_row5(rs_t, tab_off + (unsigned)ci * 20u, crow[EVAL_CHOSEN_ROW ? 0 : act]);
      } else if (EVAL_CHOSEN_ROW == 2) {
        // warm the caches with one dword of each candidate row (the chosen row's gather below then hits them)
        const int ci = p + G2 * ((s.exists | (int)dr.z) & ~col & used);
        warm += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_t, (int)(tab_off + (unsigned)ci * 20u), 0, 0));
      }
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
        if (!EVAL_CHOSEN_ROW) {
#pragma unroll
          for (int j = 0; j < 5; ++j) row[j] = crow[act][j];
        }
      }
    if (EVAL_CHOSEN_ROW) {   // one gather of the chosen next row after the choice (its latency in the chain)
      const int ci = pos + G2 * ((s.exists | (int)dr.z) & ~collected & used);
      load_row5(rs_t, tab_off + (unsigned)ci * 20u, row);
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
  if (EVAL_CHOSEN_ROW == 2 && warm == 1.2345e-38f) cum_return[i] = warm;   // keeps the warming loads (never true)
#ifdef H3_PLACE
  if (threadIdx.x == 0 && blockIdx.x < 64) {
    const unsigned slot = g_evr_launch & 63u;
    g_evr_place[(slot * 64 + blockIdx.x) * 2] = (unsigned)__builtin_amdgcn_s_getreg((3 << 11) | 20);
    g_evr_place[(slot * 64 + blockIdx.x) * 2 + 1] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
  }
#endif
}

// ---------------------------------------------------------------- train rollouts in three launches
// The same split for the train rollouts (RolloutWrapper.batch_rollout, rollout.py:45-102, T steps with the gymnax
// auto-reset, trajectories kept): toued_rollout_draws runs k_eval_keys and k_eval_draws over U batches of rollouts at
// once (the A2C antagonist's whole update chain: U x N x W independent key chains), and k_train_env is the env chain
// of one batch on those draws.  On the tabular levels the auto-reset draws nothing (reset_env<TAB> is deterministic),
// so every random decision of a step is in its four draw words.  Bit-identical to k_rollout
// (tests/test_gpu_env.py::test_train_rollout_three_launches).
template <int NMAX, bool CAND>
__global__ void __launch_bounds__(256) k_train_env(EnvSpec sp, const int* __restrict__ levels,
                                                   const float* __restrict__ theta, int D, int* __restrict__ state,
                                                   int T, int W, int n, const uint4* __restrict__ draws, long dstride,
                                                   int* __restrict__ traj_idx, int* __restrict__ traj_time,
                                                   uint8_t* __restrict__ traj_action, float* __restrict__ traj_reward,
                                                   uint8_t* __restrict__ traj_done, float* __restrict__ cum_return) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int a = i / W, w = i - a * W;
  const float* tab = theta + (size_t)a * D * 5;
  TrainWorker<NMAX, CAND> wk;
  wk.init(sp, levels, a, theta, D, state, n, i);
  wk.load_rows(tab, D);
  float cum = 0.0f, valid = 1.0f;
  const size_t base_o = (size_t)a * (T + 1) * W + w, base_t = (size_t)a * T * W + w;
  const draw4* dw = reinterpret_cast<const draw4*>(draws);
  draw4 dr0 = {0u, 0u, 0u, 0u};
  if (T > 0) dr0 = dw[i];
  draw4 dr1 = dr0;
  if (T > 1) dr1 = dw[dstride + i];
  for (int t = 0; t < T; ++t) {
    const draw4 dr = dr0;
    dr0 = dr1;
    if (t + 2 < T) dr1 = dw[(size_t)(t + 2) * dstride + i];
    int oi, ot, action;
    float rew;
    bool done;
    wk.step(sp, tab, dr, oi, ot, action, rew, done);
    cum = __fadd_rn(cum, __fmul_rn(rew, valid));
    valid = __fmul_rn(valid, done ? 0.0f : 1.0f);
    traj_idx[base_o + (size_t)t * W] = oi;
    traj_time[base_o + (size_t)t * W] = ot;
    traj_action[base_t + (size_t)t * W] = (uint8_t)action;
    traj_reward[base_t + (size_t)t * W] = rew;
    traj_done[base_t + (size_t)t * W] = done ? 1 : 0;
  }
  traj_idx[base_o + (size_t)T * W] = wk.idx;
  traj_time[base_o + (size_t)T * W] = wk.s.time;
  store_state<NMAX>(state, n, i, wk.s);
  if (cum_return) cum_return[i] = cum;
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
  // one-wave workgroups: the dispatcher spreads them one per SIMD slot instead of packing four waves per CU
  static const int kb = [] {
    const char* e = getenv("TOUED_EVAL_KEYS_BLOCK");
    return e ? atoi(e) : 64;
  }();
  hipLaunchKernelGGL(k_eval_keys_pairs, dim3((unsigned)((2L * n + kb - 1) / kb)), dim3(kb), 0, stream, agent_keys, W, T,
                     n, reinterpret_cast<uint2*>(chain));
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
                                                        W, n_agents, n, total, reinterpret_cast<const uint4*>(chain),
                                                        reinterpret_cast<uint4*>(draws)));
  TOUED_CHECK_LAUNCH();
  return 0;
}

static int eval_block() {
  static const int v = [] {
    const char* e = getenv("TOUED_EVAL_BLOCK");
    const int b = e ? atoi(e) : 256;
    return b == 64 || b == 128 ? b : 256;
  }();
  return v;
}
// CUs toued_eval_returns' non-table launch holds for n_workers chains (one workgroup per CU)
int toued_eval_returns_cus(int n_workers) { return (n_workers + eval_block() - 1) / eval_block(); }

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
  // the per-wave transition table when every wave plays one level (TOUED_EVAL_TBL=0: the register move maths)
  static const bool tbl_env = !(getenv("TOUED_EVAL_TBL") && strcmp(getenv("TOUED_EVAL_TBL"), "0") == 0);
  const bool tbl = tbl_env && W % 64 == 0 && sp.max_grid * sp.max_grid <= 256;
  if (tbl) {
    TOUED_DISPATCH_NMAX(sp.n_max, true, hipLaunchKernelGGL((k_eval_returns<NMAX, true>), dim3(nblk(n)), dim3(256), 0,
                                                          stream, sp, levels, theta, D, state, T, W, n,
                                                          reinterpret_cast<const uint4*>(draws), cum_return));
  } else {
    // workgroup size (TOUED_EVAL_BLOCK: 64, 128 or 256): smaller blocks spread the chains over more CUs, each with
    // fewer row gathers in flight on its TA (the caller reserves toued_eval_returns_cus() CUs beside the reduction)
    const int bs = eval_block();
    TOUED_DISPATCH_NMAX(sp.n_max, true, hipLaunchKernelGGL((k_eval_returns<NMAX, false>), dim3((n + bs - 1) / bs),
                                                          dim3(bs), 0, stream, sp, levels, theta, D, state, T, W, n,
                                                          reinterpret_cast<const uint4*>(draws), cum_return));
  }
#ifdef H3_PLACE
  hipLaunchKernelGGL(k_evr_next, dim3(1), dim3(64), 0, stream);
#endif
  TOUED_CHECK_LAUNCH();
  return 0;
}

#ifdef H3_PLACE
int toued_dbg_evr_place(unsigned* host, unsigned* launches) {
  if (hipMemcpyFromSymbol(launches, HIP_SYMBOL(g_evr_launch), sizeof(unsigned)) != hipSuccess) return 1;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_evr_place), sizeof(g_evr_place)) == hipSuccess ? 0 : 1;
}
#endif

// the state-independent draws of U batches of train rollouts (T steps, n_agents x W workers each): keys [U][n_agents][2]
// (the rollout keys of each batch), chain scratch and draws out [T][U * n_agents * W] of uint32x4
int toued_rollout_draws(EnvSpec sp, const int* levels, const uint32_t* keys, int n_agents, int U, int W, int T,
                        uint32_t* chain, uint32_t* draws, hipStream_t stream) {
  if (int e = check_spec(sp)) return e;
  TOUED_REQUIRE(sp.tabular, "toued_rollout_draws: tabular envs only");
  TOUED_REQUIRE(n_agents >= 0 && U >= 0 && W >= 1 && T >= 0, "toued_rollout_draws: bad sizes N=%d U=%d W=%d T=%d",
                n_agents, U, W, T);
  const long nl = (long)n_agents * U * W;
  TOUED_REQUIRE(nl < (1L << 31), "toued_rollout_draws: %ld workers", nl);
  const int n = (int)nl;
  if (n == 0 || T == 0) return 0;
  hipLaunchKernelGGL(k_eval_keys, dim3(nblk(n)), dim3(256), 0, stream, keys, W, T, n, reinterpret_cast<uint4*>(chain));
  const long total = (long)n * T;
  TOUED_DISPATCH_NMAX(sp.n_max, true, hipLaunchKernelGGL(k_eval_draws<NMAX>, dim3((unsigned)((total + 255) / 256)),
                                                        dim3(256), 0, stream, levels, W, n_agents, n, total,
                                                        reinterpret_cast<const uint4*>(chain),
                                                        reinterpret_cast<uint4*>(draws)));
  TOUED_CHECK_LAUNCH();
  return 0;
}

// one batch of train rollouts on its draws (draws = the batch's first worker at step 0, step stride dstride
// uint32x4 elements): trajectories, end state and (optional) cum_return exactly as toued_rollout
int toued_rollout_env(EnvSpec sp, const int* levels, const float* theta, int D, int* state, int n_agents, int W, int T,
                      const uint32_t* draws, long dstride, int* traj_idx, int* traj_time, uint8_t* traj_action,
                      float* traj_reward, uint8_t* traj_done, float* cum_return, hipStream_t stream) {
  if (int e = check_spec(sp)) return e;
  TOUED_REQUIRE(sp.tabular, "toued_rollout_env: the linear tabular actor needs a tabular env");
  TOUED_REQUIRE(n_agents >= 0 && W >= 1 && T >= 0, "toued_rollout_env: bad sizes N=%d W=%d T=%d", n_agents, W, T);
  TOUED_REQUIRE(D == sp.max_grid * sp.max_grid * (1 << sp.n_max) + 1, "toued_rollout_env: D=%d != obs_dim", D);
  TOUED_REQUIRE((double)n_agents * D * 20.0 < 4294967295.0, "toued_rollout_env: actor tables (%d x %d rows) exceed 4 GiB",
                n_agents, D);
  const int n = n_agents * W;
  TOUED_REQUIRE(dstride >= n, "toued_rollout_env: draw stride %ld < %d workers", dstride, n);
  TOUED_REQUIRE(traj_idx && traj_time && traj_action && traj_reward && traj_done, "toued_rollout_env: trajectory buffers");
  if (n == 0) return 0;
  // the row gathers: the chosen row after the choice (default; 73 vs 79 us per C2 train rollout) or the five
  // candidate rows ahead of it (TOUED_TRAIN_ROWS=cand; bit-identical)
  static const bool cand = getenv("TOUED_TRAIN_ROWS") && strcmp(getenv("TOUED_TRAIN_ROWS"), "cand") == 0;
  if (cand) {
    TOUED_DISPATCH_NMAX(sp.n_max, true, hipLaunchKernelGGL((k_train_env<NMAX, true>), dim3(nblk(n)), dim3(256), 0,
                                                          stream, sp, levels, theta, D, state, T, W, n,
                                                          reinterpret_cast<const uint4*>(draws), dstride, traj_idx,
                                                          traj_time, traj_action, traj_reward, traj_done, cum_return));
  } else {
    TOUED_DISPATCH_NMAX(sp.n_max, true, hipLaunchKernelGGL((k_train_env<NMAX, false>), dim3(nblk(n)), dim3(256), 0,
                                                          stream, sp, levels, theta, D, state, T, W, n,
                                                          reinterpret_cast<const uint4*>(draws), dstride, traj_idx,
                                                          traj_time, traj_action, traj_reward, traj_done, cum_return));
  }
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
