/*
 * toued.h — C ABI of libtoued_hip.so, the MI355X (gfx950) hot path of the
 * TO-UED data-parallel inner loop.
 *
 * The reference (nmonette/TO-UED, pure JAX) has no FFI: its operator
 * boundaries are Python interfaces traced into one XLA program.  Each entry
 * point below replaces one of those interfaces (cited per function); the
 * Python host package `toued` (to-ued_amd/toued) mirrors the reference's
 * Python surface on top of this ABI, and INTEGRATION.md shows the ctypes
 * binding a maintainer would add to the reference.
 *
 * Conventions
 *   - Every buffer is a DEVICE pointer owned by the caller (torch tensors in
 *     the Python host).  Kernels never allocate; no hidden global state.
 *   - Every call is asynchronous on `stream` and returns 0 on success, <0 on
 *     error (-1 bad arguments, -2 launch failure); toued_last_error() returns
 *     a thread-local message.  Calls are re-entrant across streams.
 *   - Keys are jax.random threefry keys: uint32[n][2].
 *   - Levels are packed int32[n][64] records (layout in DESIGN.md §Data
 *     layout): scalars, raw obj_ids, static object cells, per-object resolved
 *     reward/p_terminate/p_respawn, 256-bit walls mask.
 *   - Env state is SoA int32[12][n]: time, pos, exists bitmask, early_term,
 *     obj_poss[8].
 *   - Compact observations: tab_idx = pos + max_grid^2 * exists_mask and the
 *     episode time; the reference's dense obs is one_hot(tab_idx) ++ 0.001*t.
 */
#ifndef TOUED_H
#define TOUED_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* hipStream_t;

/* Static env kwargs (environments/gridworld/configs.py:430-544). */
typedef struct {
  int max_grid;  /* max_grid_size */
  int n_max;     /* max_n_objs (1..5) */
  int n_types;   /* max_n_obj_types */
  int tabular;   /* tabular observation / static respawn */
} EnvSpec;

const char* toued_last_error(void);
int toued_abi_version(void);

/* ---- PRNG (jax 0.4.13 threefry, environments/* and meta/* call sites) ---- */
/* out[i][j] = jax.random.split(keys[i], num)[j] */
int toued_split(const uint32_t* keys, int n, int num, uint32_t* out, hipStream_t stream);
/* out[i] = jax.random.fold_in(keys[i], data) */
int toued_fold_in(const uint32_t* keys, int n, uint32_t data, uint32_t* out, hipStream_t stream);
/* out[i][j] = jax.random.bits(keys[i], (m,))[j] */
int toued_random_bits(const uint32_t* keys, int n, int m, uint32_t* out, hipStream_t stream);
/* out[i][j] = jax.random.uniform(keys[i], (m,), minval=lo, maxval=hi)[j] */
int toued_uniform(const uint32_t* keys, int n, int m, float lo, float hi, float* out, hipStream_t stream);

/* ---- Level generator: environments/environments.py:22-37 reset_env_params
 *      + environments/gridworld/configs.py:12-126 (vmapped over keys). ---- */
size_t toued_mode_program_bytes(void);
/* program: device copy of a ModeProgram built by toued/modes.py.
 * buffer_ids may be NULL (0); sub_mode_out may be NULL. */
int toued_level_gen(const void* program, const uint32_t* keys, const int* buffer_ids, int* levels_out,
                    int* sub_mode_out, int n, hipStream_t stream);

/* ---- gymnax Environment plugin API (GridWorld, gridworld.py:72-211) ----
 * Worker i uses levels[i / W]; keys are per worker. */
/* reset(key, params) — gridworld.py:157-182 */
int toued_gw_reset(EnvSpec spec, const int* levels, int W, const uint32_t* keys, int* state, int* obs_idx,
                   int* obs_time, int n, hipStream_t stream);
/* step(key, state, action, params) with auto-reset — gridworld.py:72-136 + gymnax wrapper */
int toued_gw_step(EnvSpec spec, const int* levels, int W, const uint32_t* keys, int* state, const int* actions,
                  int* obs_idx, int* obs_time, float* reward, uint8_t* done, int n, hipStream_t stream);

/* ---- RolloutWrapper (environments/rollout.py:13-102), vmapped over agents ---- */
/* batch_reset(rng, env_params, W) for n_agents agents: worker keys = split(agent_key, W). */
int toued_batch_reset(EnvSpec spec, const int* levels, const uint32_t* agent_keys, int n_agents, int W, int* state,
                      int* obs_idx, int* obs_time, hipStream_t stream);
/* batch_rollout(rng, actor_state, env_params, obs, state) — T policy steps with the
 * linear softmax actor theta[n_agents][D][5].  Trajectory layout: idx/time [N][T+1][W]
 * (slot T = end obs), action/done u8 [N][T][W], reward f32 [N][T][W]; cum_return [N*W].
 * Returns-only mode (all five trajectory pointers NULL, as eval_agent uses it,
 * agents/agents.py:98-106): cum_return only; a worker stops once its first episode
 * ends and `state` is left unmodified. */
int toued_rollout(EnvSpec spec, const int* levels, const float* theta, int D, const uint32_t* agent_keys,
                  int* state, int n_agents, int W, int T, int* traj_idx, int* traj_time, uint8_t* traj_action,
                  float* traj_reward, uint8_t* traj_done, float* cum_return, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* TOUED_H */
