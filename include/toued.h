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
 *     the Python host).  Kernels never allocate.
 *   - Every call is asynchronous on `stream` and returns 0 on success, <0 on
 *     error (-1 bad arguments, -2 launch failure); toued_last_error() returns
 *     a thread-local message.  Calls are re-entrant across streams.
 *   - The only state kept between calls lives in an opaque context object (toued_ctx, below).
 *   - Keys are jax.random threefry keys: uint32[n][2].
 *   - Levels are packed int32[n][80] records (LEVEL_WORDS, layout in DESIGN.md
 *     §Data layout): scalars, raw obj_ids, static object cells, per-object
 *     resolved reward/p_terminate/p_respawn, 256-bit walls mask, type tables.
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

/* Opaque context: the only state the library keeps between calls (today the weight-gradient plans' reserved-CU
 * count, toued_set_reserved_cus).  A process-wide default context is current until a thread makes another one
 * current; the setting is then per thread, so two host threads driving separate streams plan independently.
 * toued_ctx_destroy of the calling thread's current context reverts that thread to the default; destroying a
 * context another thread still has current is refused (-1).  A thread that exits with a context current releases it
 * (a thread-exit guard), so the context can then be destroyed; the check and the delete run under the same lock as
 * toued_ctx_set_current, so no thread can make a context current while it is being destroyed.  The settings are
 * atomic, so threads sharing the
 * default context do not race on them (each sees one of the values written).  Replaces no reference interface: the
 * reference's equivalent state lives in its jitted closures. */
typedef struct toued_ctx toued_ctx;
toued_ctx* toued_ctx_create(void);
int toued_ctx_destroy(toued_ctx* ctx);
int toued_ctx_set_current(toued_ctx* ctx);   /* NULL selects the process default */
toued_ctx* toued_ctx_current(void);

/* ---- device errors and debug hooks ---- */
/* The device error word: kernels with a bounded wait (k_a2c_chain's draw-flag wait, toued_a2c_chain_self) set a bit
 * in it when the wait expires instead of hanging.  wait = 1: synchronise with `stream` and report any error of the
 * work enqueued before the call; wait = 0: never block -- report what the previous call's read-back saw (if it has
 * landed) and enqueue a new read-back.  Returns -3 and sets toued_last_error() when a bit was set (the word is then
 * cleared, and the next read-back is enqueued behind the clear, so an error is reported once), 0 otherwise.  The first call allocates the word (do it outside graph capture: toued_a2c_chain_self
 * refuses to launch before it).  Replaces no reference interface: XLA's scan cannot starve. */
int toued_device_error_check(hipStream_t stream, int wait);
/* --debug (experiments/parse_args.py:7, util/jax.py:12-14 `jax.disable_jit`): hipDeviceSynchronize + hipGetLastError,
 * -1 with the HIP error in toued_last_error() when either fails.  The host calls it after every ABI call in debug mode. */
int toued_sync_check(void);
/* --debug_nans (util/jax.py:9-10 `jax_debug_nans`): *out += the number of NaN/inf floats in x[0..n), stream-ordered
 * (one grid-stride reduction, one atomic per wave). */
int toued_nonfinite_count(const float* x, long n, int* out, hipStream_t stream);
/* the same over rows x cols floats with row pitch ld (a column block of an [rows][ld] operand, e.g. one inner update's
 * GRU state saves) */
int toued_nonfinite_count_2d(const float* x, long rows, long cols, long ld, int* out, hipStream_t stream);

/* ---- PRNG (jax 0.4.13 threefry, environments/* and meta/* call sites) ---- */
/* out[i][j] = jax.random.split(keys[i], num)[j] */
int toued_split(const uint32_t* keys, int n, int num, uint32_t* out, hipStream_t stream);
/* the same keys in planar order: out[j][i] = jax.random.split(keys[i], num)[j] (each j a contiguous key batch) */
int toued_split_planar(const uint32_t* keys, int n, int num, uint32_t* out, hipStream_t stream);
/* out[i] = jax.random.fold_in(keys[i], data) */
int toued_fold_in(const uint32_t* keys, int n, uint32_t data, uint32_t* out, hipStream_t stream);
/* out[i][j] = jax.random.bits(keys[i], (m,))[j] */
int toued_random_bits(const uint32_t* keys, int n, int m, uint32_t* out, hipStream_t stream);
/* out[i][j] = jax.random.uniform(keys[i], (m,), minval=lo, maxval=hi)[j] */
int toued_uniform(const uint32_t* keys, int n, int m, float lo, float hi, float* out, hipStream_t stream);
/* out[i][j] = jax.random.normal(keys[i], (m,))[j] in f32 (sqrt2 * erf_inv(uniform(nextafter(-1, 0), 1)));
 * used by the flax orthogonal initialiser of the LPG GRU (jax/_src/nn/initializers.py orthogonal) */
int toued_normal(const uint32_t* keys, int n, int m, float* out, hipStream_t stream);

/* ---- Level generator: environments/environments.py:22-37 reset_env_params
 *      + environments/gridworld/configs.py:12-126 (vmapped over keys). ---- */
size_t toued_mode_program_bytes(void);
/* program: device copy of a ModeProgram built by toued/modes.py.
 * buffer_ids may be NULL (0); sub_mode_out may be NULL. */
int toued_level_gen(const void* program, const uint32_t* keys, const int* buffer_ids, int* levels_out,
                    int* sub_mode_out, int n, hipStream_t stream);
/* only the levels i with mask[i] != 0 are written (in place: the level sampler's where(terminated, new, old)) */
int toued_level_gen_masked(const void* program, const uint32_t* keys, const int* buffer_ids, int* levels_out, int n,
                           const uint8_t* mask, hipStream_t stream);

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
/* only the workers of the agents a with mask[a] != 0 are reset (in place) */
int toued_batch_reset_masked(EnvSpec spec, const int* levels, const uint32_t* agent_keys, int n_agents, int W,
                             int* state, int* obs_idx, int* obs_time, const uint8_t* mask, hipStream_t stream);
/* batch_rollout(rng, actor_state, env_params, obs, state) — T policy steps with the
 * linear softmax actor theta[n_agents][D][5].  Trajectory layout: idx/time [N][T+1][W]
 * (slot T = end obs), action/done u8 [N][T][W], reward f32 [N][T][W]; cum_return [N*W].
 * Returns-only mode (all five trajectory pointers NULL, as eval_agent uses it,
 * agents/agents.py:98-106): cum_return only; a worker stops once its first episode
 * ends and `state` is left unmodified. */
int toued_rollout(EnvSpec spec, const int* levels, const float* theta, int D, const uint32_t* agent_keys,
                  int* state, int n_agents, int W, int T, int* traj_idx, int* traj_time, uint8_t* traj_action,
                  float* traj_reward, uint8_t* traj_done, float* cum_return, hipStream_t stream);
/* RolloutWrapper.batch_rollout (environments/rollout.py:45-102) in three launches, bit-identical to toued_rollout:
 * the state-independent draws of U batches of train rollouts at once (keys [U][n_agents][2]; chain scratch and draws
 * out u32x4 [T][U * n_agents * W]), then each batch's env chain on its draws (draws = the batch's first worker at
 * step 0, dstride u32x4 elements between steps).  The A2C antagonist's U = max_lifetime update rollouts
 * (agents/a2c.py:79-125) draw everything up front this way. */
int toued_rollout_draws(EnvSpec spec, const int* levels, const uint32_t* keys, int n_agents, int U, int W, int T,
                        uint32_t* chain, uint32_t* draws, hipStream_t stream);
int toued_rollout_env(EnvSpec spec, const int* levels, const float* theta, int D, int* state, int n_agents, int W, int T,
                      const uint32_t* draws, long dstride, int* traj_idx, int* traj_time, uint8_t* traj_action,
                      float* traj_reward, uint8_t* traj_done, float* cum_return, hipStream_t stream);
/* The same returns-only rollout (eval_agent, agents/agents.py:98-106 over rollout.py:45-102) in three launches,
 * bit-identical: the per-worker key chain (chain: uint32[T][n][4], n = n_agents*W), every state-independent draw of
 * every step in parallel (draws: uint32[T][n][4]), then the env chain on those draws (`state` read only). */
int toued_eval_keys(const uint32_t* agent_keys, int n_agents, int W, int T, uint32_t* chain, hipStream_t stream);
int toued_eval_draws(EnvSpec spec, const int* levels, int n_agents, int W, int T, const uint32_t* chain,
                     uint32_t* draws, hipStream_t stream);
int toued_eval_returns(EnvSpec spec, const int* levels, const float* theta, int D, const int* state, int n_agents,
                       int W, int T, const uint32_t* draws, float* cum_return, hipStream_t stream);
/* CUs the non-table toued_eval_returns launch holds for n_workers eval workers (one workgroup each, TOUED_EVAL_BLOCK
 * workers per workgroup): what the caller reserves beside the weight-gradient reduction (toued_set_reserved_cus). */
int toued_eval_returns_cus(int n_workers);


/* ---- Level sampler (environments/level_sampler.py) ---- */
/* frozen mode: random.choice(key, arange(B), p=uniform, shape=(n,), replace=True) (:157-165);
 * cdf = jnp.cumsum(p) in jax's associative-scan order (host-computed once). */
int toued_choice_cdf(const uint32_t* key, const float* cdf, int B, int n, int* out, hipStream_t stream);
/* _reset_lowest_scoring (:338-341): ids = argsort(where(active, inf, where(new, -inf, score)))[:N],
 * stable, jax float order.  Flags are bool (uint8) arrays of length B <= 8192. */
int toued_plr_reset_ids(int B, int N, const float* score, const uint8_t* active, const uint8_t* fresh, int* ids,
                        hipStream_t stream);
/* alg_regret selection (:203-227) on the buffer after the terminated-level update.
 * keys[3][2] = {replay_rng, random_rng, rng} from `rng, replay_rng, random_rng = split(rng, 3)`.
 * Outputs (int32[N]): chosen = where(use, replay, random), replay (_replay_from_buffer :355-390,
 * rank if !proportional), random (_sample_random_from_buffer :392-408), use (0/1). */
int toued_plr_sample(int B, int N, const float* score, const uint8_t* active, const uint8_t* fresh,
                     const uint32_t* keys, int proportional, float temperature, float p_replay, int* chosen, int* rep,
                     int* rnd, int* use_out, hipStream_t stream);

/* ---- Agents (agents/agents.py:31-95; models/agent.py:7-45) ---- */
/* Dense(cols, use_bias=False) lecun_normal kernels [n][D][cols]: truncated_normal(keys[i]) in
 * [lo, hi] = erf(-+2/sqrt2), times stddev.  keys are the flax per-param keys (toued/agents.py). */
int toued_init_tables(const uint32_t* keys, int n, int cols, int D, float lo, float hi, float stddev, float* out,
                      hipStream_t stream);
/* only the tables i with mask[i] != 0 are written (in place) */
int toued_init_tables_masked(const uint32_t* keys, int n, int cols, int D, float lo, float hi, float stddev,
                             float* out, const uint8_t* mask, hipStream_t stream);
/* level_sampler.sample with score_function=random (level_sampler.py:134-194): the termination test and all key
 * derivations for this rank's n agents (global indices lo .. lo+n-1 of n_total) in one launch.  mask [n] (u8) =
 * step >= levels[:, lifetime]; step (and vstep, when not NULL) zeroed where set; keys [4 or 5][n][2]: the new level's
 * key, the env reset key, the actor and critic table keys already folded with dense_hash (lecun_tables' Dense_0), and
 * with vstep the value critic's folded key.  rng [2] is the sampler's key (jax.random.split chains as in the
 * reference). */
int toued_sample_random_keys(const uint32_t* rng, int n_total, int lo, int n, int* step, const int* levels, int* vstep,
                             uint32_t dense_hash, uint8_t* mask, uint32_t* keys, hipStream_t stream);

/* ---- A2C antagonist (agents/a2c.py:19-125) ---- */
/* out[u][i] = the u-th `_rng` of `rng, _rng = split(rng)` chained from keys[i] (a2c.py:97). */
int toued_key_chain(const uint32_t* keys, int n, int U, uint32_t* out, hipStream_t stream);
/* a2c_agent_train_step gradients for N agents (a2c.py:29-68) from a trajectory in the
 * toued_rollout layout; accumulates into Ga [N][D][5], Gv [N][D] (zeroed by the caller or by
 * toued_a2c_apply) and loss_out[N][2] += {actor_loss, critic_loss}.  W*T <= ~5400. */
int toued_a2c_grad(int N, int W, int T, int D, const float* theta, const float* vcrit, const int* tidx,
                   const int* ttime, const uint8_t* tact, const float* trew, const uint8_t* tdone, float gamma,
                   float lam, float ent_coef, float* Ga, float* Gv, float* loss_out, hipStream_t stream);
/* fused, deterministic A2C update (grad + clip + SGD in one block per agent; rows summed in sample order after
 * an LDS sort by (row, sample), no atomics) for sizes where toued_a2c_update_fits(W, T, D) is 1 (W*T <= 2048) */
int toued_a2c_update_fits(int W, int T, int D);
int toued_a2c_update(int N, int W, int T, int D, float* theta, float* vcrit, const int* tidx, const int* ttime,
                     const uint8_t* tact, const float* trew, const uint8_t* tdone, float gamma, float lam,
                     float ent_coef, float lr_a, float lr_c, float max_norm, int* step, const int* levels,
                     float* loss_out, hipStream_t stream);
/* train_a2c_agent's whole scan (a2c.py:79-125) in one launch: U updates (rollout + fused update) of N antagonists,
 * one workgroup each, on the state-independent draws toued_rollout_draws made for the U update keys (toued_key_chain
 * of the agents' rng): draws [T][dstride] uint32x4, update u's worker i at column u*N*W + i.  theta/vcrit/step/state
 * updated in place, loss_out[N][2] accumulated.  Bit-identical, update by update, to toued_rollout_env +
 * toued_a2c_update.  Tabular envs, sizes where toued_a2c_chain_fits(W, T, D) is 1 (W <= 256, W*T <= 2048). */
int toued_a2c_chain_fits(int W, int T, int D);
/* 1 when toued_a2c_chain_self supports these sizes: toued_a2c_chain_fits, W <= 64 (one env wave), T <= 64 (one draw
 * flag per step); else use toued_a2c_chain with toued_rollout_draws. */
int toued_a2c_chain_self_fits(int W, int T, int D);
int toued_a2c_chain(EnvSpec spec, const int* levels, int N, int W, int T, int D, int U, float* theta, float* vcrit,
                    int* state, const uint32_t* draws, long dstride, float gamma, float lam, float ent_coef, float lr_a,
                    float lr_c, float max_norm, int* step, float* loss_out, hipStream_t stream);
/* The same scan making its own draws (toued_a2c_chain_self_fits): from the U update keys (keys [U][N][2], toued_key_chain's output),
 * each workgroup makes update u + 1's draws in the waves its env chain leaves idle during update u, into scratch
 * u32 [N][2][T][W][4] (a per-agent double buffer).  Bit-identical to toued_rollout_draws + toued_a2c_chain over the
 * same keys, with no draws pass in front of or beside the launch.  A draw wave whose wait for the key wave expires
 * sets a bit of the device error word (toued_device_error_check), which must have been allocated first. */
int toued_a2c_chain_self(EnvSpec spec, const int* levels, int N, int W, int T, int D, int U, float* theta, float* vcrit,
                         int* state, const uint32_t* keys, uint32_t* scratch, float gamma, float lam, float ent_coef,
                         float lr_a, float lr_c, float max_norm, int* step, float* loss_out, hipStream_t stream);
/* --fix_value_critic: one update of the meta-gradient value critics vcrit [N][D] on a trajectory (meta/train.py:61-81
 * with the discarded `.replace` fixed): critic loss mean_w mean_t (target - V)^2 on stop-gradient GAE targets,
 * clip_by_global_norm + SGD (lr, max_norm), vstep[i] += 1; loss_out[i][1] += the loss before the update.
 * Deterministic (the sorted-segment kernel of toued_a2c_update); W*T <= 2048. */
int toued_value_critic_update(int N, int W, int T, int D, float* vcrit, const int* tidx, const int* ttime,
                              const float* trew, const uint8_t* tdone, float gamma, float lam, float lr,
                              float max_norm, int* vstep, float* loss_out, hipStream_t stream);
/* The register bitonic sort behind every sorted-segment kernel (no reference counterpart: it stands for XLA's
 * deterministic scatter-add in a2c.py's gradient), exposed for its parity test: each of nblocks blocks sorts its 2048
 * keys ascending with `threads` (256 or 512) threads; keys and out [nblocks][2048] may not alias. */
int toued_sort_keys2048(const uint32_t* keys, uint32_t* out, int nblocks, int threads, hipStream_t stream);
/* apply_gradients (clip_by_global_norm + SGD, models/optim.py:5-11) for actor and value critic,
 * kept only while step+1 <= levels[i].lifetime (a2c.py:71-75); zeroes Ga/Gv. */
int toued_a2c_apply(int N, int D, float* theta, float* vcrit, float* Ga, float* Gv, float lr_a, float lr_c,
                    float max_norm, int* step, const int* levels, hipStream_t stream);

/* ---- LPG meta-gradient step (meta/train.py:14-130, agents/lpg_agent.py:31-140, models/lpg.py) ----
 * Sample index s = (a*T + t)*W + w; GRU row r = a*W + w; flat LPG parameters eta in
 * jax tree_flatten order (toued/lpg.py LPGLayout), offsets `off`. */
/* per-agent keys of _train_agent (meta/train.py:88-170): K train rollouts, the eval rollout, eval_agent */
int toued_meta_keys(const uint32_t* agent_keys, int N, int K, uint32_t* roll_keys, uint32_t* eval_keys,
                    uint32_t* ea_reset, uint32_t* ea_roll, hipStream_t stream);
/* LPG inputs x = [r, d, pi, e(y_t), e(y_tp1) (, step, lifetime)] (models/lpg.py:48-77) into
 * X[f*xs_f + (t*R + r)*xs_col]; eta_e* point at the embedding-MLP parameters, advanced by a*eta_stride for
 * agent a (ES candidates; 0 = shared) */
int toued_lpg_inputs(int N, int W, int T, int D, int F, const float* theta, const float* phi, const int* tidx,
                     const int* ttime, const uint8_t* tact, const float* trew, const uint8_t* tdone,
                     const float* eta_e1w, const float* eta_e1b, const float* eta_e2w, const float* eta_e2b,
                     const int* step, const int* levels, float* X, long xs_f, long xs_col, long eta_stride,
                     hipStream_t stream);
/* toued_lpg_inputs with one thread per GRU row walking its T steps (W a multiple of 64): each step gathers one critic
 * row and evaluates the embedding MLP once (y_{t+1}'s embedding is the next step's y_t one); bit-identical */
int toued_lpg_inputs_rows(int N, int W, int T, int D, int F, const float* theta, const float* phi, const int* tidx,
                          const int* ttime, const uint8_t* tact, const float* trew, const uint8_t* tdone,
                          const float* eta_e1w, const float* eta_e1b, const float* eta_e2w, const float* eta_e2b,
                          const int* step, const int* levels, float* X, long xs_f, long xs_col, long eta_stride,
                          hipStream_t stream);
/* lpg_agent_train_step gradients (lpg_agent.py:36-70) given pi_hat [T][R], y_hat [T][8][R], added to the
 * zeroed tables Gth/Gph; also gstat[a] = {|G_theta|, |G_phi|, step + 1 <= lifetime} for toued_agent_apply */
int toued_agent_grad(int N, int W, int T, int D, const float* theta, const float* phi, const int* tidx,
                     const int* ttime, const uint8_t* tact, const float* trew, const uint8_t* tdone,
                     const float* pi_hat, const float* y_hat, float alpha_y, float* Gth, float* Gph, float* met,
                     const int* step, const int* levels, float* gstat, hipStream_t stream);
/* clipped SGD of actor [D][5] and LPG critic [D][8] (lpg_agent.py:71-82) from the norms and the lifetime
 * test toued_agent_grad left in gstat; advances step where the update applied */
int toued_agent_apply(int N, int D, const float* th0, const float* ph0, const float* Gth, const float* Gph,
                      float lr_a, float lr_c, float max_norm, int* step, float* th1, float* ph1, const float* gstat,
                      hipStream_t stream);
/* batch_rollout_entropy (util/metrics.py:5-9) metrics, or its gradient scaled by coef_a/coef_c */
int toued_entropy(int N, int W, int T, int D, const float* theta, const float* phi, const int* tidx, const int* ttime,
                  float* met, float coef_a, float coef_c, float* adj_th, float* adj_ph, hipStream_t stream);
/* meta/train.py:61-100: frozen value critic GAE, normalised advantage, lpg_loss and value_loss */
int toued_eval_loss(int N, int W, int T, int D, const float* theta, const float* vcrit, const int* tidx,
                    const int* ttime, const uint8_t* tact, const float* trew, const uint8_t* tdone, float gamma,
                    float lam, float* adv_scratch, float* abar, float* out, hipStream_t stream);
/* d lpg_loss / d theta_K */
int toued_lpgloss_grad(int N, int W, int T, int D, const float* theta, const int* tidx, const int* ttime,
                       const uint8_t* tact, const float* abar, float* adj_th, hipStream_t stream);
/* VJP coefficients of clip_by_global_norm (optax) per agent */
int toued_clip_dot(int N, int D, const float* Gth, const float* Gph, const float* adj_th, const float* adj_ph,
                   const float* gstat, float lr_a, float lr_c, float max_norm, float* coef, hipStream_t stream);
/* Hessian-vector products through one LPG agent update + cotangents on pi_hat / y_hat */
int toued_hvp(int N, int W, int T, int D, int K, const float* theta, const float* phi, const int* tidx,
              const int* ttime, const uint8_t* tact, const float* pi_hat, const float* y_hat, const float* Gth,
              const float* Gph, const float* adj_th_in, const float* adj_ph_in, const float* coef, float lr_a,
              float lr_c, float alpha_y, float b2, float b3, float* adj_th_out, float* adj_ph_out, float* d_pi_hat,
              float* d_y_hat, hipStream_t stream);
/* embedding-MLP (models/lpg.py:36-46) parameter gradient from the GRU input cotangents.  phi_hist: K + 1 critic-table
 * slots phi_stride floats apart, update k's phi_k in slot (phi_slot0 + k) % (K + 1) (a ring of the step's history) */
int toued_embed_bwd(int N, int W, int T, int D, int K, const float* phi_hist, long phi_stride, int phi_slot0,
                    const int* tidx_hist,
                    long tidx_stride, const int* ttime_hist, const uint8_t* tdone_hist, long tstep_stride,
                    const float* dX3, const float* dX4, long dx_stride_k, const float* e1w, const float* e1b,
                    const float* e2w, float* partial, int n_blocks, hipStream_t stream);
/* out[dst_idx[i]] += src[src_idx[i]] for i < n, the dst indices distinct (index_add_ with unique indices): the GRU
 * weight-gradient blocks (G | GI) into eta's flat gradient layout in one launch */
int toued_gather_add(float* out, const float* src, const int* src_idx, const int* dst_idx, int n, hipStream_t stream);
/* out[j] += sum_{i < rows} part[i * cols + j]: the embedding gradient's per-block partials (toued_embed_bwd) into the
 * flat gradient.  Deterministic but not a serial sum: 256 strided partials (partial t sums rows t, t + 256, ... in
 * ascending order), then a fixed pairwise tree over the 256 partials (t += t + 128, then + 64, ... + 1). */
int toued_sum_rows_add(const float* part, int rows, int cols, float* out, hipStream_t stream);
/* optax 0.1.5 chain(scale_by_adam(b1, b2, eps), scale(lr), scale(-1)) on the flat eta (models/optim.py:12-17),
   applied to grad / n_mean (the agent mean, meta/train.py:128).  b1, b2 are the python floats (double) so that
   (1 - b) rounds to f32 once, as jax's weak-typed constants do; count is the post-increment step (>= 1). */
int toued_adam(int P, float* eta, const float* grad, float* m, float* v, float n_mean, float lr, double b1, double b2,
               float eps, int count, hipStream_t stream);

/* util/metrics.py:17-38 gae(value, reward, done, discount, gae_lambda) for N x W workers at once: value
 * [N][T+1][W], reward [N][T][W] f32, done [N][T][W] u8 -> advantages adv and value targets target [N][T][W];
 * gamma_lambda = f32(discount * gae_lambda) as the reference's python-float product.  Bit-exact with the f32
 * restatement (the reference's operation order, no contraction).  The meta-gradient and A2C kernels run the same
 * scan fused on their staged trajectories (k_eval_loss, k_a2c_update). */
int toued_gae(int N, int W, int T, const float* value, const float* reward, const uint8_t* done, float gamma,
              float gamma_lambda, float* adv, float* target, hipStream_t stream);

/* ---- LPG reverse-time GRU on MFMA (models/lpg.py:11-35, flax GRUCell) ---- */
size_t toued_gru_packed_floats(int which);
/* repack eta's GRU weights into MFMA A-fragment order (fwdA / bwdA) */
int toued_gru_pack(const float* eta, const int* off, int F, float* fwdA, float* bwdA, hipStream_t stream);
/* forward over R rows x T steps (t = T-1 .. 0, h reset on done); X[f*xs_f + (t*R + r)*xs_col];
 * heads pi_hat [T][R], y_hat [T][8][R]; saves h_in, r, z, n, W_hn h + b_hn for the backward: as [256][M] rows
 * (pointer at this update's first column, row stride M) on the f32 kernels, or -- where toued_gru_slab_saves(R) --
 * h_in in 32-column slab blocks [M/32][256][32] (element (u, m) at ((m >> 5)*256 + u)*32 + (m & 31)) and r, z,
 * W_hn h + b_hn in 32-column unit-quad blocks [M/32][64][32][4] (element (u, m) at (m >> 5)*8192 + ((u >> 2)*32 +
 * (m & 31))*4 + (u & 3)); pointers at this update's first block, base + 256 * first column; n only by the f32
 * kernels (rows) */
int toued_gru_fwd(int R, int T, int W, int F, const float* X, long xs_f, long xs_col, const uint8_t* done,
                  const float* fwdA, const float* eta, const int* off, float* pi_hat, float* y_hat, float* s_hin,
                  float* s_r, float* s_z, float* s_n, float* s_hn, long M, hipStream_t stream);
/* VJP over K updates (M = K*T*R columns): gate cotangents DG [4][256][M] (dr, dz, d(W_hn h + b_hn), dn),
 * relu(h_out) RH [256][M] (row 256 of the caller's [257][M] buffer holds ones), head cotangents DH [9][M],
 * input cotangents dX3/dX4 [K][T][R]; col_exp [M] (optional, written when toued_gru_bwd_col_exp(R)): each
 * column's cotangent scale exponent for toued_wgrad_bfp */
int toued_gru_bwd(int R, int T, int W, int K, const uint8_t* done, long done_stride_k, const float* bwdA,
                  const float* eta, const int* off, const float* y_hat, const float* d_pi_hat, const float* d_y_hat,
                  const float* s_hin, const float* s_r, const float* s_z, const float* s_n, const float* s_hn, long M,
                  float* DG, float* RH, float* DH, float* dX3, float* dX4, int8_t* col_exp, hipStream_t stream);
/* 1 when toued_gru_bwd runs its lockstep split-precision kernel for R rows (the one that writes col_exp) */
int toued_gru_bwd_col_exp(int R);
/* 1 when the forward and backward for R rows keep r, z, W_hn h + b_hn in 32-column unit-quad blocks (see
 * toued_gru_fwd): the split-precision pair's 16-byte stores and loads of a lane's four consecutive units */
int toued_gru_slab_saves(int R);
/* 1 when h_in is in slab blocks (A's first 256 rows' region; 0 only in HIN_SLAB=0 comparison builds) */
int toued_gru_hin_slab(void);
/* 1 when toued_gru_bwd_fused applies: the lockstep kernel for R rows and LPG input width F <= 6 */
int toued_gru_bwd_fused_fits(int R, int F);
/* floats of `work` toued_gru_bwd_fused needs: per-workgroup partials of the small products + their chunk sums */
size_t toued_gru_bwd_fused_work_floats(int R, int K);
/* the VJP with the small weight-gradient products fused (replaces toued_gru_bwd + toued_gru_bwd_small where it fits):
 * DG3 = dr, dz, d(W_hn h + b_hn) (the main reduction's B operand, for toued_wgrad_bfp_slab), each gate in 32-column
 * slab blocks [M/32][256][32] (element (u, m) of gate g at g*256*M + ((m >> 5)*256 + u)*32 + (m & 31)), dX3/dX4,
 * col_exp (required), and GI as toued_gru_bwd_small writes it; dn, relu(h_out) and the head cotangents stay on chip
 * (no s_n: n is recomputed).  Deterministic: per-workgroup partials summed in a fixed order. */
int toued_gru_bwd_fused(int R, int T, int W, int K, const uint8_t* done, long done_stride_k, const float* bwdA,
                        const float* eta, const int* off, const float* y_hat, const float* d_pi_hat,
                        const float* d_y_hat, const float* s_hin, const float* s_r, const float* s_z,
                        const float* s_hn, long M, float* DG3, float* dX3, float* dX4, int8_t* col_exp, float* GI,
                        float* work, size_t work_floats, hipStream_t stream);
/* the backward's small weight-gradient products: GI = [8][256] ([X; 1; 0] . dn^T: dW_in rows, b_in) followed by
 * [9][257] (DH . [relu(h_out); 1]^T: head kernels and biases); X rows start at s_hin + 256*M.
 * `work`: toued_gru_bwd_small_work_floats(M) floats. */
size_t toued_gru_bwd_small_work_floats(long M);
int toued_gru_bwd_small(long M, const float* s_hin, const float* DG, const float* RH, const float* DH, float* GI,
                        float* work, size_t work_floats, hipStream_t stream);

/* weight-gradient reduction C[ra][rb] = A[ra x K] . B[rb x K]^T (row strides lda, ldb; K % 32 == 0,
 * ra <= 272) on f32 MFMA, split over K with per-chunk partials in `work` (toued_wgrad_workspace_floats)
 * summed in chunk order (deterministic).  Replaces the weight-gradient GEMMs of the LPG backward
 * (jax.vjp of models/lpg.py:11-35 and :79-85 under meta/meta.py:177-181) */
size_t toued_wgrad_workspace_floats(int ra, int rb, long K);
int toued_wgrad(int ra, int rb, long K, const float* A, long lda, const float* B, long ldb, float* C, float* work,
                size_t work_floats, hipStream_t stream);
/* toued_wgrad into C with row stride ldc */
int toued_wgrad_ldc(int ra, int rb, long K, const float* A, long lda, const float* B, long ldb, float* C, int ldc,
                    float* work, size_t work_floats, hipStream_t stream);
/* C[i * ldc] = sum_k A[i][k] (row stride lda; K and lda multiples of 4), deterministic (chunk partials in work) */
size_t toued_rowsum_workspace_floats(int ra, long K);
int toued_rowsum_into(int ra, long K, const float* A, long lda, float* C, int ldc, float* work, size_t work_floats,
                      hipStream_t stream);
/* The LPG's main weight-gradient reduction on block-floating-point fp16 pairs (3 products instead of the bf16
 * split's 6): rows [0, a_unit_rows) of A must satisfy |a| <= 1 (scale 2^14), the others are scaled from their
 * measured maximum; col_exp[m] (from toued_gru_bwd) scales B's columns per K chunk.  Deterministic. */
size_t toued_wgrad_bfp_workspace_floats(int ra, int rb, long K);
int toued_wgrad_bfp(int ra, int rb, long K, const float* A, long lda, int a_unit_rows, const float* B, long ldb,
                    const int8_t* col_exp, float* C, float* work, size_t work_floats, hipStream_t stream);
/* the same with operands in 32-column slab blocks (the split-precision GRU pair's layouts, toued_gru_slab_saves):
 * layout bit 0 = A's rows [0, 256) (h_in) in slab blocks [K/32][256][32] at A, its rows 256.. in [ra][lda] rows
 * after them (needs ra > 256, a_unit_rows == 256); bit 1 = B in slab blocks of 256 rows [rb/256][K/32][256][32]
 * (toued_gru_bwd_fused's DG3; rb % 256 == 0; ldb unused).  Each workgroup's slabs are then contiguous 32 KB pieces
 * instead of 128-byte row segments.  Workspace as toued_wgrad_bfp. */
int toued_wgrad_bfp_slab(int ra, int rb, long K, const float* A, long lda, int a_unit_rows, const float* B, long ldb,
                         int layout, const int8_t* col_exp, float* C, float* work, size_t work_floats,
                         hipStream_t stream);

/* CUs the split-K weight-gradient plans leave free (default 0): a kernel running on a side stream beside them (the
 * eval_agent rollout) then occupies its own CUs instead of pushing one workgroup of every chunk into a second
 * round.  Workspace sizes queried before the change stay sufficient (fewer chunks).  Sets the current context's
 * value (toued_ctx_current) and returns its previous value. */
int toued_set_reserved_cus(int n);
/* Tests only: count every tile claim of the following toued_wgrad_bfp launches into visits[tile] (device int array of
 * `capacity` entries, the caller zeroes it; capacity 0 switches counting off), and the tile count of the last launch.
 * A tile claimed twice or never by k_wgrad_h3's per-XCD queues shows as a count != 1. */
int toued_dbg_wgrad_visits(int* visits, int capacity);
int toued_dbg_wgrad_last_ntiles(void);

/* toued_agent_grad + toued_agent_apply fused, in place, for an agent chain that never reads the gradient tables
 * (the ES candidates): clip + SGD on theta [N][D][5] / phi [N][D][8] of the touched rows only (bit-identical to
 * the pair on zeroed tables), step advanced when applied, met accumulated, gstat [N][4] written.  Sizes where
 * toued_agent_update_fits(W, T, D) is 1 (T*W <= 2048). */
int toued_agent_update_fits(int W, int T, int D);
int toued_agent_update(int N, int W, int T, int D, float* theta, float* phi, const int* tidx, const int* ttime,
                       const uint8_t* tact, const float* trew, const uint8_t* tdone, const float* pi_hat,
                       const float* y_hat, float alpha_y, float lr_a, float lr_c, float max_norm, float* met, int* step,
                       const int* levels, float* gstat, hipStream_t stream);

/* The meta-gradient's inner update k (agents/lpg_agent.py:88-140 inside meta/train.py:41-58) without dense table
 * passes: replaces toued_agent_grad + toued_agent_apply where toued_agent_update_fits(W, T, D).  theta1 / phi1 must
 * already hold copies of theta / phi (theta_k); the touched rows of theta1 / phi1 are rewritten (bit-identical to
 * toued_agent_apply), the touched gradient rows go to Gth / Gph (bit-identical to toued_agent_grad on zeroed tables
 * there; the other rows are NOT written).  The reverse pass (meta/train.py:174) reads touched rows only:
 * toued_entropy_clip is toued_entropy's gradient mode + toued_clip_dot over those rows in one kernel, toued_hvp
 * reads the rows of its own samples. */
int toued_agent_step(int N, int W, int T, int D, const float* theta, const float* phi, float* theta1, float* phi1,
                     const int* tidx, const int* ttime, const uint8_t* tact, const float* trew, const uint8_t* tdone,
                     const float* pi_hat, const float* y_hat, float alpha_y, float lr_a, float lr_c, float max_norm,
                     float* Gth, float* Gph, float* met, int* step, const int* levels, float* gstat, hipStream_t stream);
/* toued_agent_step, then toued_entropy's metric mode on the updated tables theta1 / phi1 (met slots 3 and 4) in the
 * same launch: bit-identical to toued_agent_step followed by toued_entropy(..., theta1, phi1, ..., met, 0, 0, NULL,
 * NULL) (lpg_agent.py:119-120's batch_rollout_entropy of the new policy on rollout k). */
int toued_agent_step_entropy(int N, int W, int T, int D, const float* theta, const float* phi, float* theta1,
                             float* phi1, const int* tidx, const int* ttime, const uint8_t* tact, const float* trew,
                             const uint8_t* tdone, const float* pi_hat, const float* y_hat, float alpha_y, float lr_a,
                             float lr_c, float max_norm, float* Gth, float* Gph, float* met, int* step,
                             const int* levels, float* gstat, hipStream_t stream);
/* The per-agent metrics of a meta-step (meta/train.py:101-117) from met [K][N][8] (k_agent_grad / k_entropy slots) and
 * loss_out [N][2]: out [6][N] = reg_lpg_loss, policy_l2, policy_entropy, critic_loss, critic_l2, critic_entropy */
int toued_meta_metrics(int N, int K, const float* met, float inv_wt, const float* loss_out, float pec, float pl2,
                       float tec, float tl2, float* out, hipStream_t stream);
int toued_entropy_clip(int N, int W, int T, int D, const float* theta, const float* phi, const int* tidx,
                       const int* ttime, float coef_a, float coef_c, float* adj_th, float* adj_ph, const float* Gth,
                       const float* Gph, const float* gstat, float lr_a, float lr_c, float max_norm, float* coef,
                       hipStream_t stream);

/* The reverse pass's step k (meta/train.py:174's scan body) in one launch: toued_entropy_clip on theta1 / phi1
 * (theta_{k+1}, phi_{k+1}), then toued_hvp on theta / phi (theta_k, phi_k) in place on adj_th / adj_ph, reading the
 * coef the first part wrote; the rollout's samples are sorted once.  Bit-identical to the two calls. */
int toued_entropy_clip_hvp(int N, int W, int T, int D, int K, const float* theta1, const float* phi1,
                           const float* theta, const float* phi, const int* tidx, const int* ttime, const uint8_t* tact,
                           const float* pi_hat, const float* y_hat, float coef_a, float coef_c, float* adj_th,
                           float* adj_ph, const float* Gth, const float* Gph, const float* gstat, float lr_a,
                           float lr_c, float max_norm, float* coef, float alpha_y, float b2, float b3, float* d_pi_hat,
                           float* d_y_hat, hipStream_t stream);

/* ES inference path: pack n candidates' forward fragments (candidate c at eta + c*eta_stride) */
int toued_gru_pack_fwd_multi(const float* eta, long eta_stride, int n, const int* off, int F, float* fwdA,
                             hipStream_t stream);
/* forward with per-candidate parameters: rows [c*rows_per_cand, (c+1)*rows_per_cand) use candidate c
 * (fwdA from toued_gru_pack_fwd_multi); nothing is saved for a backward */
int toued_gru_fwd_multi(int R, int T, int W, int F, int rows_per_cand, const float* X, long xs_f, long xs_col,
                        const uint8_t* done, const float* fwdA, const float* eta, long eta_stride, const int* off,
                        float* pi_hat, float* y_hat, hipStream_t stream);

/* ---- OpenES (evosax 0.1.4 as configured by models/optim.py:21-34; meta/train.py:133-227) ---- */
/* ask for z rows [row_lo, row_lo+n_rows) of normal(key, (half_pop, nd)): x[2i] = mean + sigma z_i,
 * x[2i+1] = mean - sigma z_i (the antithetic reorder of meta/train.py:152-158); key is a device key */
int toued_es_ask(const uint32_t* key, long nd, long half_pop, long row_lo, long n_rows, const float* mean,
                 float sigma, float* x, hipStream_t stream);
/* out[j] = sum_c ((x[c][j] - mean[j]) / sigma) * fitness[c] over this rank's C candidates */
int toued_es_grad(const float* x, const float* mean, float sigma, const float* fitness, int C, long nd, float* out,
                  hipStream_t stream);
/* evosax optimiser step on the mean with grad*scale: opt 0 = SGD, 1 = Adam (bias corrections bc1, bc2) */
int toued_es_opt(long nd, int opt, float* mean, const float* grad, float scale, float* m, float* v, float lrate,
                 float b1, float b2, float eps, float bc1, float bc2, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* TOUED_H */
