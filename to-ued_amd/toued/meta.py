"""LPG meta-gradient train step on MI355X (meta/train.py:14-130, meta/meta.py:33-52).

``MetaGradStep(spec...)(rng, eta, agents)`` performs, for all N agents at once:
  forward  K x [fused rollout -> LPG inputs -> MFMA GRU forward -> LPG-agent
           gradient -> clipped SGD (+lifetime discard) -> entropy metrics],
           eval rollout, frozen-value-critic GAE + lpg_loss, eval_agent (4 workers)
  reverse  the explicit adjoint of jax.grad(_train_agent) w.r.t. eta through the
           K clipped-SGD steps: lpg_loss seed, entropy-regulariser gradients,
           clip VJPs, Hessian-vector products, then one batched MFMA GRU backward
           over all K x N x W rows and the weight-gradient GEMMs
  update   mean over agents (all-reduce across ranks when distributed), Adam.

Everything stays on the GPU; the host only enqueues launches.  Per-agent keys
follow meta/train.py exactly (split(rng, N); per agent the scan keys of
train_lpg_agent, then the eval-rollout and eval_agent keys).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch

from . import _lib, prng
from .agents import AgentBatch
from .debug import nan_checker
from .lpg import LPGGRU, LPGLayout, Y
from .rollout import RolloutWrapper, Transition, split_rollouts


@dataclass
class LpgHyperparams:
    """util/data.py:7-35 + the agent/meta hyperparameters the step needs."""
    num_agent_updates: int = 5
    agent_target_coeff: float = 0.5
    policy_entropy_coeff: float = 5e-2
    target_entropy_coeff: float = 1e-3
    policy_l2_coeff: float = 5e-3
    target_l2_coeff: float = 1e-3
    gamma: float = 0.99
    gae_lambda: float = 0.95
    actor_lr: float = 40.0
    critic_lr: float = 4.0
    max_grad_norm: float = 0.5
    lpg_lr: float = 1e-4
    eval_workers: int = 4        # meta/train.py:115
    fix_value_critic: bool = False   # train the value critic (the reference discards its update)


class AdamState:
    """optax.scale_by_adam state for the flat LPG parameters."""

    def __init__(self, P: int, device):
        self.m = torch.zeros(P, dtype=torch.float32, device=device)
        self.v = torch.zeros(P, dtype=torch.float32, device=device)
        self.count = 0


def lpg_inputs_fn(rows: int, W: int) -> str:
    """toued_lpg_inputs_rows (one thread per GRU row over its T steps: half the critic gathers and embedding MLPs) for
    64k rows and more with W a multiple of 64 (the ES candidates: 58.8 vs 66.7 us per launch), else the per-sample
    toued_lpg_inputs (the C2 batch's 32 k rows are too few threads for T-step chains: 42 vs 21 us);
    TOUED_LPG_INPUTS_ROWS=0 / 1 forces either (bit-identical)."""
    force = os.environ.get("TOUED_LPG_INPUTS_ROWS")
    if W % 64 == 0 and (force == "1" or (force is None and rows >= 65536)):
        return "toued_lpg_inputs_rows"
    return "toued_lpg_inputs"


class KernelTimers:
    """HIP-event timing of selected launches on the stream they are enqueued on (torch's current stream)."""

    def __init__(self):
        self.events = {}
        self.enabled = False

    def start(self, name):
        if not self.enabled:
            return None
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return (name, ev)

    def stop(self, tok):
        if tok is None:
            return
        name, ev0 = tok
        ev1 = torch.cuda.Event(enable_timing=True)
        ev1.record()
        self.events.setdefault(name, []).append((ev0, ev1))

    def summary(self):
        """name -> (launches, mean ms); call after synchronize."""
        out = {}
        for k, v in self.events.items():
            ms = [a.elapsed_time(b) for a, b in v]
            out[k] = (len(ms), sum(ms) / len(ms), sum(ms))
        return out

    def reset(self):
        self.events = {}


# the GRU kernels address one batch's K * T * N * W columns (up to 264 floats each) through 32-bit buffer offsets
GRU_MAX_COLUMNS = 4294967295 // (264 * 4) - 1


def gru_max_agents(K: int, T: int, W: int) -> int:
    """The most agents one meta-gradient batch can hold (K updates of T steps, W workers) in the GRU kernels'
    32-bit operand range (635 at K=5, T=20, W=64)."""
    return max(1, GRU_MAX_COLUMNS // (K * T * W))


def local_mini_batches(n_local: int, num_agents: int, num_mini_batches: int, max_chunk: int | None = None) -> int:
    """This rank's sequential chunk count for ``--num_mini_batches``.

    The reference checks the split globally: mini_batch_vmap reshapes all num_agents into num_mini_batches
    equal batches (util/jax.py:25-41), each of num_agents / num_mini_batches agents.  Chunking is a memory bound
    (the summed meta-gradient is the same), so each rank runs its n_local agents as the fewest equal chunks no
    larger than that batch: the smallest divisor of n_local that is >= ceil(n_local / batch).  ``max_chunk`` (the
    kernels' range, gru_max_agents) bounds a chunk the same way, so that a batch too large for one launch runs as
    equal chunks instead of failing."""
    if num_mini_batches < 1 or num_agents % num_mini_batches:
        raise ValueError(f"num_agents={num_agents} does not split into num_mini_batches={num_mini_batches} equal "
                         "mini-batches (util/jax.py:25-41 reshapes them)")
    if n_local < 1:
        raise ValueError(f"this rank holds {n_local} agents")
    batch = num_agents // num_mini_batches
    need = -(-n_local // batch)
    if max_chunk:
        need = max(need, -(-n_local // max_chunk))
    return next(d for d in range(need, n_local + 1) if n_local % d == 0)


class MetaGradStep:
    """``n_agents`` is the agents per call (this rank's); with ``num_mini_batches`` > 1 they run as that many
    sequential chunks of n_agents / num_mini_batches (util/jax.py:25-41 mini_batch_vmap: chunk i holds agents
    [i N/nmb, (i+1) N/nmb)), accumulating the summed meta-gradient before the one all-reduce and Adam step.
    The per-chunk buffers (GRU saves etc.) are sized for one chunk."""

    def __init__(self, rollout: RolloutWrapper, n_agents: int, hyp: LpgHyperparams, lifetime_conditioning: bool,
                 device=None, world=None, num_mini_batches: int = 1, num_agents_global: int | None = None):
        self.n_total_local = n_agents
        self.n_chunks = local_mini_batches(n_agents, num_agents_global or n_agents, num_mini_batches,
                                           gru_max_agents(hyp.num_agent_updates, rollout.train_rollout_len,
                                                          rollout.env_workers))
        n_agents //= self.n_chunks
        self.ro = rollout
        self.N = n_agents
        self.W = rollout.env_workers
        self.T = rollout.train_rollout_len
        self.K = hyp.num_agent_updates
        self.D = rollout.obs_dim
        self.hyp = hyp
        self.F = 7 if lifetime_conditioning else 5
        self.lay = LPGLayout(self.F)
        self.world = world
        dev = torch.device(device) if device is not None else torch.device("cuda")
        self.dev = dev
        N, W, T, K, D = self.N, self.W, self.T, self.K, self.D
        R = N * W
        if R % 32 or W % 32:
            raise ValueError(f"env_workers={W} must be a multiple of 32 for the MFMA GRU row blocks")
        self.R = R
        f32, i32, u8 = torch.float32, torch.int32, torch.uint8
        z = lambda *s, dt=f32: torch.zeros(s, dtype=dt, device=dev)
        # parameter history theta_0 .. theta_K as a ring of K + 1 slots: a step keeps theta_k in slot (r + k) % (K + 1),
        # r = self._ring; the agents' own tables are bound to slot r (theta_0) and after the step to slot r + K
        # (theta_K), which is the next step's theta_0 -- no copy back into a fixed slot
        self._theta_store = z(K + 1, N, D, 5)
        self._phi_store = z(K + 1, N, D, Y)
        self._ring = 0        # this step's slot of theta_0
        self._ring_last = 0   # the last step's (theta_h / phi_h below)
        self.G_th = z(K, N, D, 5)
        self.G_ph = z(K, N, D, Y)
        # inner updates as toued_agent_step (sparse: theta_{k+1} copied on a side stream beside rollout k and the
        # LPG forward, then only the touched rows rewritten; the touched gradient rows kept for the reverse pass's
        # toued_entropy_clip / toued_hvp) where one agent's samples fit the sorted row kernel;
        # TOUED_META_FUSED_STEP=0 keeps the dense grad + apply + entropy + clip_dot path
        self.fused_step = (os.environ.get("TOUED_META_FUSED_STEP", "1") != "0"
                           and bool(_lib.lib().toued_agent_update_fits(W, T, D)))
        # the update's entropy metrics in the same launch (toued_agent_step_entropy); TOUED_STEP_ENTROPY=0: a separate
        # toued_entropy launch (bit-identical)
        self.step_entropy = os.environ.get("TOUED_STEP_ENTROPY", "1") != "0"
        # the reverse pass's entropy-clip and HVP of step k in one launch (toued_entropy_clip_hvp);
        # TOUED_REVERSE_PAIR=0: two launches (bit-identical)
        self.reverse_pair = os.environ.get("TOUED_REVERSE_PAIR", "1") != "0"
        self.gstat = z(K, N, 4)
        self.met = z(K, N, 8)
        self.traj = Transition(z(K + 1, N, T + 1, W, dt=i32), z(K + 1, N, T + 1, W, dt=i32),
                               z(K + 1, N, T, W, dt=u8), z(K + 1, N, T, W), z(K + 1, N, T, W, dt=u8))
        self.pi_hat = z(K, T, R)
        self.y_hat = z(K, T, Y, R)
        self.d_pi_hat = z(K, T, R)
        self.d_y_hat = z(K, T, Y, R)
        self.adv = z(N, W, T)
        self.abar = z(N, W)
        self.loss_out = z(N, 2)
        self.vc_loss = z(N, 2)           # --fix_value_critic update losses (scratch)
        self.adj_th = [z(N, D, 5)]       # adjoint tables, accumulated in place over k (toued_hvp)
        self.adj_ph = [z(N, D, Y)]
        self.coef = z(N, 4)
        # the K train rollouts' keys and the eval rollout's, one buffer (the step's draws take all K + 1 at once)
        self.keys_train = z(K + 1, N, 2, dt=i32)
        self.keys_roll = self.keys_train[:K]
        self.keys_eval = self.keys_train[K]
        self.keys_ea_reset = z(N, 2, dt=i32)
        self.keys_ea_roll = z(N, 2, dt=i32)
        self.gru = LPGGRU(self.lay, R, T, K, W, dev)
        self.X = self.gru.X                      # [F, K, T, R] view into the augmented GEMM operand
        self.grad = z(self.lay.size)
        self.embed_blocks = 768
        self.embed_partial = z(self.embed_blocks, 161)
        self.ea_cum = None
        self.timers = KernelTimers()
        self.side = torch.cuda.Stream(device=dev)
        self._ea_draws = None   # eval_agent draws buffer (rollout.eval_draws), reused every step
        self._draws = None      # the K + 1 train rollouts' draws (rollout.train_draws), reused every step

    # ------------------------------------------------------------------ helpers
    @property
    def theta_h(self) -> torch.Tensor:
        """theta_0 .. theta_K of the last step [K + 1, N, D, 5] (copied out of the ring in that order; slot K holds the
        agents' tables, which the level sampler rewrites in place for terminated agents)."""
        return torch.roll(self._theta_store, -self._ring_last, dims=0)

    @property
    def phi_h(self) -> torch.Tensor:
        return torch.roll(self._phi_store, -self._ring_last, dims=0)

    def _t(self, k: int) -> Transition:
        tr = self.traj
        return Transition(tr.obs_idx[k], tr.obs_time[k], tr.action[k], tr.reward[k], tr.done[k])

    def _eta(self, eta, name):
        return self.lay.view(eta, name)

    # ------------------------------------------------------------------ step
    def __call__(self, rng: torch.Tensor, eta: torch.Tensor, adam: AdamState, agents, rank_slice=None):
        """One meta-gradient train step (meta/train.py:14-130).

        rng: device key [2]; eta: flat LPG params (updated in place); agents: AgentBatch of this rank's
        agents (updated in place: actor/critic tables, steps, env state).  Returns a dict of per-agent metric
        tensors.
        """
        # meta/train.py:121 rng = split(rng, num_agents); under data parallelism every rank derives all N
        # keys and keeps its contiguous slice (identical keys at any world size)
        n_all = self.n_total_local if rank_slice is None else rank_slice[2]
        lo = 0 if rank_slice is None else rank_slice[0]
        keys_all = prng.split(rng, n_all)
        # the GRU fragments of eta (six small launches) on the side stream, beside the step's key, level and draws
        # launches; the first LPG forward waits for them
        main = torch.cuda.current_stream()
        pack_stream = self.side if os.environ.get("TOUED_PACK_SIDE", "1") != "0" else main
        pack_stream.wait_stream(main)
        with torch.cuda.stream(pack_stream):
            self.gru.pack(eta)
            self._packed = torch.cuda.Event()
            self._packed.record(pack_stream)
        self.grad.zero_()
        parts = []
        for c in range(self.n_chunks):
            a0, a1 = c * self.N, (c + 1) * self.N
            if self.n_chunks == 1:
                ag = agents
            else:
                ag = AgentChunk(agents, a0, a1, self.W)
            m = self._chunk(keys_all[lo + a0:lo + a1].contiguous(), eta, ag)
            if self.n_chunks > 1:     # the metric tensors view per-chunk buffers the next chunk overwrites
                m = _map_metrics(m, torch.clone)
                ag.write_back()
            parts.append(m)
        # ---------------- mean over agents (+ all-reduce across ranks), Adam (meta/train.py:127-129)
        n_total = n_all
        if self.world is not None and self.world.size > 1:
            self.world.all_reduce_sum(self.grad)
        nan_checker().check("meta_gradient", self.grad)
        adam.count += 1
        _lib.call("toued_adam", self.lay.size, _lib.ptr(eta), _lib.ptr(self.grad), _lib.ptr(adam.m), _lib.ptr(adam.v),
                  float(n_total), self.hyp.lpg_lr, 0.9, 0.999, 1e-8, adam.count, _lib.stream_ptr())
        nan_checker().check("eta_after_adam", eta)
        if len(parts) == 1:
            return parts[0]
        return _cat_metrics(parts)

    def _chunk(self, agent_keys: torch.Tensor, eta: torch.Tensor, agents):
        """_train_agent (meta/train.py:36-117) for one chunk of N agents: the forward, the eval, and the
        explicit adjoint accumulated into self.grad."""
        L = _lib
        N, W, T, K, D, R = self.N, self.W, self.T, self.K, self.D, self.R
        hyp = self.hyp
        st = L.stream_ptr()
        ptr = L.ptr
        L.call("toued_meta_keys", ptr(agent_keys), N, K, ptr(self.keys_roll), ptr(self.keys_eval),
               ptr(self.keys_ea_reset), ptr(self.keys_ea_roll), st)
        # the history ring's slots in this step's order (theta_k = th[k])
        bound = self.n_chunks == 1 and isinstance(agents, AgentBatch)
        ring = bound and os.environ.get("TOUED_HIST_RING", "1") != "0"
        r0 = self._ring if ring else 0
        th = [self._theta_store[(r0 + k) % (K + 1)] for k in range(K + 1)]
        ph = [self._phi_store[(r0 + k) % (K + 1)] for k in range(K + 1)]
        self._ring_last = r0
        if bound:
            # the agents' tables live in the ring (bound at the first step): theta_0 needs no copy, and theta_K's slot
            # becomes the agents' tables (and the next step's theta_0) at the end
            if agents.theta.data_ptr() != th[0].data_ptr():
                th[0].copy_(agents.theta)
                ph[0].copy_(agents.phi)
                agents.theta = th[0]
                agents.phi = ph[0]
        else:
            th[0].copy_(agents.theta)
            ph[0].copy_(agents.phi)
        if not self.fused_step:   # the fused step writes the touched gradient rows, and nothing reads the others
            self.G_th.zero_()
            self.G_ph.zero_()
        self.met.zero_()
        main = torch.cuda.current_stream()
        e1w, e1b = self._eta(eta, "e1_w"), self._eta(eta, "e1_b")
        e2w, e2b = self._eta(eta, "e2_w"), self._eta(eta, "e2_b")
        state = agents.state
        # the state-independent draws of all K + 1 train-length rollouts of the step (K inner updates + the eval
        # rollout; keys and levels are known now) in one launch instead of one per rollout
        draws = None
        if split_rollouts():
            if self._draws is None:    # the step's own (chain scratch, draws) pair: [T][(K + 1) * N * W][4]
                self._draws = tuple(torch.empty((T, (K + 1) * N * W, 4), dtype=torch.int32, device=self.dev)
                                    for _ in range(2))
            draws = self.ro.train_draws(self.keys_train, agents.levels, W,
                                        self._draws)
        ea = {}

        def start_eval_prep():
            # eval_agent's worker reset, key chain and draws read only the step's keys and the levels; only the env
            # chain on the draws waits for theta_K and the backward
            self.side.wait_stream(main)
            with torch.cuda.stream(self.side):
                (_, _), ea["state"] = self.ro.batch_reset(self.keys_ea_reset, agents.levels, hyp.eval_workers)
                self._ea_draws = self.ro.eval_draws(self.keys_ea_roll, agents.levels, hyp.eval_workers,
                                                    self._ea_draws)
                ea["draws_done"] = torch.cuda.Event()
                ea["draws_done"].record(self.side)

        # ---------------- forward: K inner updates (agents/lpg_agent.py:88-140)
        for k in range(K):
            tk = self._t(k)
            if self.fused_step:
                # theta_{k+1} <- theta_k beside this update's rollout and LPG forward (theta_k is final here)
                self.side.wait_stream(main)
                with torch.cuda.stream(self.side):
                    th[k + 1].copy_(th[k])
                    ph[k + 1].copy_(ph[k])
                    copy_done = torch.cuda.Event()
                    copy_done.record(self.side)
            tok = self.timers.start("rollout")
            if draws is not None:
                self.ro.rollout_from_draws(draws, k, th[k], agents.levels, state, tk)
            else:
                self.ro.batch_rollout(self.keys_roll[k], th[k], agents.levels, state, out=tk,
                                      inplace_state=True)
            self.timers.stop(tok)
            nan_checker().check("rollout_rewards", tk.reward)
            L.call(lpg_inputs_fn(R, W), N, W, T, D, self.F, ptr(th[k]), ptr(ph[k]),
                   ptr(tk.obs_idx), ptr(tk.obs_time), ptr(tk.action), ptr(tk.reward), ptr(tk.done),
                   ptr(e1w), ptr(e1b), ptr(e2w), ptr(e2b), ptr(agents.step), ptr(agents.levels),
                   ptr(self.X) + 4 * k * T * R, self.gru.M, 1, 0, st)
            if k == 0:
                main.wait_event(self._packed)
            tok = self.timers.start("gru_fwd")
            self.gru.forward(k, self.X, tk.done, eta, self.pi_hat, self.y_hat)
            self.timers.stop(tok)
            if k == K - 1 and eval_keys_early() and eval_prep_after_forwards():
                start_eval_prep()
            if nan_checker().enabled:   # the update's saved GRU states h_in [256][T*R] (a column block of the operand)
                nan_checker().check("lpg_gru_states", self.gru.hin_block(k))
            nan_checker().check("lpg_outputs", self.pi_hat[k], self.y_hat[k])
            if self.fused_step:
                # the update and the new policy's entropy metrics (toued_entropy's metric mode) in one launch, once
                # theta_{k+1}'s copy is done (an event: the side stream may hold eval_agent's chain behind it)
                main.wait_event(copy_done)
                L.call("toued_agent_step_entropy" if self.step_entropy else "toued_agent_step", N, W, T, D,
                       ptr(th[k]), ptr(ph[k]), ptr(th[k + 1]), ptr(ph[k + 1]), ptr(tk.obs_idx), ptr(tk.obs_time),
                       ptr(tk.action), ptr(tk.reward), ptr(tk.done), ptr(self.pi_hat[k]), ptr(self.y_hat[k]),
                       hyp.agent_target_coeff, hyp.actor_lr, hyp.critic_lr, hyp.max_grad_norm, ptr(self.G_th[k]),
                       ptr(self.G_ph[k]), ptr(self.met[k]), ptr(agents.step), ptr(agents.levels), ptr(self.gstat[k]),
                       st)
                if not self.step_entropy:
                    L.call("toued_entropy", N, W, T, D, ptr(th[k + 1]), ptr(ph[k + 1]),
                           ptr(tk.obs_idx), ptr(tk.obs_time), ptr(self.met[k]), 0.0, 0.0, None, None, st)
            else:
                L.call("toued_agent_grad", N, W, T, D, ptr(th[k]), ptr(ph[k]), ptr(tk.obs_idx),
                       ptr(tk.obs_time), ptr(tk.action), ptr(tk.reward), ptr(tk.done), ptr(self.pi_hat[k]),
                       ptr(self.y_hat[k]), hyp.agent_target_coeff, ptr(self.G_th[k]), ptr(self.G_ph[k]),
                       ptr(self.met[k]), ptr(agents.step), ptr(agents.levels), ptr(self.gstat[k]), st)
                L.call("toued_agent_apply", N, D, ptr(th[k]), ptr(ph[k]), ptr(self.G_th[k]),
                       ptr(self.G_ph[k]), hyp.actor_lr, hyp.critic_lr, hyp.max_grad_norm, ptr(agents.step),
                       ptr(th[k + 1]), ptr(ph[k + 1]), ptr(self.gstat[k]), st)
                L.call("toued_entropy", N, W, T, D, ptr(th[k + 1]), ptr(ph[k + 1]),
                       ptr(tk.obs_idx), ptr(tk.obs_time), ptr(self.met[k]), 0.0, 0.0, None, None, st)
            nan_checker().check("agent_params", th[k + 1], ph[k + 1])
        # ---------------- value critic on the train rollouts (--fix_value_critic), eval rollout, lpg loss
        if hyp.fix_value_critic:
            self.vc_loss.zero_()
            for k in range(K):
                self._value_critic_update(self._t(k), agents)
        te = self._t(K)
        if draws is not None:
            self.ro.rollout_from_draws(draws, K, th[K], agents.levels, state, te)
        else:
            self.ro.batch_rollout(self.keys_eval, th[K], agents.levels, state, out=te, inplace_state=True)
        L.call("toued_eval_loss", N, W, T, D, ptr(th[K]), ptr(agents.vcrit), ptr(te.obs_idx),
               ptr(te.obs_time), ptr(te.action), ptr(te.reward), ptr(te.done), hyp.gamma, hyp.gae_lambda,
               ptr(self.adv), ptr(self.abar), ptr(self.loss_out), st)
        if hyp.fix_value_critic:
            self._value_critic_update(te, agents)
        # value critic (meta/train.py:61-81).  Reference: `value_critic_state.replace(params=...)` is discarded, the
        # gradient is identically zero, so only the TrainState step advances (K train rollouts + 1
        # eval rollout) and the advantages come from the frozen critic.  --fix_value_critic: K updates on the
        # train rollouts, the advantages and value loss at those parameters, then the eval-rollout update.
        if not hyp.fix_value_critic:
            agents.vstep.add_(K + 1)
        # eval_agent (agents/agents.py:98-106): fresh 4-worker reset, eval-length rollout, mean return.
        # It only reads theta_K and the levels; its sequential chains (key chain, then the env chain on the
        # precomputed draws: rollout.eval_draws / eval_returns_from_draws) hold few CUs (one per 256 eval
        # workers) for ~5 ms, so they run on a side stream beside the weight-gradient reductions, whose split-K
        # plans leave those CUs free.  (Beside the recurrent backward instead, whose 64-row workgroups fill exactly
        # K*R/64/256 rounds of the chip, any CU held pushes that kernel into one more round; beside the
        # latency-bound agent kernels the key chain slowed them by more than it took.)
        key_cus = 2 * -(-N * hyp.eval_workers // 256)   # the key chain: two lanes per eval worker (k_eval_keys_pairs)
        eval_cus = int(L.lib().toued_eval_returns_cus(N * hyp.eval_workers))

        def launch_eval():
            self.side.wait_stream(main)
            if "draws_done" not in ea:
                with torch.cuda.stream(self.side):
                    (_, _), ea["state"] = self.ro.batch_reset(self.keys_ea_reset, agents.levels, hyp.eval_workers)
                    self._ea_draws = self.ro.eval_draws(self.keys_ea_roll, agents.levels, hyp.eval_workers,
                                                        self._ea_draws)
                    # the draws kernel spreads over the whole chip for ~0.1 ms: the main weight-gradient reduction
                    # (one workgroup per CU) starts after it (ea_draws_done), or its workgroups wait behind its blocks
                    ea["draws_done"] = torch.cuda.Event()
                    ea["draws_done"].record(self.side)
            # the small products run beside the key chain, the main reduction beside the env chain
            ea["prev_reserve"] = L.lib().toued_set_reserved_cus(key_cus)

        def before_main_wgrad():
            # (enqueued after the small products) the env chain's 8 workgroups start once the small products are
            # done, beside the main reduction (which plans its tiles around the CUs they hold: k_wgrad_h3's tile
            # queues in wgrad.hip)
            small_done = torch.cuda.Event()
            small_done.record(main)
            self.side.wait_event(small_done)
            with torch.cuda.stream(self.side):
                ea["cum"] = self.ro.eval_returns_from_draws(self._ea_draws, th[K], agents.levels,
                                                            ea["state"])
            main.wait_event(ea["draws_done"])
            if os.environ.get("TOUED_EVAL_ALONE") == "1":
                # timing study: the env chain alone, the main reduction after it on every CU (bit-identical)
                main.wait_stream(self.side)
                return
            L.lib().toued_set_reserved_cus(eval_cus)
        if eval_keys_early() and "draws_done" not in ea:
            # eval_agent's reset, key chain and draws beside the reverse agent loop (latency-bound per-agent kernels)
            # instead of in front of the weight-gradient reduction, which waits for the draws (with the small
            # products fused into the backward nothing else covers them there)
            start_eval_prep()
        # ---------------- reverse: explicit adjoint w.r.t. eta
        a_in = 0
        self.adj_th[a_in].zero_()
        self.adj_ph[a_in].zero_()
        L.call("toued_lpgloss_grad", N, W, T, D, ptr(th[K]), ptr(te.obs_idx), ptr(te.obs_time),
               ptr(te.action), ptr(self.abar), ptr(self.adj_th[a_in]), st)
        for k in range(K - 1, -1, -1):
            tk = self._t(k)
            # d(-b0*H_pi - b1*H_y)/K at (theta_{k+1}, phi_{k+1}) on rollout k, then the clip-VJP coefficients
            if self.fused_step and self.reverse_pair:
                # entropy adjoint + clip coefficients, then the HVP rows, in one launch (one sort of rollout k)
                L.call("toued_entropy_clip_hvp", N, W, T, D, K, ptr(th[k + 1]), ptr(ph[k + 1]),
                       ptr(th[k]), ptr(ph[k]), ptr(tk.obs_idx), ptr(tk.obs_time), ptr(tk.action),
                       ptr(self.pi_hat[k]), ptr(self.y_hat[k]), -hyp.policy_entropy_coeff / K,
                       -hyp.target_entropy_coeff / K, ptr(self.adj_th[a_in]), ptr(self.adj_ph[a_in]),
                       ptr(self.G_th[k]), ptr(self.G_ph[k]), ptr(self.gstat[k]), hyp.actor_lr, hyp.critic_lr,
                       hyp.max_grad_norm, ptr(self.coef), hyp.agent_target_coeff, hyp.policy_l2_coeff,
                       hyp.target_l2_coeff, ptr(self.d_pi_hat[k]), ptr(self.d_y_hat[k]), st)
                continue
            if self.fused_step:
                # one kernel: the entropy gradient's rows are the rows update k touched, so their owners add
                # <G_k, adjoint> as they write them (toued_clip_dot's dot up to the summation order)
                L.call("toued_entropy_clip", N, W, T, D, ptr(th[k + 1]), ptr(ph[k + 1]),
                       ptr(tk.obs_idx), ptr(tk.obs_time), -hyp.policy_entropy_coeff / K,
                       -hyp.target_entropy_coeff / K, ptr(self.adj_th[a_in]), ptr(self.adj_ph[a_in]),
                       ptr(self.G_th[k]), ptr(self.G_ph[k]), ptr(self.gstat[k]), hyp.actor_lr, hyp.critic_lr,
                       hyp.max_grad_norm, ptr(self.coef), st)
            else:
                L.call("toued_entropy", N, W, T, D, ptr(th[k + 1]), ptr(ph[k + 1]),
                       ptr(tk.obs_idx), ptr(tk.obs_time), None, -hyp.policy_entropy_coeff / K,
                       -hyp.target_entropy_coeff / K, ptr(self.adj_th[a_in]), ptr(self.adj_ph[a_in]), st)
                L.call("toued_clip_dot", N, D, ptr(self.G_th[k]), ptr(self.G_ph[k]), ptr(self.adj_th[a_in]),
                       ptr(self.adj_ph[a_in]), ptr(self.gstat[k]), hyp.actor_lr, hyp.critic_lr, hyp.max_grad_norm,
                       ptr(self.coef), st)
            # theta_bar_k = theta_bar_{k+1} + (sparse second-order rows): accumulated in place.  k_rows_sorted reads
            # every sample's adjoint rows before its first row write (the sort's barriers separate the phases), and
            # each agent's tables belong to one workgroup, so no copy of the 144 MB adjoint is needed.
            L.call("toued_hvp", N, W, T, D, K, ptr(th[k]), ptr(ph[k]), ptr(tk.obs_idx),
                   ptr(tk.obs_time), ptr(tk.action), ptr(self.pi_hat[k]), ptr(self.y_hat[k]), ptr(self.G_th[k]),
                   ptr(self.G_ph[k]), ptr(self.adj_th[a_in]), ptr(self.adj_ph[a_in]), ptr(self.coef), hyp.actor_lr,
                   hyp.critic_lr, hyp.agent_target_coeff, hyp.policy_l2_coeff, hyp.target_l2_coeff,
                   ptr(self.adj_th[a_in]), ptr(self.adj_ph[a_in]), ptr(self.d_pi_hat[k]), ptr(self.d_y_hat[k]), st)
        try:
            self.gru.backward(self.traj.done, eta, self.y_hat, self.d_pi_hat, self.d_y_hat, self.X, self.grad,
                              self.timers, after_bwd=launch_eval,
                              before_main_wgrad=before_main_wgrad)
        finally:
            # the CU reservation is process-global split-K planning state: restore it whatever happened
            if "prev_reserve" in ea:
                L.lib().toued_set_reserved_cus(ea["prev_reserve"])
        if "cum" not in ea:
            raise RuntimeError("MetaGradStep: the GRU backward returned without launching eval_agent")
        tr = self.traj
        L.call("toued_embed_bwd", N, W, T, D, K, ptr(self._phi_store), self._phi_store[0].numel(), r0, ptr(tr.obs_idx),
               tr.obs_idx[0].numel(), ptr(tr.obs_time), ptr(tr.done), tr.done[0].numel(), ptr(self.gru.dX3),
               ptr(self.gru.dX4), T * R, ptr(e1w), ptr(e1b), ptr(e2w), ptr(self.embed_partial), self.embed_blocks, st)
        # e1_b, e1_w, e2_b, e2_w are contiguous in eta in the partials' order: the block sums added in one launch
        o = self.lay.offsets["e1_b"]
        assert self.lay.offsets["e2_w"] + 16 == o + 161
        L.call("toued_sum_rows_add", ptr(self.embed_partial), self.embed_blocks, 161, ptr(self.grad) + 4 * o, st)
        # ---------------- agent state out + metrics
        main.wait_stream(self.side)
        ea_cum = ea["cum"]
        ea_cum.record_stream(main)
        ea["state"].record_stream(main)
        nan_checker().check("eval_returns", ea_cum)
        if ring:
            agents.theta = th[K]
            agents.phi = ph[K]
            self._ring = (r0 + K) % (K + 1)
        else:
            agents.theta.copy_(th[K])
            agents.phi.copy_(ph[K])
        # (met * inv_wt).mean over the K updates and the regularised loss, one launch (toued_meta_metrics)
        mo = torch.empty((6, N), dtype=torch.float32, device=self.dev)
        L.call("toued_meta_metrics", N, K, ptr(self.met), 1.0 / (W * T), ptr(self.loss_out),
               hyp.policy_entropy_coeff, hyp.policy_l2_coeff, hyp.target_entropy_coeff, hyp.target_l2_coeff, ptr(mo), st)
        return {
            "lpg_loss": self.loss_out[:, 0], "reg_lpg_loss": mo[0], "value_loss": self.loss_out[:, 1],
            "lpg_agent": {"policy_l2": mo[1], "policy_entropy": mo[2], "critic_loss": mo[3],
                          "critic_l2": mo[4], "critic_entropy": mo[5]},
            "lpg_agent_return": ea_cum.mean(dim=1),
        }

    def _value_critic_update(self, tk: Transition, agents):
        L = _lib
        L.call("toued_value_critic_update", self.N, self.W, self.T, self.D, L.ptr(agents.vcrit), L.ptr(tk.obs_idx),
               L.ptr(tk.obs_time), L.ptr(tk.reward), L.ptr(tk.done), self.hyp.gamma, self.hyp.gae_lambda,
               self.hyp.critic_lr, self.hyp.max_grad_norm, L.ptr(agents.vstep), L.ptr(self.vc_loss), L.stream_ptr())

    def _eval_rollout(self, keys, theta, levels, state):
        """Eval-length rollout that only accumulates returns (no trajectory storage)."""
        N = keys.shape[0]
        n = state.shape[1]
        cum = torch.empty((N, n // N), dtype=torch.float32, device=state.device)
        L = _lib
        L.call("toued_rollout", self.ro._c, L.ptr(levels), L.ptr(theta), theta.shape[1], L.ptr(keys), L.ptr(state),
               N, n // N, self.ro.eval_rollout_len, None, None, None, None, None, L.ptr(cum), L.stream_ptr())
        return cum


class AgentChunk:
    """Agents [a0, a1) of an AgentBatch as the step sees them: row views of the tables (written in place) and a
    contiguous copy of the chunk's env-state columns [12, n*W] (the rollout updates it in place), copied back
    by write_back()."""

    def __init__(self, agents, a0: int, a1: int, W: int):
        self._src = agents
        self._cols = (a0 * W, a1 * W)
        self.levels = agents.levels[a0:a1]
        self.theta = agents.theta[a0:a1]
        self.phi = agents.phi[a0:a1]
        self.step = agents.step[a0:a1]
        self.vcrit = None if agents.vcrit is None else agents.vcrit[a0:a1]
        self.vstep = None if agents.vstep is None else agents.vstep[a0:a1]
        self.state = agents.state[:, self._cols[0]:self._cols[1]].contiguous()

    @property
    def n(self) -> int:
        return self.levels.shape[0]

    def write_back(self):
        self._src.state[:, self._cols[0]:self._cols[1]].copy_(self.state)


def _map_metrics(m, fn):
    return {k: (_map_metrics(v, fn) if isinstance(v, dict) else fn(v)) for k, v in m.items()}


def _cat_metrics(parts):
    out = {}
    for k, v in parts[0].items():
        out[k] = _cat_metrics([p[k] for p in parts]) if isinstance(v, dict) else torch.cat([p[k] for p in parts])
    return out


# ---------------------------------------------------------------------------------------------------------------------
# The reference's functional surface (meta/meta.py:10-52): create_lpg_train_state / make_lpg_train_step returning
# train_step(rng, lpg_train_state, agent_states, value_critic_states) -> the same 4-tuple as lpg_meta_grad_train_step
# (meta/train.py:14-130) and lpg_es_train_step (meta/train.py:133-227).  The device tables are large (144 MB of
# agent tables per copy at N=512), so the step updates them in place and the returned states alias the inputs.


@dataclass
class LpgTrainState:
    """flax ``TrainState`` of the LPG (meta/meta.py:21-24): ``params`` is the flat eta in jax tree order
    (lpg.LPGLayout), ``opt`` the optax Adam state (count, mu, nu); with --use_es ``es`` holds the OpenES strategy and
    state of ``ESTrainState`` (util/data.py:63-68) once the step has been built."""
    params: torch.Tensor
    opt: AdamState | None
    es: object | None = None

    @property
    def step(self) -> int:
        return self.opt.count if self.opt is not None else 0


@dataclass
class ValueCriticStates:
    """The per-agent value critics (agents/agents.py:70-95): params f32 [N, D], step int32 [N]."""
    params: torch.Tensor
    step: torch.Tensor


def lpg_hypers_from_args(args, sampler) -> LpgHyperparams:
    """LpgHyperparams.from_run_args (util/data.py) plus the agent hyperparameters of the level sampler."""
    ah = sampler.agent_hypers
    return LpgHyperparams(
        num_agent_updates=args.num_agent_updates, agent_target_coeff=args.lpg_agent_target_coeff,
        policy_entropy_coeff=args.lpg_policy_entropy_coeff, target_entropy_coeff=args.lpg_target_entropy_coeff,
        policy_l2_coeff=args.lpg_policy_l2_coeff, target_l2_coeff=args.lpg_target_l2_coeff, gamma=args.gamma,
        gae_lambda=args.gae_lambda, actor_lr=ah.actor_learning_rate, critic_lr=ah.critic_learning_rate,
        max_grad_norm=ah.max_grad_norm, lpg_lr=args.lpg_learning_rate,
        fix_value_critic=bool(getattr(args, "fix_value_critic", False)))


def create_lpg_train_state(rng: torch.Tensor, args) -> LpgTrainState:
    """meta/meta.py:10-30: flax's init of the LPG from ``rng`` (lpg.flax_init_lpg_params) and a fresh Adam state;
    with --use_es the OpenES strategy is attached by make_lpg_train_step's first call."""
    from .lpg import flax_init_lpg_params
    eta = flax_init_lpg_params(rng, 7 if args.lifetime_conditioning else 5)
    return LpgTrainState(eta, None if args.use_es else AdamState(eta.numel(), eta.device))


def eval_prep_after_forwards() -> bool:
    """With eval_keys_early: eval_agent's key chain starts right after the last LPG forward (default), beside that
    update's agent kernels, the eval rollout and the reverse loop, so that it ends before the recurrent backward
    starts (a CU still holding a chain wave when the backward's exactly-filled rounds begin finishes its last
    round that much later).  TOUED_EVAL_PREP=reverse: at the reverse loop, as in round 4 (bit-identical)."""
    return os.environ.get("TOUED_EVAL_PREP", "forwards") != "reverse"


def eval_keys_early() -> bool:
    """The meta-step's eval_agent reset, key chain and draws beside the reverse agent loop (default; C2 20.07-20.09 ms
    against 20.36-20.44 with them after the backward, where the weight-gradient reduction waited ~0.8 ms for them:
    profiles/r04/c2_eval_keys_early_r04f.txt).  TOUED_EVAL_KEYS_EARLY=0: after the backward."""
    return os.environ.get("TOUED_EVAL_KEYS_EARLY", "1") == "1"


def make_lpg_train_step(args, level_sampler, n_agents: int | None = None, world=None, rank_slice=None, impl=None):
    """meta/meta.py:33-52.  Returns ``train_step(rng, lpg_train_state, agent_states, value_critic_states=None)`` ->
    ``(lpg_train_state, agent_states, value_critic_states, metrics)``.

    agent_states: agents.AgentBatch of this rank's agents (``rank_slice`` = (lo, hi, n_total) under data
    parallelism; n_agents defaults to its size).  The meta-gradient step binds ``agent_states.theta`` / ``.phi`` to
    slots of its parameter-history ring (copying the tables once at the first call) and rebinds them to theta_K's
    slot at the end of every call (no copy back), so the returned states are the inputs with updated attributes; a
    tensor reference taken to the tables before a call is not updated by it.  value_critic_states: ValueCriticStates or None (then the ones
    inside agent_states are used); ignored by the ES step, as in the reference.  ``impl``: an already built
    MetaGradStep / ESTrainStep to drive (train.Trainer keeps its instance for timers and buffers)."""
    n_local = n_agents if n_agents is not None else (args.num_agents if rank_slice is None
                                                     else rank_slice[1] - rank_slice[0])
    holder = {} if impl is None else {"step": impl}
    if args.use_es:

        def es_step(rng, lpg_train_state, agent_states, value_critic_states=None):
            from .es import ESTrainStep
            if "step" not in holder:
                holder["step"] = ESTrainStep(args, level_sampler, n_local, lpg_train_state.params,
                                             lpg_train_state.params.device, world)
            lpg_train_state.es = holder["step"].es
            metrics = holder["step"](rng, agent_states, rank_slice)
            return lpg_train_state, agent_states, value_critic_states, metrics
        return es_step

    hyp = lpg_hypers_from_args(args, level_sampler)

    def meta_grad_step(rng, lpg_train_state, agent_states, value_critic_states=None):
        if "step" not in holder:
            holder["step"] = MetaGradStep(level_sampler.rollout_manager, n_local, hyp, args.lifetime_conditioning,
                                          lpg_train_state.params.device, world,
                                          num_mini_batches=args.num_mini_batches, num_agents_global=args.num_agents)
        if value_critic_states is not None:
            agent_states.vcrit, agent_states.vstep = value_critic_states.params, value_critic_states.step
        metrics = holder["step"](rng, lpg_train_state.params, lpg_train_state.opt, agent_states, rank_slice)
        return (lpg_train_state, agent_states, ValueCriticStates(agent_states.vcrit, agent_states.vstep), metrics)

    meta_grad_step.step = holder   # the MetaGradStep instance (timers, buffers) once built
    return meta_grad_step
