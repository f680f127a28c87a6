"""TA-LPG: the LPG optimised with OpenES on MI355X (meta/train.py:133-227, meta/meta.py:10-52).

``ESTrainStep(rng, agents, rank_slice)`` = ``lpg_es_train_step``:
  1. ``rng, _rng = split(rng)``; OpenES ask (toued_es_ask): P = 2 * num_agents candidates,
     reordered into antithetic pairs (2i: mean + sigma z_i, 2i+1: mean - sigma z_i).
  2. ``rng, _rng = split(rng)``; ``split(_rng, P)`` per-candidate keys; every agent is repeated
     for its two candidates; per candidate ``rng_c, _rng_c = split(key_c)``: ``train_lpg_agent``
     for ``max_lifetime`` updates with that candidate's LPG (per-candidate GRU weights on MFMA,
     toued_gru_fwd_multi), then ``eval_agent(rng_c)`` over ``env_workers`` workers = fitness.
  3. rank per antithetic pair, keep the winning agent of each pair, OpenES tell
     (toued_es_grad + all-reduce + toued_es_opt).

OpenES is evosax 0.1.4 (not vendored) restated from its published algorithm:
the search mean starts at zero (``initialize`` draws uniform(init_min=0, init_max=0)); the
fitness shaper negates the rank fitness (maximize=True); Adam uses evosax's defaults
(b1=0.99, b2=0.999, eps=1e-8); lrate and sigma decay exponentially to their limits after
every tell.  Multi-GPU: rank r owns agents [lo, hi) -> candidates [2lo, 2hi) and z rows [lo, hi);
the tell gradient is one all-reduce of a [num_params] vector per ES step.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import _lib, prng
from .debug import nan_checker
from .agents import eval_agent, eval_agent_reset
from .lpg import LPGLayout
from .meta import lpg_inputs_fn
from .rollout import Transition, split_rollouts

_Y = 8
DRAW_CHUNK = 32        # candidate-update rollouts whose draws are made in one launch
EVAL_DRAWS_MAX_BYTES = 4 << 30   # the fitness eval's draws (+ key-chain scratch) are made ahead when they fit


class OpenES:
    """evosax.OpenES(popsize, maximize=True, opt_name, lrate_*, sigma_*, mean_decay) state on the device."""

    def __init__(self, popsize: int, num_dims: int, opt_name="adam", lrate_init=0.05, lrate_decay=1.0,
                 lrate_limit=0.001, sigma_init=0.03, sigma_decay=1.0, sigma_limit=0.01, mean_decay=0.0, device=None):
        opt_name = opt_name.lower()
        if opt_name not in ("adam", "sgd"):
            raise NotImplementedError(f"OpenES optimiser {opt_name}: adam and sgd are implemented")
        if mean_decay != 0.0:
            raise NotImplementedError("es_mean_decay != 0 is not implemented (reference default 0.0)")
        self.popsize = popsize
        self.nd = num_dims
        self.lrate_init, self.sigma_init = np.float32(lrate_init), np.float32(sigma_init)
        # evosax Strategy.tell's best-member tracker (get_best_fitness_member on the fitness given to tell), kept on
        # the device (best_member / best_fitness read it back)
        dev0 = torch.device(device) if device is not None else torch.device("cuda")
        self._best_member_t = None
        self._best_improved = None
        self._best_fit_t = torch.tensor(np.finfo(np.float32).max, dtype=torch.float32, device=dev0)
        self.opt = 1 if opt_name == "adam" else 0
        self.lrate_decay, self.lrate_limit = np.float32(lrate_decay), np.float32(lrate_limit)
        self.sigma_decay, self.sigma_limit = np.float32(sigma_decay), np.float32(sigma_limit)
        dev = torch.device(device) if device is not None else torch.device("cuda")
        self.mean = torch.zeros(num_dims, dtype=torch.float32, device=dev)
        self.m = torch.zeros_like(self.mean)
        self.v = torch.zeros_like(self.mean)
        self.grad = torch.zeros_like(self.mean)
        self.n = 0
        self.lrate = np.float32(lrate_init)
        self.sigma = np.float32(sigma_init)
        self.gen_counter = 0

    def ask(self, rng: torch.Tensor, row_lo: int, n_rows: int, out: torch.Tensor):
        """Candidates 2*row_lo .. 2*(row_lo+n_rows) of the reordered population into out [2n, nd]."""
        _lib.call("toued_es_ask", _lib.ptr(rng.contiguous()), self.nd, self.popsize // 2, row_lo, n_rows,
                  _lib.ptr(self.mean), float(self.sigma), _lib.ptr(out), _lib.stream_ptr())
        return out

    def track_best(self, x_local: torch.Tensor, rank_fitness: torch.Tensor, lo: int, world=None):
        """evosax 0.1.4 get_best_fitness_member (maximize=True) on the full rank-fitness vector, before the
        generation counter advances: the first candidate with the largest fitness replaces the best member when
        it beats the stored best (compared in the minimisation frame; restated, unpinned).  On the device, without
        a host synchronisation: argmax's first maximum, the candidate's row masked in on the rank that holds it
        (summed over ranks), and the replacement as selects."""
        fmin = -rank_fitness.float()
        idx = torch.argmin(fmin)                       # first minimum = first maximum of the fitness
        val = fmin[idx]
        best = self._best_fit_t
        best_min = -best if self.gen_counter > 0 else best
        better = val < best_min
        n = x_local.shape[0]
        rel = (idx - lo).clamp(0, n - 1)
        mine = (idx >= lo) & (idx < lo + n)
        row = torch.where(mine, x_local[rel].float(), torch.zeros((), device=x_local.device))
        if world is not None:
            world.all_reduce_sum(row)
        prev = self._best_member_t if self._best_member_t is not None else torch.zeros_like(row)
        self._best_member_t = torch.where(better, row, prev)
        self._best_improved = better if self._best_improved is None else (self._best_improved | better)
        self._best_fit_t = -torch.where(better, val, best_min)

    @property
    def best_member(self):
        """the tracked best member (None until a generation has been scored), as evosax's EvoState.best_member"""
        if self._best_member_t is None or not bool(self._best_improved):
            return None
        return self._best_member_t

    @property
    def best_fitness(self):
        return np.float32(self._best_fit_t.item())

    def tell(self, x_local: torch.Tensor, rank_fitness_local: torch.Tensor, world=None):
        fit = (-rank_fitness_local).float().contiguous()          # FitnessShaper(maximize=True)
        _lib.call("toued_es_grad", _lib.ptr(x_local), _lib.ptr(self.mean), float(self.sigma), _lib.ptr(fit),
                  x_local.shape[0], self.nd, _lib.ptr(self.grad), _lib.stream_ptr())
        if world is not None:
            world.all_reduce_sum(self.grad)
        scale = np.float32(1.0) / (np.float32(self.popsize) * self.sigma)
        b1, b2, eps = np.float32(0.99), np.float32(0.999), np.float32(1e-8)
        bc1 = np.float32(1.0) - b1 ** np.float32(self.n + 1)
        bc2 = np.float32(1.0) - b2 ** np.float32(self.n + 1)
        _lib.call("toued_es_opt", self.nd, self.opt, _lib.ptr(self.mean), _lib.ptr(self.grad), float(scale),
                  _lib.ptr(self.m), _lib.ptr(self.v), float(self.lrate), float(b1), float(b2), float(eps), float(bc1),
                  float(bc2), _lib.stream_ptr())
        self.n += 1
        self.lrate = np.maximum(np.float32(self.lrate * self.lrate_decay), self.lrate_limit)
        self.sigma = np.maximum(np.float32(self.sigma * self.sigma_decay), self.sigma_limit)
        self.gen_counter += 1


class ESTrainStep:
    def __init__(self, args, sampler, n_local: int, eta: torch.Tensor, device=None, world=None,
                 num_agent_updates: int | None = None):
        self.sampler = sampler
        self.ro = sampler.rollout_manager
        self.world = world
        self.dev = torch.device(device) if device is not None else eta.device
        self.N = n_local
        self.C = 2 * n_local
        self.W = self.ro.env_workers
        self.T = self.ro.train_rollout_len
        self.D = self.ro.obs_dim
        # make_lpg_train_step (meta/meta.py:35-37): ES trains each agent for its whole lifetime
        self.K = sampler.max_lifetime if num_agent_updates is None else num_agent_updates
        self.F = 7 if args.lifetime_conditioning else 5
        self.lay = LPGLayout(self.F)
        if eta.numel() != self.lay.size:
            raise ValueError("eta does not match the LPG layout")
        ah = sampler.agent_hypers
        self.lr_a, self.lr_c, self.mn = ah.actor_learning_rate, ah.critic_learning_rate, ah.max_grad_norm
        self.alpha_y = args.lpg_agent_target_coeff
        n_total = args.num_agents
        self.es = OpenES(2 * n_total, self.lay.size, args.lpg_opt, args.lpg_learning_rate, args.es_lrate_decay,
                         args.es_lrate_limit, args.es_sigma_init, args.es_sigma_decay, args.es_sigma_limit,
                         args.es_mean_decay, self.dev)
        C, W, T, D = self.C, self.W, self.T, self.D
        R = C * W
        if W % 32:
            raise ValueError(f"env_workers={W} must be a multiple of 32 for the MFMA GRU row blocks")
        self.R = R
        f32, i32, u8 = torch.float32, torch.int32, torch.uint8
        z = lambda *s, dt=f32: torch.zeros(s, dtype=dt, device=self.dev)
        self.x = z(C, self.lay.size)
        self.fwdA = z(C, _lib.lib().toued_gru_packed_floats(2))
        self.theta = [z(C, D, 5), z(C, D, 5)]
        self.phi = [z(C, D, _Y), z(C, D, _Y)]
        self.G_th, self.G_ph = z(C, D, 5), z(C, D, _Y)
        self.gstat = z(C, 4)
        self.met = z(C, 8)
        self.tr = Transition(z(C, T + 1, W, dt=i32), z(C, T + 1, W, dt=i32), z(C, T, W, dt=u8), z(C, T, W),
                             z(C, T, W, dt=u8))
        self.X = z(self.F, T, R)
        self.pi_hat = z(T, R)
        self.y_hat = z(T, _Y, R)
        self.fitness = None
        # test hook: a list receives, per agent update k, the candidates' (theta_k, phi_k, env state before the
        # rollout, trajectory k) as device clones (tests/test_gpu_es.py regenerates every rollout from them)
        self.trace = None
        self._side = None       # side stream of the draws made ahead
        self._bufs = {}
        # the fused in-place agent update (toued_agent_update) when one candidate's samples fit the sorted kernel;
        # TOUED_ES_FUSED_UPDATE=0 keeps toued_agent_grad + toued_agent_apply (bit-identical)
        self.fused_update = (os.environ.get("TOUED_ES_FUSED_UPDATE") != "0"
                             and bool(_lib.lib().toued_agent_update_fits(self.W, self.T, self.D)))
        # HIP-event timing of the per-update launches (bench.py's C4 roofline); disabled by default
        from .meta import KernelTimers
        self.timers = KernelTimers()

    def _eta(self, name):
        o = self.lay.offsets[name]
        return self.x.view(-1)[o:]

    def _chunk_bufs(self, C, W):
        """Two (key-chain scratch, draws) buffer pairs of DRAW_CHUNK updates' train rollouts, [T][32 * C * W][4]."""
        key = ("chunk", C, W)
        if key not in self._bufs:
            z = lambda: torch.empty((self.T, DRAW_CHUNK * C * W, 4), dtype=torch.int32, device=self.dev)
            self._bufs[key] = [(z(), z()) for _ in range(2)]
        return self._bufs[key]

    def _eval_draw_bytes(self, C, W):
        return 2 * 16 * self.ro.eval_rollout_len * C * W

    def _fit_draws_buf(self, C, W):
        key = ("fit", C, W)
        if key not in self._bufs:
            self._bufs[key] = torch.empty((self.ro.eval_rollout_len, C * W, 4), dtype=torch.int32, device=self.dev)
        return self._bufs[key]

    def __call__(self, rng: torch.Tensor, agents, rank_slice=None):
        L = _lib
        st = L.stream_ptr()
        ptr = L.ptr
        N, C, W, T, D, K, R = self.N, self.C, self.W, self.T, self.D, self.K, self.R
        lo = 0 if rank_slice is None else rank_slice[0]
        n_total = N if rank_slice is None else rank_slice[2]
        nd = self.lay.size
        # ---- ask (meta/train.py:147-158)
        ks = prng.split(rng, 2)
        rng, sub = ks[0].contiguous(), ks[1].contiguous()
        self.es.ask(sub, lo, N, self.x)
        L.call("toued_gru_pack_fwd_multi", ptr(self.x), nd, C, self.lay.c_offsets, self.F, ptr(self.fwdA), st)
        # ---- per-candidate keys (:187-189) and repeated agents (:184-186)
        ks = prng.split(rng, 2)
        rng, sub = ks[0].contiguous(), ks[1].contiguous()
        ck = prng.split(sub, 2 * n_total)[2 * lo:2 * lo + C]
        ck2 = prng.split(ck.contiguous(), 2)
        fit_keys, train_keys = ck2[:, 0].contiguous(), ck2[:, 1].contiguous()
        chain = torch.empty((K, C, 2), dtype=torch.int32, device=self.dev)
        if K:
            L.call("toued_key_chain", ptr(train_keys), C, K, ptr(chain), st)
        levels = agents.levels.repeat_interleave(2, dim=0).contiguous()
        step = agents.step.repeat_interleave(2).contiguous()
        state = agents.state.view(12, agents.n, W).repeat_interleave(2, dim=1).reshape(12, C * W).contiguous()
        cur = 0
        self.theta[cur].copy_(agents.theta.repeat_interleave(2, dim=0))
        self.phi[cur].copy_(agents.phi.repeat_interleave(2, dim=0))
        self.met.zero_()
        e1w, e1b, e2w, e2b = (self._eta(n) for n in ("e1_w", "e1_b", "e2_w", "e2_b"))
        tr = self.tr
        # ---- train_lpg_agent for K = max_lifetime updates (agents/lpg_agent.py:88-140)
        split = split_rollouts()
        draws = None
        # the state-independent draws of DRAW_CHUNK updates' rollouts in one launch, made one chunk ahead on a side
        # stream into the other of two buffers (beside the per-candidate forwards), and eval_agent's draws for the
        # fitness behind the last chunk's; each update's env chain then runs on its batch (bit-identical to the
        # per-update rollout)
        # (TOUED_ES_AHEAD=1; off by default: the side stream's draws slow the per-candidate forwards beside them by
        # as much as they save, 2.35 -> 2.39 ms per launch against 19.5 -> 12.2 ms of rollouts per ES step)
        ahead = split and K > 0 and os.environ.get("TOUED_ES_AHEAD", "0") == "1"
        fit_state = fit_rkeys = None
        if ahead:
            main = torch.cuda.current_stream()
            if self._side is None:
                self._side = torch.cuda.Stream(device=self.dev)
            side = self._side
            n_ch = -(-K // DRAW_CHUNK)
            fit_state, fit_rkeys = eval_agent_reset(self.ro, fit_keys, levels, W)
            fit_ev = self._fit_draws_buf(C, W) if self._eval_draw_bytes(C, W) <= EVAL_DRAWS_MAX_BYTES else None
            ready, used = [None] * n_ch, [None] * n_ch

            def draws_ahead(c):
                m = min(DRAW_CHUNK, K - c * DRAW_CHUNK)
                bufs = tuple(x.view(-1)[:T * m * C * W * 4].view(T, m * C * W, 4) for x in self._chunk_bufs(C, W)[c % 2])
                with torch.cuda.stream(side):
                    out = self.ro.train_draws(chain[c * DRAW_CHUNK:c * DRAW_CHUNK + m], levels, W, bufs,
                                              stream=side.cuda_stream)
                    if c + 1 == n_ch and fit_ev is not None:
                        self.ro.eval_draws(fit_rkeys, levels, W, buf=fit_ev)
                ready[c] = torch.cuda.Event()
                ready[c].record(side)
                return out

            side.wait_stream(main)
            pending = draws_ahead(0)
        for k in range(K):
            th, ph = self.theta[cur], self.phi[cur]
            if self.trace is not None:
                rec = {"theta": th.clone(), "phi": ph.clone(), "state": state.clone(), "step": step.clone()}
            tok = self.timers.start("rollout")
            if ahead:
                c = k // DRAW_CHUNK
                if k % DRAW_CHUNK == 0:
                    main.wait_event(ready[c])
                    draws = pending
                    if c + 1 < n_ch:
                        if c >= 1:
                            side.wait_event(used[c - 1])   # buffer (c + 1) % 2 was chunk c - 1's
                        pending = draws_ahead(c + 1)
                self.ro.rollout_from_draws(draws, k % DRAW_CHUNK, th, levels, state, tr)
                if k % DRAW_CHUNK == DRAW_CHUNK - 1 or k == K - 1:
                    used[c] = torch.cuda.Event()
                    used[c].record(main)
            elif split:
                if k % DRAW_CHUNK == 0:
                    # this step's own buffers (a short last chunk views a prefix of them): the rollout wrapper's shared
                    # buffer would be reallocated at every change of shape and is also used by other callers
                    m = min(DRAW_CHUNK, K - k)
                    bufs = tuple(x.view(-1)[:T * m * C * W * 4].view(T, m * C * W, 4) for x in self._chunk_bufs(C, W)[0])
                    draws = self.ro.train_draws(chain[k:k + m], levels, W, bufs)
                self.ro.rollout_from_draws(draws, k % DRAW_CHUNK, th, levels, state, tr)
            else:
                self.ro.batch_rollout(chain[k], th, levels, state, out=tr, inplace_state=True)
            self.timers.stop(tok)
            if self.trace is not None:
                rec["traj"] = Transition(tr.obs_idx.clone(), tr.obs_time.clone(), tr.action.clone(), tr.reward.clone(),
                                         tr.done.clone())
                self.trace.append(rec)
            L.call(lpg_inputs_fn(C * W, W), C, W, T, D, self.F, ptr(th), ptr(ph), ptr(tr.obs_idx), ptr(tr.obs_time),
                   ptr(tr.action), ptr(tr.reward), ptr(tr.done), ptr(e1w), ptr(e1b), ptr(e2w), ptr(e2b), ptr(step),
                   ptr(levels), ptr(self.X), T * R, 1, nd, st)
            tok = self.timers.start("gru_fwd_multi")
            L.call("toued_gru_fwd_multi", R, T, W, self.F, W, ptr(self.X), T * R, 1, ptr(tr.done), ptr(self.fwdA),
                   ptr(self.x), nd, self.lay.c_offsets, ptr(self.pi_hat), ptr(self.y_hat), st)
            self.timers.stop(tok)
            if self.fused_update:
                # gradient + clip + SGD in one kernel, in place on the candidates' tables (bit-identical to the pair
                # below: the gradient tables are never read again on this path)
                L.call("toued_agent_update", C, W, T, D, ptr(th), ptr(ph), ptr(tr.obs_idx), ptr(tr.obs_time),
                       ptr(tr.action), ptr(tr.reward), ptr(tr.done), ptr(self.pi_hat), ptr(self.y_hat), self.alpha_y,
                       self.lr_a, self.lr_c, self.mn, ptr(self.met), ptr(step), ptr(levels), ptr(self.gstat), st)
            else:
                self.G_th.zero_()
                self.G_ph.zero_()
                L.call("toued_agent_grad", C, W, T, D, ptr(th), ptr(ph), ptr(tr.obs_idx), ptr(tr.obs_time),
                       ptr(tr.action), ptr(tr.reward), ptr(tr.done), ptr(self.pi_hat), ptr(self.y_hat), self.alpha_y,
                       ptr(self.G_th), ptr(self.G_ph), ptr(self.met), ptr(step), ptr(levels), ptr(self.gstat), st)
                L.call("toued_agent_apply", C, D, ptr(th), ptr(ph), ptr(self.G_th), ptr(self.G_ph), self.lr_a,
                       self.lr_c, self.mn, ptr(step), ptr(self.theta[1 - cur]), ptr(self.phi[1 - cur]),
                       ptr(self.gstat), st)
                cur = 1 - cur
            L.call("toued_entropy", C, W, T, D, ptr(self.theta[cur]), ptr(self.phi[cur]), ptr(tr.obs_idx),
                   ptr(tr.obs_time), ptr(self.met), 0.0, 0.0, None, None, st)
        self.cur = cur                  # index of the candidates' final tables in self.theta / self.phi
        # ---- fitness = eval_agent(rng_c) (:178-186)
        if ahead and fit_ev is not None:
            fitness = self.ro.eval_returns_from_draws(fit_ev, self.theta[cur], levels, fit_state).mean(dim=1)
        elif ahead:
            fitness = self.ro.eval_returns(fit_rkeys, self.theta[cur], levels, fit_state).mean(dim=1)
        else:
            fitness = eval_agent(self.ro, fit_keys, levels, self.theta[cur], W)
        self.fitness = fitness
        nan_checker().check("es_fitness", fitness)
        # ---- rank per antithetic pair, winners (:199-211)
        first_greater = fitness[0::2] > fitness[1::2]
        rank = torch.empty_like(fitness)
        rank[0::2] = first_greater.float()
        rank[1::2] = 1.0 - first_greater.float()
        sel = torch.where(first_greater, torch.arange(N, device=self.dev) * 2, torch.arange(N, device=self.dev) * 2 + 1)
        agents.theta.copy_(self.theta[cur][sel])
        agents.phi.copy_(self.phi[cur][sel])
        agents.step.copy_(step[sel])
        agents.state.copy_(state.view(12, C, W)[:, sel].reshape(12, N * W))
        # ---- tell (:214-217); evosax tracks the best member on the fitness passed to tell (the rank fitness)
        multi = self.world is not None and self.world.size > 1
        rank_all = self.world.all_gather_cat(rank) if multi else rank
        self.es.track_best(self.x, rank_all, 2 * lo, self.world if multi else None)
        self.es.tell(self.x, rank, self.world if multi else None)
        nan_checker().check("es_mean_after_tell", self.es.mean)
        inv = 1.0 / (W * T * max(K, 1))
        m = self.met * inv
        fit_all = fitness if self.world is None or self.world.size == 1 else self.world.all_gather_cat(fitness)
        return {
            "fitness": {"mean": fit_all.mean(), "min": fit_all.min(), "max": fit_all.max(),
                        "var": fit_all.var(unbiased=False)},
            "lpg_agent": {"critic_loss": m[:, 0], "policy_l2": m[:, 1], "critic_l2": m[:, 2],
                          "policy_entropy": m[:, 3], "critic_entropy": m[:, 4]},
        }
