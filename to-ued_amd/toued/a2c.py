"""A2C antagonist on MI355X (agents/a2c.py:12-125).

``A2CTrainer.train`` runs ``train_a2c_agent`` for a batch of antagonists: a chain of
``num_train_steps`` updates, each = one fused rollout (toued_rollout) + one fused
gradient kernel (toued_a2c_grad: GAE, advantage normalisation, actor/critic/entropy
gradients) + one clipped-SGD apply (toued_a2c_apply).  The per-update keys of the
scan carry (``rng, _rng = split(rng)``, a2c.py:97) are produced up front by
toued_key_chain.  All buffers are allocated once per batch shape and the update loop
is replayed from a captured HIP graph (torch.cuda.CUDAGraph on ROCm), so the
hundreds of small launches per regret evaluation cost one graph launch.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch

from . import _lib
from .debug import debug_sync
from .agents import AgentHyperparams
from .env import LEVEL_WORDS
from .rollout import RolloutWrapper, Transition, split_rollouts


# updates whose rollout draws are produced by one toued_rollout_draws call (32 x N x W x T x 16 B of scratch)
DRAW_CHUNK = 32
# chunk sizes of the chain path: the first chunk's draws are the only ones not made beside a chain launch.  Round 3
# started the chunks short and grew them ~1.5x (4, 6, 9, 14, 21, then DRAW_CHUNK) so the first chain launch started
# early; since the round-4 chain speed-ups the short launches cost more than the wait they save (regret round 17.55 /
# 17.69 ms without the ramp against 17.76 / 18.39 with it on the same boxes, profiles/r04/c3_ramp_r04p.txt), so the
# default is no ramp (TOUED_A2C_RAMP: "1" this tuple, "0" none, or a comma list)
DRAW_RAMP = ()


def chunk_sizes(U: int) -> list[int]:
    """Update counts of the successive toued_a2c_chain launches of a U-update chain."""
    out, done = [], 0
    env = os.environ.get("TOUED_A2C_RAMP", "1")
    # "1": DRAW_RAMP; "0": none; a comma list: that ramp (timing studies)
    ramp = DRAW_RAMP if env == "1" else () if env == "0" else tuple(int(x) for x in env.split(",") if x)
    for m in ramp:
        if done >= U:
            break
        out.append(min(m, U - done))
        done += out[-1]
    full, r = divmod(U - done, DRAW_CHUNK)
    if r:   # a partial chunk goes with the short ones: the last launches stay full (they cover the eval draws)
        out.append(r)
    return sorted(out) + [DRAW_CHUNK] * full


@dataclass
class A2CHyperparams:
    """agents/a2c.py:12-16 (level_sampler.py:86-88 builds it from --gamma/--gae_lambda/--entropy_coeff)."""
    gamma: float = 0.99
    gae_lambda: float = 0.95
    entropy_coeff: float = 0.01


class A2CTrainer:
    def __init__(self, ro: RolloutWrapper, hyp: A2CHyperparams, agent_hypers: AgentHyperparams,
                 use_graph: bool = True, fused: bool | None = None, chain: bool | None = None):
        agent_hypers.check_supported()
        self.ro = ro
        self.hyp = hyp
        self.ah = agent_hypers
        self.use_graph = use_graph
        self._graphs = {}
        self.eval_draws_out = None
        self.fused = fused          # None: the LDS-fused update whenever it fits (toued_a2c_update_fits)
        # None: the whole update chain in one kernel per DRAW_CHUNK updates (toued_a2c_chain) whenever it fits and
        # the rollouts are split (unless TOUED_A2C_CHAIN=0); False: one rollout + one update launch per update
        self.chain = chain
        self._bufs = None
        self._graph = None
        self._graph_key = None
        self._side = None           # side stream of the chain path's draws
        # test hook: a list here makes train() run eagerly and append, after every update, the actor/critic
        # tables it started from, the rollout it ran and the tables it produced (tests/test_gpu_plr.py)
        self.record = None
        # optional toued.meta.KernelTimers: while enabled, train() runs eagerly and times each rollout ("a2c_rollout")
        # and update ("a2c_update") launch with HIP events on the launching stream (bench.py's C3 roofline)
        self.timers = None

    def _alloc(self, n, D, W, T, U, dev):
        key = (n, D, W, T, U, str(dev))
        if self._bufs is not None and self._bufs["key"] == key:
            return self._bufs
        z = lambda *s, dt=torch.float32: torch.zeros(s, dtype=dt, device=dev)
        self._bufs = {
            "key": key,
            "tr": Transition(z(n, T + 1, W, dt=torch.int32), z(n, T + 1, W, dt=torch.int32),
                             z(n, T, W, dt=torch.uint8), z(n, T, W), z(n, T, W, dt=torch.uint8)),
            "Ga": z(n, D, 5), "Gv": z(n, D), "loss": z(n, 2),
            "chain": z(U, n, 2, dt=torch.int32),
            # rollout draws of DRAW_CHUNK updates (split_rollouts): two (key-chain scratch, draws [T][chunk * n * W][4])
            # buffers, the chain kernel reading one while the side stream fills the other
            "dbuf": [tuple(z(T, min(U, DRAW_CHUNK) * n * W, 4, dt=torch.int32) for _ in range(2)) for _ in range(2)],
            # graph-static inputs
            "rng": z(n, 2, dt=torch.int32), "theta": z(n, D, 5), "vcrit": z(n, D),
            "step": z(n, dt=torch.int32), "levels": z(n, LEVEL_WORDS, dt=torch.int32),
            "state": z(12, n * W, dt=torch.int32),
        }
        self._graph = None
        self._graphs = {}
        return self._bufs

    def _eval_bufs(self, b, keys, levels, W):
        """Graph-static buffers of the eval draws enqueued behind the update chain (train(..., eval_keys=...))."""
        n2, T = keys.shape[0], self.ro.eval_rollout_len
        dev = keys.device
        if b.get("ev_shape") != (n2, W, T):
            b["ev_shape"] = (n2, W, T)
            b["ev_keys"] = torch.zeros((n2, 2), dtype=torch.int32, device=dev)
            b["ev_levels"] = torch.zeros((n2, LEVEL_WORDS), dtype=torch.int32, device=dev)
            b["ev_draws"] = torch.zeros((T, n2 * W, 4), dtype=torch.int32, device=dev)
            self._graphs.pop(True, None)
        b["ev_keys"].copy_(keys)
        b["ev_levels"].copy_(levels)
        return lambda: self.ro.eval_draws(b["ev_keys"], b["ev_levels"], W, buf=b["ev_draws"])

    def use_chain(self, W, T, D) -> bool:
        if self.chain is False or os.environ.get("TOUED_A2C_CHAIN") == "0" or not split_rollouts():
            return False
        if self.fused is False:
            return False
        return bool(_lib.lib().toued_a2c_chain_fits(W, T, D))

    def use_self_draws(self, W: int, T: int, D: int) -> bool:
        """The chain makes its own draws (toued_a2c_chain_self: the env chain's idle waves make the next update's) when
        its env workers fit one wave and its steps the draw flags (toued_a2c_chain_self_fits: W <= 64, T <= 64;
        TOUED_A2C_SELF=0: the draws pass beside chunked launches instead; regret round 14.7-15.1 vs 16.6-16.7 ms,
        profiles/r04/c3_self_prio_r04zd.txt)."""
        return (os.environ.get("TOUED_A2C_SELF", "1") != "0"
                and bool(_lib.lib().toued_a2c_chain_self_fits(W, T, D)))

    def _self_updates(self, b, n, D, W, T, U, tm, ev=None):
        """All U updates in one toued_a2c_chain_self launch.  The eval draws `ev` (threefry, full chip) go first: beside
        the chain's workgroups, which fill every register file, a kernel runs only where it held CUs when the launch
        began (profiles/r04/c3_draws_overlap_r04st.txt)."""
        L = _lib
        if ev is not None:
            ev()
        if b.get("sscr") is None:   # the per-agent draw double buffer [n][2][T][W] uint32x4
            b["sscr"] = torch.empty((n, 2, T, W, 4), dtype=torch.int32, device=b["theta"].device)
        tok = tm.start("a2c_chain") if tm is not None else None
        L.call("toued_a2c_chain_self", self.ro._c, L.ptr(b["levels"]), n, W, T, D, U, L.ptr(b["theta"]),
               L.ptr(b["vcrit"]), L.ptr(b["state"]), L.ptr(b["chain"]), L.ptr(b["sscr"]), self.hyp.gamma,
               self.hyp.gae_lambda, self.hyp.entropy_coeff, self.ah.actor_learning_rate, self.ah.critic_learning_rate,
               self.ah.max_grad_norm, L.ptr(b["step"]), L.ptr(b["loss"]), L.stream_ptr())
        if tm is not None:
            tm.stop(tok)

    def _chain_updates(self, b, n, D, W, T, U, tm, ev=None):
        """All U updates as toued_a2c_chain launches of DRAW_CHUNK updates each, every chunk on its precomputed draws.
        Untimed, the next chunk's draws (threefry VALU work, no LDS, ~24 VGPRs) run on a side stream beside the
        current chunk's chain kernel (latency-bound, two workgroups per CU), into the other of two draw buffers.
        `ev` (the eval rollout's draws, state-independent) is enqueued on the side stream behind the last chunk's
        draws, beside the last two chain launches; without the overlap it runs after the chain."""
        L = _lib
        st = L.stream_ptr()
        lr_a, lr_c, mn = self.ah.actor_learning_rate, self.ah.critic_learning_rate, self.ah.max_grad_norm
        sizes = chunk_sizes(U)
        starts = [sum(sizes[:c]) for c in range(len(sizes))]
        overlap = tm is None and len(starts) > 1
        main = torch.cuda.current_stream()
        if overlap:
            if self._side is None:
                self._side = torch.cuda.Stream(device=b["theta"].device)
            side = self._side
            fork = torch.cuda.Event()
            fork.record(main)
            side.wait_event(fork)

        def draws_for(c, stream_ptr):
            u, m = starts[c], sizes[c]
            full = b["dbuf"][c % 2] if overlap else b["dbuf"][0]
            # the chunk's (key-chain scratch, draws) as contiguous [T][m * n * W][4] views of the DRAW_CHUNK buffers
            bufs = tuple(x.view(-1)[:T * m * n * W * 4].view(T, m * n * W, 4) for x in full)
            return self.ro.train_draws(b["chain"][u:u + m], b["levels"], W, bufs,
                                       stream=stream_ptr)

        d_ev, c_ev, pending = [], [], None
        # the eval draws go on the side stream behind the draws of chunk len - ev_ahead + 1 (2: beside the last two
        # chain launches)
        ev_ahead = max(2, min(len(starts), int(os.environ.get("TOUED_A2C_EV_AHEAD", "2"))))
        if overlap:
            with torch.cuda.stream(side):
                pending = draws_for(0, side.cuda_stream)
            e = torch.cuda.Event()
            e.record(side)
            d_ev.append(e)
        for c, u in enumerate(starts):
            m = sizes[c]
            if overlap:
                draws = pending
                if c + 1 < len(starts):
                    if c >= 1:
                        side.wait_event(c_ev[c - 1])      # buffer (c + 1) % 2 was chunk c - 1's
                    with torch.cuda.stream(side):
                        pending = draws_for(c + 1, side.cuda_stream)
                    e = torch.cuda.Event()
                    e.record(side)
                    d_ev.append(e)
                    if ev is not None and c + ev_ahead == len(starts):
                        with torch.cuda.stream(side):
                            ev()
                        ev_done = torch.cuda.Event()
                        ev_done.record(side)
                main.wait_event(d_ev[c])
            else:
                tok = tm.start("a2c_draws") if tm is not None else None
                draws = draws_for(c, None)
                if tm is not None:
                    tm.stop(tok)
            tok = tm.start("a2c_chain") if tm is not None else None
            L.call("toued_a2c_chain", self.ro._c, L.ptr(b["levels"]), n, W, T, D, m, L.ptr(b["theta"]),
                   L.ptr(b["vcrit"]), L.ptr(b["state"]), L.ptr(draws), draws.shape[1], self.hyp.gamma,
                   self.hyp.gae_lambda, self.hyp.entropy_coeff, lr_a, lr_c, mn, L.ptr(b["step"]), L.ptr(b["loss"]), st)
            if tm is not None:
                tm.stop(tok)
            if overlap:
                e = torch.cuda.Event()
                e.record(main)
                c_ev.append(e)
        if ev is not None:
            if overlap:
                main.wait_event(ev_done)
            else:
                ev()

    def _updates(self, b, n, D, W, T, U, record=None, ev=None):
        L = _lib
        st = L.stream_ptr()
        b["loss"].zero_()
        if U == 0:
            if ev is not None:
                ev()
            return
        L.call("toued_key_chain", L.ptr(b["rng"]), n, U, L.ptr(b["chain"]), st)
        tm = self.timers if self.timers is not None and self.timers.enabled else None
        if record is None and self.use_chain(W, T, D):
            if self.use_self_draws(W, T, D):
                self._self_updates(b, n, D, W, T, U, tm, ev)
            else:
                self._chain_updates(b, n, D, W, T, U, tm, ev)
            return
        if ev is not None:   # the eval draws first: the per-update path below returns from inside its loop
            ev()
        tr = b["tr"]
        lr_a, lr_c, mn = self.ah.actor_learning_rate, self.ah.critic_learning_rate, self.ah.max_grad_norm
        fits = bool(L.lib().toued_a2c_update_fits(W, T, D))
        fused = fits if self.fused is None else (self.fused and fits)
        split = split_rollouts()
        draws, d0 = None, 0
        for u in range(U):
            if record is not None:
                before = (b["theta"].clone(), b["vcrit"].clone(), b["step"].clone())
            if split and (draws is None or u - d0 >= DRAW_CHUNK):
                # every state-independent draw of the next DRAW_CHUNK updates' rollouts at once (their keys are the
                # update key chain): U x N x W independent key chains instead of one dependent chain per update
                d0 = u
                tok = tm.start("a2c_draws") if tm is not None else None
                ch = min(U, DRAW_CHUNK)
                keys = b["chain"][u:u + ch]
                if keys.shape[0] < ch:      # the last chunk: its unused key rows are never rolled
                    keys = torch.cat([keys, b["chain"][:ch - keys.shape[0]]])
                draws = self.ro.train_draws(keys, b["levels"], W, b["dbuf"][0])
                if tm is not None:
                    tm.stop(tok)
            tok = tm.start("a2c_rollout") if tm is not None else None
            if split:
                self.ro.rollout_from_draws(draws, u - d0, b["theta"], b["levels"], b["state"], tr)
            else:
                L.call("toued_rollout", self.ro._c, L.ptr(b["levels"]), L.ptr(b["theta"]), D, L.ptr(b["chain"][u]),
                       L.ptr(b["state"]), n, W, T, L.ptr(tr.obs_idx), L.ptr(tr.obs_time), L.ptr(tr.action),
                       L.ptr(tr.reward), L.ptr(tr.done), None, st)
            if tm is not None:
                tm.stop(tok)
                tok = tm.start("a2c_update")
            if fused:   # gradient tables in LDS, grad + clip + SGD in one kernel
                L.call("toued_a2c_update", n, W, T, D, L.ptr(b["theta"]), L.ptr(b["vcrit"]), L.ptr(tr.obs_idx),
                       L.ptr(tr.obs_time), L.ptr(tr.action), L.ptr(tr.reward), L.ptr(tr.done), self.hyp.gamma,
                       self.hyp.gae_lambda, self.hyp.entropy_coeff, lr_a, lr_c, mn, L.ptr(b["step"]),
                       L.ptr(b["levels"]), L.ptr(b["loss"]), st)
            else:
                L.call("toued_a2c_grad", n, W, T, D, L.ptr(b["theta"]), L.ptr(b["vcrit"]), L.ptr(tr.obs_idx),
                       L.ptr(tr.obs_time), L.ptr(tr.action), L.ptr(tr.reward), L.ptr(tr.done), self.hyp.gamma,
                       self.hyp.gae_lambda, self.hyp.entropy_coeff, L.ptr(b["Ga"]), L.ptr(b["Gv"]), L.ptr(b["loss"]),
                       st)
                L.call("toued_a2c_apply", n, D, L.ptr(b["theta"]), L.ptr(b["vcrit"]), L.ptr(b["Ga"]), L.ptr(b["Gv"]),
                       lr_a, lr_c, mn, L.ptr(b["step"]), L.ptr(b["levels"]), st)
            if tm is not None:
                tm.stop(tok)
            if record is not None:
                record.append({"theta": before[0], "vcrit": before[1], "step": before[2],
                               "traj": Transition(tr.obs_idx.clone(), tr.obs_time.clone(), tr.action.clone(), tr.reward.clone(),
                                                  tr.done.clone()), "theta_out": b["theta"].clone(),
                               "vcrit_out": b["vcrit"].clone(), "step_out": b["step"].clone()})

    def train(self, rng: torch.Tensor, theta: torch.Tensor, vcrit: torch.Tensor, step: torch.Tensor,
              levels: torch.Tensor, state: torch.Tensor, num_train_steps: int, eval_keys: torch.Tensor | None = None,
              eval_levels: torch.Tensor | None = None):
        """train_a2c_agent (a2c.py:79-125) for n agents; updates theta [n,D,5], vcrit [n,D], step [n],
        state [12, n*W] in place.  Returns mean (actor_loss, critic_loss) over the updates, [n, 2].
        With eval_keys [m,2] / eval_levels [m,80] (the rollout keys and levels of a later eval_returns over W
        workers), that rollout's state-independent draws (RolloutWrapper.eval_draws) are produced beside the update
        chain; they are in `self.eval_draws_out` afterwards, for RolloutWrapper.eval_returns_from_draws."""
        n, D = theta.shape[0], theta.shape[1]
        if n == 0:
            return torch.zeros((0, 2), device=theta.device)
        W = state.shape[1] // n
        T = self.ro.train_rollout_len
        U = int(num_train_steps)
        b = self._alloc(n, D, W, T, U, theta.device)
        for name, src in (("rng", rng), ("theta", theta), ("vcrit", vcrit.reshape(n, D)), ("step", step),
                          ("levels", levels), ("state", state)):
            b[name].copy_(src)
        ev = self._eval_bufs(b, eval_keys, eval_levels, W) if eval_keys is not None else None
        self.eval_draws_out = b["ev_draws"] if ev is not None else None
        # the device error word (a draw wave's expired wait in toued_a2c_chain_self): allocated here, outside any
        # capture, on the first call; reports what an earlier round's read-back saw without blocking
        _lib.check_device_errors(wait=False)
        self._graph = self._graphs.get(ev is not None)
        if self.record is not None or (self.timers is not None and self.timers.enabled):
            self._updates(b, n, D, W, T, U, self.record, ev)
        elif self.use_graph and U > 0:
            if self._graph is None:
                # warm the path once outside capture (library load, kernel code objects)
                s = torch.cuda.Stream(device=theta.device)
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=s):
                        self._updates(b, n, D, W, T, U, ev=ev)
                torch.cuda.current_stream().wait_stream(s)
                self._graph = g
                self._graphs[ev is not None] = g
                # the capture did not execute: restore inputs and run it
                for name, src in (("rng", rng), ("theta", theta), ("vcrit", vcrit.reshape(n, D)), ("step", step),
                                  ("levels", levels), ("state", state)):
                    b[name].copy_(src)
            self._graph.replay()
        else:
            self._updates(b, n, D, W, T, U, ev=ev)
        # read the error word back behind this round (raised at the next round's check, or here under --debug)
        _lib.check_device_errors(wait=debug_sync())
        theta.copy_(b["theta"])
        vcrit.copy_(b["vcrit"].reshape(vcrit.shape))
        step.copy_(b["step"])
        state.copy_(b["state"])
        return b["loss"] / max(U, 1)
