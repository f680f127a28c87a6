"""The meta-gradient step's scheduling defaults against their env fallbacks, over several meta-steps with
level_sampler.sample in between (train.py:36-54):

  * TOUED_HIST_RING=0    -- the parameter history copied into fixed slots instead of the K + 1 slot ring that rebinds
                            agents.theta / phi to theta_K's slot after every step;
  * TOUED_PACK_SIDE=0    -- the GRU fragment packing on the main stream instead of the side stream;
  * TOUED_EVAL_PREP=reverse -- eval_agent's reset, key chain and draws at the reverse loop instead of after the last
                            LPG forward.

Each is a scheduling choice with the same arithmetic, so the meta-gradient, eta, Adam's moments, the agents' tables,
steps and env state, and every metric must be bit-identical to the defaults after every step.  Agent 0's level
lifetime is overridden to 7 (5 updates per meta-step), so sample() terminates it and rewrites its tables in the ring
slot the step bound them to (the interaction the ring's rebinding has to survive)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

N, STEPS = 4, 4
FALLBACKS = [("TOUED_HIST_RING", "0"), ("TOUED_PACK_SIDE", "0"), ("TOUED_EVAL_PREP", "reverse")]


def _flat_metrics(m, pre=""):
    out = {}
    for k, v in m.items():
        if isinstance(v, dict):
            out.update(_flat_metrics(v, pre + k + "."))
        else:
            out[pre + k] = v.detach().clone()
    return out


def _run(monkeypatch, env):
    from toued.env import L_LIFETIME
    from toued.parse_args import parse_args
    from toued.train import Trainer
    for name, _ in FALLBACKS:
        monkeypatch.delenv(name, raising=False)
    if env:
        monkeypatch.setenv(*env)
    args = parse_args(["--env_mode", "tabular", "--num_agents", str(N), "--num_mini_batches", "1", "--seed", "3",
                       "--score_function", "random"])
    tr = Trainer(args)
    tr.agents.levels[0, L_LIFETIME] = 7
    trace = []
    terminated = 0
    for _ in range(STEPS):
        m = tr.meta_step()
        torch.cuda.synchronize()
        terminated += int(tr.agents.step[0].item() == 0)
        tr.agents.levels[0, L_LIFETIME] = 7     # re-applied to a regenerated level
        ag = tr.agents
        trace.append({"grad": tr.step_fn.grad.clone(), "eta": tr.eta.clone(), "m": tr.adam.m.clone(),
                      "v": tr.adam.v.clone(), "theta": ag.theta.clone(), "phi": ag.phi.clone(),
                      "vcrit": ag.vcrit.clone(), "step": ag.step.clone(), "state": ag.state.clone(),
                      "levels": ag.levels.clone(), **_flat_metrics(m)})
    return trace, terminated


def test_meta_step_fallbacks_bit_identical(monkeypatch):
    base, term = _run(monkeypatch, None)
    assert term >= 1, "agent 0 never terminated: the sampler's rewrite of a ring slot was not exercised"
    for env in FALLBACKS:
        got, _ = _run(monkeypatch, env)
        for s, (a, b) in enumerate(zip(base, got)):
            for key in a:
                assert torch.equal(a[key], b[key]), f"{env[0]}={env[1]}: step {s} {key} differs"
