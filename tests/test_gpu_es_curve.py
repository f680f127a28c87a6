"""ES meta-return curve (BASELINE.md "Reported per config": fitness.mean for ES; meta/train.py:218-226): the training
driver's TA-LPG loop (--use_es --lifetime_conditioning, env_mode=all_vrandlife, score_function=random) for seeds
0-2 x 5 ES steps, certified step by step against the oracle (tests/test_gpu_es.py certify_es_step):
  * ask bit-exact; every candidate's K rollouts bit-exact from the oracle's key chain; each float64 agent update
    under the candidate's LPG (from the device's tables before it) within 2e-5 relative L2, the agent metrics within 2e-5; fitness (eval_agent) within 1e-5; pair winners;
    rank -> OpenES tell: the population gradient within 1e-6 relative L2, the Adam step on it within f32 rounding;
  * level_sampler.sample (random): levels, agents and step counters bit-exact vs oracle/sampler.py.
Size: N = 2 agents (4 candidates) and K = 5 agent updates per candidate instead of the mode's max_lifetime (250:
meta/meta.py:35-37), so that the float64 oracle replays an ES step in seconds; every check is per candidate and
size-independent.  Agent 0's level lifetime is overridden to 7 on both sides (device level word and oracle level),
so its lifetime-conditioned updates past step 7 are discarded and sample() regenerates its level and agent inside
the curve (the override is re-applied to each regenerated level of agent 0).
With TOUED_ES_CURVE_OUT=<path> the per-step curve is written there as JSON.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import jaxrand as jr
from oracle import levels as olv
from oracle import sampler as osp

pytestmark = pytest.mark.gpu

N, S, K, MODE, LIFE0 = 2, 5, 5, "all_vrandlife", 7
_CURVES = {}


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_es_fitness_curve_certified(seed):
    from test_gpu_env import _state_np
    from test_gpu_es import certify_es_step, es_pre
    from toued import prng
    from toued.env import L_LIFETIME
    from toued.parse_args import parse_args
    from toued.train import Trainer
    args = parse_args(["--env_mode", MODE, "--num_agents", str(N), "--num_mini_batches", "1", "--seed", str(seed),
                       "--score_function", "random", "--use_es", "--lifetime_conditioning",
                       "--lpg_learning_rate", "0.01"])
    tr = Trainer(args)
    step = tr.step_fn
    step.K = K
    spec = olv.env_spec(MODE)
    W, Y = args.env_workers, 8
    rng = jr.PRNGKey(seed)
    rng, _, _ = jr.split(rng, 3)
    rng, sub = jr.split(rng, 2)
    lv, th, ph, st, _ = osp.initial_sample(spec, MODE, "random", sub, None, N, W, Y, False)
    assert np.array_equal(tr.agents.levels.cpu().numpy(), olv.pack_levels(lv[0], lv[1], spec, lv[2]))
    assert np.array_equal(tr.agents.theta.cpu().numpy(), th) and np.array_equal(tr.agents.phi.cpu().numpy(), ph)
    assert np.array_equal(prng.to_uint32_numpy(tr.rng), rng)
    assert float(step.es.mean.abs().max()) == 0.0          # evosax initialize: uniform(0, 0)

    def override_life0():
        tr.agents.levels[0, L_LIFETIME] = LIFE0
        lv[1][0] = LIFE0
    override_life0()
    curve = []
    resampled = 0
    for s in range(S):
        pre = es_pre(step, tr.agents)
        ks = prng.split(tr.rng, 2)
        tr.rng, sub_d = ks[0].contiguous(), ks[1].contiguous()
        step.trace = []
        m = step(sub_d, tr.agents, tr.sl)
        torch.cuda.synchronize()
        rng, sub = jr.split(rng, 2)
        assert np.array_equal(prng.to_uint32_numpy(sub_d), sub)
        f, f_ref, winners, steps_w, th_w, ph_w, ost = certify_es_step(args, tr.sampler, step, sub, pre, m, lv[0])
        post_state = _state_np(tr.agents.state, spec)
        rows = np.concatenate([np.arange(w * W, (w + 1) * W) for w in winners])
        for kname in ("time", "pos", "obj_existss", "early_term", "obj_poss"):
            np.testing.assert_array_equal(post_state[kname], ost[kname][rows], err_msg=kname)
        assert np.array_equal(tr.agents.theta.cpu().numpy(), th_w)
        assert np.array_equal(tr.agents.step.cpu().numpy(), steps_w)
        # ---- level_sampler.sample (random): train.py:46-48
        ks = prng.split(tr.rng, 2)
        tr.rng, sub_s = ks[0].contiguous(), ks[1].contiguous()
        tr.buffer, tr.agents = tr.sampler.sample(sub_s, tr.buffer, tr.agents, tr.sl)
        torch.cuda.synchronize()
        rng, sub = jr.split(rng, 2)
        term = steps_w >= lv[1]
        lv, th, ph, st, _, stp = osp.sample_nonplr(spec, MODE, "random", sub, None, term,
                                                   (lv, th_w, ph_w, post_state, None, steps_w), W, Y)
        assert np.array_equal(tr.agents.levels.cpu().numpy(), olv.pack_levels(lv[0], lv[1], spec, lv[2]))
        assert np.array_equal(tr.agents.theta.cpu().numpy(), th) and np.array_equal(tr.agents.phi.cpu().numpy(), ph)
        assert np.array_equal(tr.agents.step.cpu().numpy(), stp)
        post2 = _state_np(tr.agents.state, spec)
        for kname in ("time", "pos", "obj_existss", "early_term", "obj_poss"):
            np.testing.assert_array_equal(post2[kname], st[kname], err_msg=kname)
        if term[0]:
            resampled += 1
            override_life0()
        curve.append({"es_step": s, "fitness_mean": float(m["fitness"]["mean"]), "fitness_mean_oracle": float(f_ref.mean()),
                      "fitness_max": float(f.max()), "fitness_min": float(f.min()),
                      "es_sigma": float(step.es.sigma), "terminated": int(term.sum())})
        print(json.dumps({"seed": seed, **curve[-1]}), flush=True)
    assert resampled >= 1          # agent 0 (lifetime 7, 5 updates per ES step) terminates and is regenerated
    _CURVES[seed] = curve
    out = os.environ.get("TOUED_ES_CURVE_OUT")
    if out:
        with open(out, "w") as fh:
            json.dump({"config": f"C4 loop (reduced) env_mode={MODE} --use_es --lifetime_conditioning num_agents={N} "
                                 f"candidates={2 * N} W={W} K={K} agent updates per candidate (max_lifetime 250 in "
                                 f"the full config) score_function=random lpg_learning_rate=0.01; agent 0 lifetime {LIFE0}",
                       "tolerances": {"agent_update_rel_l2": 2e-5, "fitness_abs": 1e-5, "tell_grad_rel_l2": 1e-6, "adam_step_rel": 1e-6,
                                      "rollouts": "bit-exact", "ask": "bit-exact", "sample": "bit-exact"},
                       "curves": _CURVES}, fh, indent=1)
