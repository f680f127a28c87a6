"""Meta-return curve (BASELINE.md "Reported per config"; train.py:32-56, meta/train.py:101-117): the training
driver's C2 loop (env_mode=tabular, score_function=random, W=64, T=20, K=5) for seeds 0-2 x 10 meta-steps,
certified step by step against the oracle.

Every meta-step of the GPU run is replayed by the oracle from the GPU's state before it:
  * the K train rollouts and the eval rollout bit-exact (oracle keys from the driver's rng chain, oracle
    env state carried across the rollouts, the GPU's theta_k);
  * the meta-gradient within 1e-5 relative L2 of the float64 autograd oracle on those trajectories, with the
    LPG's relu decisions (h_out > 0, models/lpg.py:81) taken from the device: every decision that differs from
    float64 must sit within 1e-6 of the kink (|h_out| < 1e-6, float32 rounding of a sum of O(1) terms), where
    the derivative jumps and no float32 implementation -- the reference's included -- is determined; the
    count of such kinks and the error without the override are recorded;
  * Adam (optax) on it bit-exact; the agents' tables after the K updates within 2e-5;
  * lpg_agent_return (eval_agent over 4 workers of the eval length): the oracle's eval rollouts from the
    GPU's theta_K, within 1e-6 per agent; lpg_loss within 2e-5;
  * level_sampler.sample (random): new levels / agents / env states bit-exact.
Starting point: flax init of eta from lpg_rng and the initial levels/agents, bit-exact / within 1e-6.
With TOUED_CURVE_OUT=<path> the per-step curve (GPU and oracle values) is written there as JSON.

The tabular lifetime (2500) is never reached in 10 x K=5 updates, so the plain curve's sample() only re-checks
"nothing changed".  The extra case (seed 0, life0=7) overrides agent 0's level lifetime to 7 on both sides (device
level word, oracle level): its updates past step 7 are discarded (lpg_agent.py:77-80), it terminates, and sample()
regenerates its level, agent and env state inside the curve (the override re-applied to each new level of agent 0).

Small agent count (N=4) so that the float64 oracle replays a step in seconds; the per-step
checks are size-independent.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import agents as oag
from oracle import flaxinit
from oracle import jaxrand as jr
from oracle import levels as olv
from oracle import meta as ometa
from oracle import rollout as oro
from oracle import sampler as osp

pytestmark = pytest.mark.gpu

N, S, MODE = 4, 10, "tabular"
_CURVES = {}


def _tr(traj, k, a):
    return {"idx": traj.obs_idx[k, a].T.copy(), "time": traj.obs_time[k, a].T.copy(),
            "action": traj.action[k, a].T.astype(np.int64), "reward": traj.reward[k, a].T.copy(),
            "done": traj.done[k, a].T.astype(bool)}


@pytest.mark.parametrize("seed,life0", [(0, None), (1, None), (2, None), (0, 7)])
def test_meta_return_curve_certified(seed, life0):
    from test_gpu_env import _state_np
    from toued import prng
    from toued.parse_args import parse_args
    from toued.train import Trainer
    args = parse_args(["--env_mode", MODE, "--num_agents", str(N), "--num_mini_batches", "1", "--seed", str(seed),
                       "--score_function", "random"])
    tr = Trainer(args)
    tr.step_fn.gru.keep_inputs = True     # the relu decisions of every step's backward (gru.relu_out)
    spec = olv.env_spec(MODE)
    W, T, K, Y = args.env_workers, args.train_rollout_len, args.num_agent_updates, 8
    L = tr.sampler.max_rollout_len
    hyp = ometa.Hypers()
    # ---- start: train.py:17-27
    rng = jr.PRNGKey(seed)
    rng, lpg_rng, _ = jr.split(rng, 3)
    eta_ref = flaxinit.lpg_init(lpg_rng, 5)
    np.testing.assert_allclose(tr.eta.cpu().numpy(), eta_ref, atol=1e-6, rtol=0)
    rng, sub = jr.split(rng, 2)
    lv, th, ph, st, vc = osp.initial_sample(spec, MODE, "random", sub, None, N, W, Y, True)
    assert np.array_equal(tr.agents.levels.cpu().numpy(), olv.pack_levels(lv[0], lv[1], spec, lv[2]))
    assert np.array_equal(tr.agents.theta.cpu().numpy(), th) and np.array_equal(tr.agents.vcrit.cpu().numpy(),
                                                                                   vc.reshape(N, -1))
    assert np.array_equal(prng.to_uint32_numpy(tr.rng), rng)
    from toued.env import L_LIFETIME

    def override_life0():
        tr.agents.levels[0, L_LIFETIME] = life0
        lv[1][0] = life0
    if life0:
        override_life0()
    resampled = 0
    curve = []
    for s in range(S):
        ag = tr.agents
        pre = {"eta": tr.eta.cpu().numpy(), "m": tr.adam.m.cpu().numpy(), "v": tr.adam.v.cpu().numpy(),
               "count": tr.adam.count, "theta": ag.theta.cpu().numpy(), "phi": ag.phi.cpu().numpy(),
               "vcrit": ag.vcrit.cpu().numpy(), "step": ag.step.cpu().numpy(), "state": _state_np(ag.state, spec)}
        # _meta_train_loop (train.py:36-54), the two halves observed separately
        ks = prng.split(tr.rng, 2)
        tr.rng, sub_d = ks[0].contiguous(), ks[1].contiguous()
        metrics = tr.step_fn(sub_d, tr.eta, tr.adam, tr.agents, tr.sl)
        torch.cuda.synchronize()
        sf = tr.step_fn
        traj = type("Tr", (), {k: getattr(sf.traj, k).cpu().numpy() for k in
                               ("obs_idx", "obs_time", "action", "reward", "done")})
        th_h = sf.theta_h.cpu().numpy()
        th_h[0] = pre["theta"]    # slot 0 is the agents' own table storage: after the step it holds theta_K
        R = N * W
        hpos = (sf.gru.relu_out() > 0).cpu().numpy().reshape(256, K, T, R)
        g_sum = sf.grad.cpu().numpy()
        ret_gpu = metrics["lpg_agent_return"].cpu().numpy()
        loss_gpu = metrics["lpg_loss"].cpu().numpy()
        post = {"theta": tr.agents.theta.cpu().numpy(), "phi": tr.agents.phi.cpu().numpy(),
                "vcrit": tr.agents.vcrit.cpu().numpy(), "step": tr.agents.step.cpu().numpy(),
                "state": _state_np(tr.agents.state, spec)}
        # ---- oracle key chain (meta/train.py:41,47,109,121; lpg_agent.py:107)
        rng, sub = jr.split(rng, 2)
        assert np.array_equal(prng.to_uint32_numpy(sub_d), sub)
        ka = jr.split(sub, N)
        r0t = jr.split(ka, 2)
        r0, tk = r0t[:, 0], r0t[:, 1]
        ost = pre["state"]
        for k in range(K + 1):
            if k < K:
                s2 = jr.split(tk, 2)
                tk, rk = s2[:, 0], s2[:, 1]
            else:
                s2 = jr.split(r0, 2)
                r0, rk = s2[:, 0], s2[:, 1]
            otr, ost, _ = oro.batch_rollout(spec, rk, th_h[k], lv[0], ost, T)
            for name, got in (("idx", traj.obs_idx), ("action", traj.action), ("reward", traj.reward),
                              ("done", traj.done)):
                np.testing.assert_array_equal(got[k], otr[name].transpose(0, 2, 1).astype(got.dtype),
                                              err_msg=f"seed {seed} step {s} rollout {k} {name}")
        for kname in ("time", "pos", "obj_existss", "early_term", "obj_poss"):
            np.testing.assert_array_equal(post["state"][kname], ost[kname])
        ea = jr.split(r0, 2)[:, 1]
        # ---- meta-gradient (float64 autograd on the same trajectories) and Adam
        ags = [dict(theta=pre["theta"][a], phi=pre["phi"][a], vcrit=pre["vcrit"][a][:, None],
                    step=int(pre["step"][a]), lifetime=int(lv[1][a]), trajs=[_tr(traj, k, a) for k in range(K)],
                    eval=_tr(traj, K, a), h_record=[],
                    relu_masks=[hpos[:, k, :, a * W:(a + 1) * W].transpose(2, 1, 0) for k in range(K)])
               for a in range(N)]
        g_ref, aux, _ = ometa.meta_gradient(pre["eta"].astype(np.float64), ags, hyp, K)
        kinks = 0
        for a in range(N):
            for k in range(K):
                h = ags[a]["h_record"][k].numpy()
                flip = ags[a]["relu_masks"][k] != (h > 0)
                assert np.all(np.abs(h[flip]) < 1e-6), (seed, s, a, k, np.abs(h[flip]).max())
                kinks += int(flip.sum())
        err = np.linalg.norm(g_sum / N - g_ref) / np.linalg.norm(g_ref)
        assert err < 1e-5, (seed, s, err, kinks)
        err_nomask = err
        if kinks:
            for ag_ in ags:
                ag_.pop("relu_masks")
                ag_["h_record"] = None
            g_free, _, _ = ometa.meta_gradient(pre["eta"].astype(np.float64), ags, hyp, K)
            err_nomask = np.linalg.norm(g_sum / N - g_free) / np.linalg.norm(g_free)
        eta_a, m_a, v_a, c_a = ometa.adam_f32(pre["eta"], g_sum, N, pre["m"], pre["v"], pre["count"])
        assert np.array_equal(tr.eta.cpu().numpy(), eta_a) and np.array_equal(tr.adam.m.cpu().numpy(), m_a)
        for a in range(N):
            np.testing.assert_allclose(post["theta"][a], aux[a]["theta"], rtol=2e-5, atol=2e-5)
            np.testing.assert_allclose(post["phi"][a], aux[a]["phi"], rtol=2e-5, atol=2e-5)
            assert int(post["step"][a]) == int(aux[a]["step"])
        loss_ref = np.array([x["lpg_loss"] for x in aux])
        np.testing.assert_allclose(loss_gpu, loss_ref, rtol=2e-5, atol=1e-7)
        # ---- lpg_agent_return: eval_agent (agents/agents.py:98-106) from the GPU's theta_K
        ret_ref = oag.eval_agent(spec, ea, lv[0], post["theta"], 4, L)
        np.testing.assert_allclose(ret_gpu, ret_ref, atol=1e-6, rtol=0)
        # ... and from the oracle's own float64-updated tables rounded to f32 (equal unless an action draw
        # falls within rounding of a cumsum boundary)
        ret_own = oag.eval_agent(spec, ea, lv[0], np.stack([aux[a]["theta"] for a in range(N)]).astype(np.float32),
                                 4, L)
        # ---- level_sampler.sample (random): train.py:46-48
        ks = prng.split(tr.rng, 2)
        tr.rng, sub_s = ks[0].contiguous(), ks[1].contiguous()
        tr.buffer, tr.agents = tr.sampler.sample(sub_s, tr.buffer, tr.agents, tr.sl)
        torch.cuda.synchronize()
        rng, sub = jr.split(rng, 2)
        term = post["step"] >= lv[1]
        lv, th, ph, st, vc, stp = osp.sample_nonplr(spec, MODE, "random", sub, None, term,
                                                    (lv, post["theta"], post["phi"], post["state"],
                                                     post["vcrit"].reshape(N, -1, 1), post["step"]), W, Y)
        assert np.array_equal(tr.agents.levels.cpu().numpy(), olv.pack_levels(lv[0], lv[1], spec, lv[2]))
        assert np.array_equal(tr.agents.theta.cpu().numpy(), th)
        assert np.array_equal(tr.agents.vcrit.cpu().numpy(), vc.reshape(N, -1))
        assert np.array_equal(tr.agents.step.cpu().numpy(), stp)
        post2 = _state_np(tr.agents.state, spec)
        for kname in ("time", "pos", "obj_existss", "early_term", "obj_poss"):
            np.testing.assert_array_equal(post2[kname], st[kname], err_msg=kname)
        if life0 and term[0]:
            resampled += 1
            override_life0()
        curve.append({"meta_step": s, "lpg_agent_return": float(ret_gpu.mean()),
                      "lpg_agent_return_oracle": float(ret_ref.mean()),
                      "lpg_agent_return_oracle_own_tables": float(ret_own.mean()),
                      "lpg_loss": float(loss_gpu.mean()), "lpg_loss_oracle": float(loss_ref.mean()),
                      "meta_grad_rel_l2": float(err), "relu_kinks_taken_from_device": kinks,
                      "meta_grad_rel_l2_float64_relu": float(err_nomask), "terminated": int(term.sum())})
        print(json.dumps({"seed": seed, **curve[-1]}), flush=True)
    if life0:
        assert resampled >= 2      # lifetime 7 at 5 updates per meta-step: terminated every second step
    _CURVES[seed if life0 is None else f"{seed}_life0_{life0}"] = curve
    out = os.environ.get("TOUED_CURVE_OUT")
    if out:
        with open(out, "w") as f:
            json.dump({"config": f"C2 loop env_mode={MODE} num_agents={N} W={W} T={T} K={K} score_function=random",
                       "tolerances": {"meta_grad_rel_l2": 1e-5, "relu_kink_band": 1e-6, "lpg_agent_return_abs": 1e-6, "lpg_loss_rel": 2e-5,
                                      "rollouts": "bit-exact", "adam": "bit-exact", "sample": "bit-exact"},
                       "curves": _CURVES}, f, indent=1)
