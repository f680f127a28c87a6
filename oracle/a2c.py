"""torch-CPU restatement of the A2C antagonist update — test oracle.

agents/a2c.py:19-76 ``a2c_agent_train_step``:
  critic: per worker GAE on value = critic(obs ++ next_obs[T-1]) ([T+1, 1] — the value
          critic keeps its trailing dim), loss mean((target - V)^2) with stop-gradient on
          (adv, target); advantages normalised over the agent's [W, T, 1]
  actor:  per worker mean(-log(pi(a)+1e-8) [T] * adv [T,1])  -> the [T, T] broadcast
          (= -mean_t log pi * mean_t adv), minus entropy_coeff * entropy of (pi + 1e-8)
  both:   optax clip_by_global_norm -> SGD (models/optim.py:6-11); discard when the new
          step exceeds the lifetime (a2c.py:82-86).
"""
from __future__ import annotations

import numpy as np
import torch

from .meta import EPS, clip_sgd, gae, linear_logits


def a2c_step(theta, vcrit, step, lifetime, traj, hyp, actor_lr, critic_lr, max_norm, entropy_coeff=0.01):
    """One update for one agent.  theta [D,5], vcrit [D,1] torch tensors; traj numpy dict [W, T(+1)].
    Returns (theta', vcrit', step', actor_loss, critic_loss)."""
    theta = theta.detach().requires_grad_(True)
    vcrit = vcrit.detach().requires_grad_(True)
    idx, tm = traj["idx"], traj["time"]
    r = torch.from_numpy(traj["reward"].astype(np.float64)).to(theta.dtype)
    d = torch.from_numpy(traj["done"].astype(np.float64)).to(theta.dtype)
    a = torch.from_numpy(traj["action"].astype(np.int64))
    # critic (a2c.py:285-305)
    value = linear_logits(vcrit, idx, tm)                         # [W, T+1, 1]
    adv, target = gae(value[..., 0], r, d, hyp.gamma, hyp.gae_lambda)
    adv, target = adv.detach(), target.detach()
    losses = torch.mean((target - value[:, :-1, 0]) ** 2, dim=-1)  # [W]
    critic_loss = torch.mean(losses)
    g_c = torch.autograd.grad(critic_loss, vcrit)[0]
    advn = (adv - adv.mean()) / (adv.std(unbiased=False) + EPS)   # [W, T]
    # actor (a2c.py:308-324)
    probs = torch.softmax(linear_logits(theta, idx[:, :-1], tm[:, :-1]), -1) + EPS
    logp = torch.log(probs)
    sel = torch.gather(logp, -1, a[..., None])[..., 0]            # [W, T]
    pol = -(sel[:, None, :] * advn[:, :, None])                   # [W, T, T] broadcast
    ent = -torch.mean(torch.sum(probs * logp, -1), dim=-1)         # [W]
    actor_loss = torch.mean(torch.mean(pol, dim=(1, 2)) - entropy_coeff * ent)
    g_a = torch.autograd.grad(actor_loss, theta)[0]
    with torch.no_grad():
        new_theta = clip_sgd(theta, g_a, actor_lr, max_norm)
        new_v = clip_sgd(vcrit, g_c, critic_lr, max_norm)
    if step + 1 <= lifetime:
        return new_theta.detach(), new_v.detach(), step + 1, float(actor_loss.detach()), float(critic_loss.detach())
    return theta.detach(), vcrit.detach(), step, float(actor_loss.detach()), float(critic_loss.detach())
