"""torch-CPU float64 restatement of the LPG inner loop and meta-gradient — test oracle.

Follows:
  agents/lpg_agent.py:31-85   lpg_agent_train_step (LPG-driven actor/critic update,
                              clip-by-global-norm SGD (models/optim.py:6-11), discard
                              when step > lifetime)
  agents/lpg_agent.py:88-140  train_lpg_agent (K updates; entropy metrics, util/metrics.py:5-9)
  agents/agents.py:109-116    compute_advantage + util/metrics.py:17-38 gae
  meta/train.py:36-170        _train_agent: eval rollout, frozen value critic,
                              normalised advantage, lpg_loss with the [T]x[T,1] broadcast
                              (value critic returns [T+1,1] -> adv [T,1]),
                              regularisers, jax.grad w.r.t. the LPG params (here torch
                              autograd with create_graph through the K clipped-SGD steps)
  meta/train.py:172-182       mean of per-agent gradients, Adam (optax scale_by_adam).

The rollouts (trajectories) are *inputs*: the environment is not differentiable
(actions are integer draws) and the HIP rollout is bit-exact against
oracle/rollout.py, so the meta-gradient is checked on identical trajectories.
Observations are compact (idx, time); obs @ W == W[idx] + (0.001*t) * W[D-1].
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import lpg as olpg

EPS = 1e-8


@dataclass
class Hypers:
    actor_lr: float = 40.0
    critic_lr: float = 4.0
    max_grad_norm: float = 0.5
    agent_target_coeff: float = 0.5
    policy_entropy_coeff: float = 5e-2
    target_entropy_coeff: float = 1e-3
    policy_l2_coeff: float = 5e-3
    target_l2_coeff: float = 1e-3
    gamma: float = 0.99
    gae_lambda: float = 0.95
    lifetime_conditioning: bool = False
    stop_gradient: bool = True   # agents/lpg_agent.py:54-56; False only for finite-difference self-tests
    fix_value_critic: bool = False   # train the value critic (meta/train.py:61-81 without the discarded .replace)


def linear_logits(table, idx, time):
    """table [D,K] (one agent); idx/time int [..] -> logits [..,K] = W[idx] + (f32(t)*0.001) W[D-1]."""
    c = torch.from_numpy((time.astype(np.float32) * np.float32(0.001)).astype(np.float64)).to(table.dtype)
    return table[torch.from_numpy(idx.astype(np.int64))] + c[..., None] * table[-1]


def clip_sgd(params, grad, lr, max_norm):
    """optax chain(clip_by_global_norm, scale(lr), scale(-1)) + apply_updates."""
    gn = torch.sqrt(torch.sum(grad * grad))
    g = grad if bool(gn < max_norm) else (grad / gn) * max_norm
    return params - lr * g


def entropy(probs):
    """util/metrics.py:5-9 batch_rollout_entropy (mean over all leading dims)."""
    p = probs + EPS
    return -torch.mean(torch.sum(p * torch.log(p), dim=-1))


def lpg_agent_step(theta, phi, step, lifetime, eta, traj, hyp: Hypers, relu_mask=None, h_record=None):
    """agents/lpg_agent.py:31-85 for one agent.  traj: dict of numpy arrays [W,T(+1)].
    relu_mask / h_record: see oracle/lpg.lpg_apply.

    Returns (theta', phi', step', metrics dict, (pi_hat, y_hat))."""
    idx, tm = traj["idx"], traj["time"]
    a = torch.from_numpy(traj["action"].astype(np.int64))
    r = torch.from_numpy(traj["reward"].astype(np.float64)).to(theta.dtype)
    d = torch.from_numpy(traj["done"].astype(bool))
    probs = torch.softmax(linear_logits(theta, idx[:, :-1], tm[:, :-1]), -1)       # [W,T,5]
    probs_e = probs + EPS
    pi = torch.gather(probs_e, -1, a[..., None])[..., 0]                             # [W,T]
    y_t = torch.softmax(linear_logits(phi, idx[:, :-1], tm[:, :-1]), -1)             # [W,T,8]
    y_tp1 = torch.softmax(linear_logits(phi, idx[:, 1:], tm[:, 1:]), -1)
    W = idx.shape[0]
    sg = (lambda x: x.detach()) if hyp.stop_gradient else (lambda x: x)
    if hyp.lifetime_conditioning:
        st = torch.full((W,), float(step), dtype=theta.dtype)
        lt = torch.full((W,), float(lifetime), dtype=theta.dtype)
        pi_hat, y_hat = olpg.lpg_apply(eta, r, d, sg(pi), sg(y_t), sg(y_tp1), st, lt, relu_mask=relu_mask,
                                       h_record=h_record)
    else:
        pi_hat, y_hat = olpg.lpg_apply(eta, r, d, sg(pi), sg(y_t), sg(y_tp1), relu_mask=relu_mask,
                                       h_record=h_record)
    y_l2 = torch.mean(torch.sum(y_hat * y_hat, -1))
    kl = torch.sum(y_t * (torch.log(y_t + EPS) - torch.log(y_hat + EPS)), -1)        # [W,T]
    actor_loss = torch.log(pi) * pi_hat
    pi_l2 = torch.mean(pi_hat * pi_hat)
    g_theta = torch.autograd.grad(torch.mean(actor_loss), theta, create_graph=True)[0]
    g_phi = torch.autograd.grad(hyp.agent_target_coeff * torch.mean(kl), phi, create_graph=True)[0]
    new_theta = clip_sgd(theta, g_theta, hyp.actor_lr, hyp.max_grad_norm)
    new_phi = clip_sgd(phi, g_phi, hyp.critic_lr, hyp.max_grad_norm)
    if step + 1 <= lifetime:
        theta, phi, step = new_theta, new_phi, step + 1
    metrics = {"critic_loss": torch.mean(kl), "policy_l2": pi_l2, "critic_l2": y_l2}
    return theta, phi, step, metrics, (pi_hat, y_hat)


def gae(value, reward, done, gamma, lam):
    """util/metrics.py:17-38 per worker: value [T+1], reward/done [T] -> adv [T], target [T]."""
    T = reward.shape[-1]
    adv = []
    g = torch.zeros_like(value[..., 0])
    for t in reversed(range(T)):
        nd = 1.0 - done[..., t]
        delta = reward[..., t] + (gamma * value[..., t + 1] * nd - value[..., t])
        g = delta + gamma * lam * nd * g
        adv.append(g)
    adv = torch.stack(adv[::-1], -1)
    return adv, adv + value[..., :-1]


def train_agent_meta(eta, theta0, phi0, step0, lifetime, vcrit, trajs, eval_traj, hyp: Hypers, K: int,
                     relu_masks=None, h_record=None):
    """meta/train.py:36-100 (_train_agent) for one agent, given K train trajectories and the
    eval trajectory (all dicts of numpy [W, T(+1)]).  Returns (reg_lpg_loss, aux dict).
    relu_masks: optional per-update LPG relu decisions [W,T,H] (oracle/lpg.lpg_apply)."""
    theta, phi, step = theta0, phi0, step0
    mets = []
    for k in range(K):
        mk = None if relu_masks is None else torch.as_tensor(relu_masks[k])
        theta, phi, step, m, _ = lpg_agent_step(theta, phi, step, lifetime, eta, trajs[k], hyp, mk, h_record)
        tr = trajs[k]
        m["policy_entropy"] = entropy(torch.softmax(linear_logits(theta, tr["idx"][:, :-1], tr["time"][:, :-1]), -1))
        m["critic_entropy"] = entropy(torch.softmax(linear_logits(phi, tr["idx"][:, :-1], tr["time"][:, :-1]), -1))
        mets.append(m)
    agent = {k: torch.mean(torch.stack([m[k] for m in mets])) for k in mets[0]}
    # value critic (frozen: SURVEY B.3), advantage on the eval rollout (agents.py:109-116); with
    # fix_value_critic the scan of _update_critic over the K train rollouts runs first (meta/train.py:74-77)
    if hyp.fix_value_critic:
        vcrit = vcrit.detach()
        for k in range(K):
            vcrit, _ = value_critic_step(vcrit, trajs[k], hyp)
    ev = eval_traj
    v = linear_logits(vcrit, ev["idx"], ev["time"])[..., 0]                      # [W,T+1]
    r = torch.from_numpy(ev["reward"].astype(np.float64)).to(v.dtype)
    dn = torch.from_numpy(ev["done"].astype(np.float64)).to(v.dtype)
    adv, target = gae(v, r, dn, hyp.gamma, hyp.gae_lambda)
    value_loss = torch.mean(torch.mean((target - v[:, :-1]) ** 2, -1))
    advn = (adv - adv.mean()) / (adv.std(unbiased=False) + EPS)
    probs = torch.softmax(linear_logits(theta, ev["idx"][:, :-1], ev["time"][:, :-1]), -1)
    a = torch.from_numpy(ev["action"].astype(np.int64))
    logp = torch.gather(torch.log(probs + EPS), -1, a[..., None])[..., 0]        # [W,T]
    # -multiply(logp [T], adv [T,1]) -> [T,T] per worker, mean over [W,T,T]
    lpg_loss = torch.mean(-(logp[:, None, :] * advn[:, :, None]))
    reg = (lpg_loss - hyp.policy_entropy_coeff * agent["policy_entropy"] + hyp.policy_l2_coeff * agent["policy_l2"]
           - hyp.target_entropy_coeff * agent["critic_entropy"] + hyp.target_l2_coeff * agent["critic_l2"])
    aux = {"lpg_loss": lpg_loss, "reg_lpg_loss": reg, "value_loss": value_loss, "lpg_agent": agent,
           "theta": theta, "phi": phi, "step": step}
    if hyp.fix_value_critic:        # meta/train.py:78-81: the eval-rollout update after its loss and advantages
        aux["vcrit"], _ = value_critic_step(vcrit, ev, hyp)
    return reg, aux


def value_critic_step(vcrit, traj, hyp: Hypers):
    """_update_critic (meta/train.py:61-72) as the reference means it: compute_advantage (agents/agents.py:109-116)
    per worker -- mean_t (target - V)^2 on stop-gradient GAE targets -- mean over workers, its gradient,
    clip_by_global_norm + SGD (critic lr, max_norm).  vcrit [D, 1].  Returns (vcrit', loss)."""
    vc = vcrit.detach().requires_grad_(True)
    v = linear_logits(vc, traj["idx"], traj["time"])[..., 0]
    r = torch.from_numpy(traj["reward"].astype(np.float64)).to(v.dtype)
    dn = torch.from_numpy(traj["done"].astype(np.float64)).to(v.dtype)
    adv, target = gae(v, r, dn, hyp.gamma, hyp.gae_lambda)
    loss = torch.mean(torch.mean((target.detach() - v[:, :-1]) ** 2, -1))
    g = torch.autograd.grad(loss, vc)[0]
    with torch.no_grad():
        return clip_sgd(vc, g, hyp.critic_lr, hyp.max_grad_norm).detach(), float(loss)


def meta_gradient(eta_np, agents, hyp: Hypers, K: int, dtype=torch.float64):
    """Per-agent jax.grad of _train_agent w.r.t. eta, then the mean over agents (meta/train.py:172-180).

    agents: list of dicts with theta [D,5], phi [D,8], vcrit [D,1], step, lifetime, trajs (K dicts), eval.
    Returns (mean grad np [P], list of per-agent aux)."""
    grads = []
    auxs = []
    for ag in agents:
        eta = torch.tensor(eta_np, dtype=dtype, requires_grad=True)
        theta = torch.tensor(ag["theta"], dtype=dtype, requires_grad=True)
        phi = torch.tensor(ag["phi"], dtype=dtype, requires_grad=True)
        vc = torch.tensor(ag["vcrit"], dtype=dtype)
        reg, aux = train_agent_meta(eta, theta, phi, ag["step"], ag["lifetime"], vc, ag["trajs"], ag["eval"], hyp, K,
                                    ag.get("relu_masks"), ag.get("h_record"))
        g = torch.autograd.grad(reg, eta)[0]
        grads.append(g.detach().numpy())
        auxs.append({k: (v.detach().numpy() if torch.is_tensor(v) else
                         ({kk: vv.detach().numpy() for kk, vv in v.items()} if isinstance(v, dict) else v))
                     for k, v in aux.items()})
    return np.mean(grads, axis=0), auxs, grads


_LIBM = None


def _powf(b, e) -> np.float32:
    global _LIBM
    if _LIBM is None:
        import ctypes
        import ctypes.util
        _LIBM = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
        _LIBM.powf.restype = ctypes.c_float
        _LIBM.powf.argtypes = [ctypes.c_float, ctypes.c_float]
    return np.float32(_LIBM.powf(float(b), float(e)))


def adam_f32(eta, grad_sum, n_mean, m, v, count, lr=1e-4, b1=0.9, b2=0.999, eps=1e-8):
    """optax 0.1.5 chain(scale_by_adam(), scale(lr), scale(-1.0)) (models/optim.py:12-17) on the agent-mean
    gradient (meta/train.py:128 ``x.mean(axis=0)`` = sum / N), in the float32 operation order jax traces:
      update_moment:           (1 - b1) * g + b1 * mu          (python-float constants, weak-typed -> f32 once)
      update_moment_per_elem_norm: (1 - b2) * g**2 + b2 * nu
      bias_correction:         t / (1 - b**count)              (count = the incremented int32 step)
      updates = mu_hat / (sqrt(nu_hat + eps_root=0) + eps); * lr; * -1; params + updates.
    ``b**count`` is libm powf (what XLA-CPU calls for an f32 pow; unpinned against XLA itself).
    Returns (eta', m', v', count') as float32 arrays."""
    F = np.float32
    g = (np.asarray(grad_sum, F) / F(n_mean)).astype(F)
    count = int(count) + 1
    m = (F(1.0 - b1) * g + F(b1) * np.asarray(m, F)).astype(F)
    v = (F(1.0 - b2) * (g * g) + F(b2) * np.asarray(v, F)).astype(F)
    # f32 pow: XLA-CPU lowers lax.pow on f32 to the llvm.pow intrinsic, i.e. a call to the C library's powf;
    # numpy's float32 power and a rounded double power both differ from glibc powf in the last bit at some counts
    bc1 = F(F(1.0) - _powf(F(b1), count))
    bc2 = F(F(1.0) - _powf(F(b2), count))
    upd = ((m / bc1) / (np.sqrt(v / bc2) + F(eps))).astype(F)
    eta = (np.asarray(eta, F) + (upd * F(lr)) * F(-1.0)).astype(F)
    return eta, m, v, count


def adam_update(eta, grad, m, v, count, lr=1e-4, b1=0.9, b2=0.999, eps=1e-8):
    """optax scale_by_adam + scale(lr) + scale(-1) (models/optim.py:12-17)."""
    m = b1 * m + (1 - b1) * grad
    v = b2 * v + (1 - b2) * grad * grad
    count = count + 1
    mh = m / (1 - b1 ** count)
    vh = v / (1 - b2 ** count)
    upd = mh / (np.sqrt(vh) + eps)
    return eta - lr * upd, m, v, count


def gae_f32(value, reward, done, discount, gae_lambda):
    """util/metrics.py:17-38 in numpy float32 with the reference's operation order, per element (bit-exact target of
    toued_gae): value [..., T+1], reward/done [..., T].  discount * gae_lambda is a python-float product (weak-typed
    constants: f32 of the double product); (1 - done) is exactly 0 or 1."""
    f = np.float32
    value = np.asarray(value, f)
    reward = np.asarray(reward, f)
    nd = (1 - np.asarray(done).astype(np.int32)).astype(f)
    g_d, gl = f(discount), f(float(discount) * float(gae_lambda))
    T = reward.shape[-1]
    adv = np.zeros(reward.shape, f)
    g = np.zeros(reward.shape[:-1], f)
    for t in reversed(range(T)):
        value_diff = (g_d * value[..., t + 1]).astype(f) * nd[..., t] - value[..., t]
        delta = reward[..., t] + value_diff
        g = (delta + (gl * nd[..., t]).astype(f) * g).astype(f)
        adv[..., t] = g
    return adv, (adv + value[..., :-1]).astype(f)
