"""GPU parity: HIP env / level generator / rollout vs the numpy oracle — bit-exact.

All integer/bool outputs (levels, states, tabular indices, actions, dones) and
the rewards/returns (exact f32: at most one nonzero term per step) must match
exactly on the same seeded inputs.
"""
import numpy as np
import pytest
import torch

from oracle import gridworld as ogw
from oracle import jaxrand as jr
from oracle import levels as olv
from oracle import rollout as oro

pytestmark = pytest.mark.gpu

MODES = ["dense", "sparse", "long", "longer", "long_dense", "tabular", "all_shortlife", "all_vrandlife", "mazes",
         "small", "medium", "large", "debug", "rand_dense", "rand_small", "rand_all", "sixteen_rooms", "labyrinth"]


def dev_keys(keys_np):
    from toued.prng import from_uint32_numpy
    return from_uint32_numpy(keys_np, "cuda")


def oracle_levels(mode, keys):
    spec = olv.env_spec(mode)
    p, lt = olv.reset_env_params(keys, mode)
    return spec, p, lt, olv.pack_levels(p, lt, spec)


@pytest.mark.parametrize("mode", MODES)
def test_level_gen_bitexact(mode):
    from toued.env import LevelGenerator
    keys = jr.split(jr.PRNGKey(17), 257)
    spec, p, lt, packed = oracle_levels(mode, keys)
    gen = LevelGenerator(mode)
    lev, sub = gen(dev_keys(keys), with_sub_mode=True)
    got = lev.cpu().numpy()
    np.testing.assert_array_equal(got, packed)
    np.testing.assert_array_equal(sub.cpu().numpy(), p["sub_mode"])


def test_device_split_and_uniform():
    from toued import prng
    keys = jr.split(jr.PRNGKey(5), 33)
    dk = dev_keys(keys)
    np.testing.assert_array_equal(prng.to_uint32_numpy(prng.split(dk, 7)), jr.split(keys, 7))
    np.testing.assert_array_equal(prng.to_uint32_numpy(prng.split_planar(dk, 7)),
                                  np.ascontiguousarray(jr.split(keys, 7).transpose(1, 0, 2)))
    np.testing.assert_array_equal(prng.to_uint32_numpy(prng.fold_in(dk, 123)), jr.fold_in(keys, 123))
    np.testing.assert_array_equal(prng.to_uint32_numpy(prng.random_bits(dk, 9)), jr.random_bits(keys, (9,)))
    np.testing.assert_array_equal(prng.uniform(dk, 5, -1.0, 1.0).cpu().numpy(), jr.uniform(keys, (5,), -1.0, 1.0))


def _state_np(st, spec):
    n = st.shape[1]
    s = st.cpu().numpy()
    ex = np.stack([(s[2] >> i) & 1 for i in range(spec.max_n_objs)], 1).astype(bool)
    return {"time": s[0], "pos": s[1], "obj_existss": ex, "early_term": s[3].astype(bool),
            "obj_poss": s[4:4 + spec.max_n_objs].T.copy()}


def _assert_state(dev_state, ost, spec):
    g = _state_np(dev_state, spec)
    for k in ("time", "pos", "obj_existss", "early_term", "obj_poss"):
        np.testing.assert_array_equal(g[k], ost[k], err_msg=k)


@pytest.mark.parametrize("mode", ["dense", "tabular", "all_shortlife", "mazes", "rand_dense", "rand_small",
                                  "rand_sparse", "debug"])
def test_env_reset_step_bitexact(mode):
    from toued.env import GridWorld, get_env_spec
    B = 512
    keys = jr.split(jr.PRNGKey(3), B)
    spec, p, lt, packed = oracle_levels(mode, keys)
    dspec, _, _ = get_env_spec(mode)
    env = GridWorld(dspec)
    lev = torch.from_numpy(packed).cuda()
    rk = jr.split(jr.PRNGKey(4), B)
    (idx, tm), st = env.reset(dev_keys(rk), lev, 1)
    ost = ogw.env_reset(spec, rk, p)
    _assert_state(st, ost, spec)
    rs = np.random.RandomState(0)
    key = jr.PRNGKey(8)
    for t in range(200):
        key, sk = jr.split(key)
        sk = jr.split(sk, B)
        act = rs.randint(0, 5, B).astype(np.int32)
        (idx, tm), st, r, d = env.step(dev_keys(sk), st, torch.from_numpy(act).cuda(), lev, 1)
        ost, orew, odone = ogw.env_step(spec, sk, ost, act, p)
        _assert_state(st, ost, spec)
        np.testing.assert_array_equal(r.cpu().numpy(), orew)
        np.testing.assert_array_equal(d.cpu().numpy(), odone)
        if spec.tabular:
            oidx, otm = ogw.obs_compact(spec, ost)
            np.testing.assert_array_equal(idx.cpu().numpy(), oidx)


@pytest.mark.parametrize("mode,W,T", [("dense", 64, 20), ("tabular", 64, 20), ("all_shortlife", 64, 30),
                                      ("mazes", 64, 50), ("debug", 7, 13), ("sparse", 32, 25),
                                      ("all_shortlife", 8, 300), ("tabular", 8, 250)])
def test_rollout_bitexact(mode, W, T):
    from toued.rollout import RolloutWrapper
    N = 12
    keys = jr.split(jr.PRNGKey(21), N)
    spec, p, lt, packed = oracle_levels(mode, keys)
    rw = RolloutWrapper(mode, T, env_workers=W)
    lev = torch.from_numpy(packed).cuda()
    rk = jr.split(jr.PRNGKey(22), N)
    (idx0, tm0), st = rw.batch_reset(dev_keys(rk), lev)
    ost = oro.batch_reset(spec, rk, p, W)
    _assert_state(st, ost, spec)
    # a peaked random actor so trajectories are diverse but not uniform
    theta = (np.random.RandomState(1).randn(N, spec.obs_dim, 5) * 3).astype(np.float32)
    th = torch.from_numpy(theta).cuda()
    for k in range(3):
        ak = jr.split(jr.PRNGKey(100 + k), N)
        tr, st, cum = rw.batch_rollout(dev_keys(ak), th, lev, st)
        otr, ost, ocum = oro.batch_rollout(spec, ak, theta, p, ost, T)
        np.testing.assert_array_equal(tr.obs_idx.cpu().numpy(), otr["idx"].transpose(0, 2, 1))
        np.testing.assert_array_equal(tr.obs_time.cpu().numpy(), otr["time"].transpose(0, 2, 1))
        np.testing.assert_array_equal(tr.action.cpu().numpy(), otr["action"].transpose(0, 2, 1))
        np.testing.assert_array_equal(tr.reward.cpu().numpy(), otr["reward"].transpose(0, 2, 1))
        np.testing.assert_array_equal(tr.done.cpu().numpy().astype(bool), otr["done"].transpose(0, 2, 1))
        np.testing.assert_array_equal(cum.cpu().numpy(), ocum)
        _assert_state(st, ost, spec)


def test_rollout_large_properties():
    """Full-size C2 shape (512 agents x 64 workers x 20 steps): size-independent invariants."""
    from toued.env import LevelGenerator
    from toued.rollout import RolloutWrapper
    N, W, T = 512, 64, 20
    gen = LevelGenerator("tabular")
    keys = jr.split(jr.PRNGKey(0), N)
    lev = gen(dev_keys(keys))
    rw = RolloutWrapper("tabular", T, env_workers=W)
    (i0, t0), st = rw.batch_reset(dev_keys(jr.split(jr.PRNGKey(1), N)), lev)
    D = rw.obs_dim
    th = torch.zeros((N, D, 5), device="cuda")
    tr, st2, cum = rw.batch_rollout(dev_keys(jr.split(jr.PRNGKey(2), N)), th, lev, st)
    a = tr.action.cpu().numpy()
    assert a.max() <= 4
    # uniform policy: every action roughly 20% of the time
    frac = np.bincount(a.ravel(), minlength=5) / a.size
    assert np.all(np.abs(frac - 0.2) < 0.01)
    # next_obs_t == obs_{t+1}; time increments unless done
    tm = tr.obs_time.cpu().numpy().astype(np.int64)
    d = tr.done.cpu().numpy().astype(bool)
    assert np.all(np.where(d, tm[:, 1:] == 0, tm[:, 1:] == tm[:, :-1] + 1))
    idx = tr.obs_idx.cpu().numpy()
    assert idx.min() >= 0 and idx.max() < D - 1
    # a second run with the same keys is identical (determinism)
    tr2, _, cum2 = rw.batch_rollout(dev_keys(jr.split(jr.PRNGKey(2), N)), th, lev, st)
    assert torch.equal(tr.obs_idx, tr2.obs_idx) and torch.equal(cum, cum2)


@pytest.mark.parametrize("mode,N,W", [("tabular", 96, 4), ("dense", 40, 4), ("longer", 24, 4), ("all_shortlife", 64, 4),
                                      ("all_vrandlife", 64, 4), ("sparse", 33, 3), ("debug", 17, 5),
                                      ("all_shortlife", 6, 64), ("mazes", 5, 128)])   # W % 64 == 0: the table kernel
def test_eval_returns_three_launches(mode, N, W):
    """eval_agent's returns-only rollout as key chain + parallel draws + env chain (toued_eval_keys/_draws/_returns)
    is bit-identical to the single-kernel returns-only mode (itself checked against the oracle below and in
    tests/test_gpu_plr.py), on peaked and uniform actors over the full eval length."""
    from toued.rollout import RolloutWrapper
    keys = jr.split(jr.PRNGKey(31), N)
    spec, p, lt, packed = oracle_levels(mode, keys)
    rw = RolloutWrapper(mode, 20, env_workers=W)
    lev = torch.from_numpy(packed).cuda()
    (_, _), st = rw.batch_reset(dev_keys(jr.split(jr.PRNGKey(32), N)), lev)
    st0 = st.clone()
    for scale in (3.0, 0.0):
        theta = (np.random.RandomState(2).randn(N, spec.obs_dim, 5) * scale).astype(np.float32)
        th = torch.from_numpy(theta).cuda()
        ak = dev_keys(jr.split(jr.PRNGKey(33), N))
        ref = rw.eval_returns(ak, th, lev, st)
        draws = rw.eval_draws(ak, lev, W)
        got = rw.eval_returns_from_draws(draws, th, lev, st)
        np.testing.assert_array_equal(got.cpu().numpy(), ref.cpu().numpy())
        assert torch.equal(st, st0)
    if mode == "sparse":   # short episodes: the numpy oracle over the whole eval length is cheap here
        _, _, ocum = oro.batch_rollout(spec, jr.split(jr.PRNGKey(33), N), theta, p, _state_np(st0, spec),
                                       rw.eval_rollout_len)
        np.testing.assert_array_equal(got.cpu().numpy(), ocum)


@pytest.mark.parametrize("mode,N,W", [("dense", 3, 64), ("tabular", 2, 64), ("all_shortlife", 5, 32), ("mazes", 2, 64),
                                      ("debug", 3, 16)])
def test_train_rollout_three_launches(mode, N, W):
    """The train rollouts as draws (toued_rollout_draws, U batches at once: the A2C update chain's form) + env chain
    (toued_rollout_env) are bit-identical to the single-kernel toued_rollout: every batch's trajectory, end state and
    cum_return, batches rolled one after another from the carried state, on peaked and uniform actors; the
    production batch_rollout (split path) likewise."""
    from toued import _lib
    from toued.rollout import RolloutWrapper, Transition
    keys = jr.split(jr.PRNGKey(41), N)
    spec, p, lt, packed = oracle_levels(mode, keys)
    T = 20
    rw = RolloutWrapper(mode, T, env_workers=W)
    lev = torch.from_numpy(packed).cuda()
    (_, _), st0 = rw.batch_reset(dev_keys(jr.split(jr.PRNGKey(42), N)), lev)
    U = 3
    ukeys = dev_keys(jr.split(jr.PRNGKey(43), U * N)).view(U, N, 2).contiguous()
    for scale in (3.0, 0.0):
        th = torch.from_numpy((np.random.RandomState(4).randn(N, spec.obs_dim, 5) * scale).astype(np.float32)).cuda()
        draws = rw.train_draws(ukeys, lev, W)
        s_ref, s_got = st0.clone(), st0.clone()
        for u in range(U):
            def buf():
                return Transition(torch.zeros((N, T + 1, W), dtype=torch.int32, device="cuda"),
                                  torch.zeros((N, T + 1, W), dtype=torch.int32, device="cuda"),
                                  torch.zeros((N, T, W), dtype=torch.uint8, device="cuda"),
                                  torch.zeros((N, T, W), dtype=torch.float32, device="cuda"),
                                  torch.zeros((N, T, W), dtype=torch.uint8, device="cuda"))
            ref, got = buf(), buf()
            c_ref = torch.zeros((N, W), device="cuda")
            c_got = torch.zeros((N, W), device="cuda")
            _lib.call("toued_rollout", rw._c, _lib.ptr(lev), _lib.ptr(th), spec.obs_dim, _lib.ptr(ukeys[u]),
                      _lib.ptr(s_ref), N, W, T, _lib.ptr(ref.obs_idx), _lib.ptr(ref.obs_time), _lib.ptr(ref.action),
                      _lib.ptr(ref.reward), _lib.ptr(ref.done), _lib.ptr(c_ref), _lib.stream_ptr())
            rw.rollout_from_draws(draws, u, th, lev, s_got, got, c_got)
            for name in ("obs_idx", "obs_time", "action", "reward", "done"):
                assert torch.equal(getattr(got, name), getattr(ref, name)), (scale, u, name)
            assert torch.equal(s_got, s_ref) and torch.equal(c_got, c_ref), (scale, u)
        # the production path (batch_rollout's default split path) on batch 0's keys
        o, s2, c2 = rw.batch_rollout(ukeys[0], th, lev, st0)
        ref0, s0r, c0r = buf(), st0.clone(), torch.zeros((N, W), device="cuda")
        _lib.call("toued_rollout", rw._c, _lib.ptr(lev), _lib.ptr(th), spec.obs_dim, _lib.ptr(ukeys[0]),
                  _lib.ptr(s0r), N, W, T, _lib.ptr(ref0.obs_idx), _lib.ptr(ref0.obs_time), _lib.ptr(ref0.action),
                  _lib.ptr(ref0.reward), _lib.ptr(ref0.done), _lib.ptr(c0r), _lib.stream_ptr())
        assert torch.equal(o.action, ref0.action) and torch.equal(s2, s0r) and torch.equal(c2, c0r)
