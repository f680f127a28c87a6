"""The C++/OpenMP CPU restatement (oracle/cpu, the bench's second CPU baseline) against the numpy oracle:
rollout trajectories, end states and returns bit-exact (tabular, non-tabular with Gumbel respawn, mazes);
GAE within float32 rounding of the float64 oracle."""
import numpy as np
import pytest
import torch

from oracle import cpu
from oracle import jaxrand as jr
from oracle import levels as olv
from oracle import meta as ometa
from oracle import rollout as oro


def _soa(st, nmax):
    n = st["pos"].shape[0]
    s = np.zeros((12, n), np.int32)
    s[0], s[1] = st["time"], st["pos"]
    s[2] = np.sum(st["obj_existss"] * (1 << np.arange(nmax))[None, :], axis=1)
    s[3] = st["early_term"]
    s[4:4 + nmax] = st["obj_poss"].T
    return s


def _ptr(a):
    return a.ctypes.data


@pytest.mark.parametrize("mode", ["dense", "tabular", "all_shortlife", "mazes"])
def test_cpu_rollout_bitexact(mode):
    N, W, T = 3, 16, 40
    spec = olv.env_spec(mode)
    keys = jr.split(jr.PRNGKey(5), N)
    p, lt = olv.reset_env_params(keys, mode)
    lev = np.ascontiguousarray(olv.pack_levels(p, lt, spec))
    D = spec.obs_dim
    theta = (np.random.RandomState(0).randn(N, D, 5) * 3).astype(np.float32)
    st0 = oro.batch_reset(spec, jr.split(jr.PRNGKey(6), N), p, W)
    rk = np.ascontiguousarray(jr.split(jr.PRNGKey(7), N))
    otr, ost, ocum = oro.batch_rollout(spec, rk, theta, p, st0, T)
    state = np.ascontiguousarray(_soa(st0, spec.max_n_objs))
    idx = np.zeros((N, T + 1, W), np.int32)
    tm = np.zeros_like(idx)
    act = np.zeros((N, T, W), np.uint8)
    rew = np.zeros((N, T, W), np.float32)
    dn = np.zeros((N, T, W), np.uint8)
    cum = np.zeros(N * W, np.float32)
    rc = cpu.lib().toued_cpu_rollout(spec.max_grid_size, spec.max_n_objs, spec.max_n_obj_types, int(spec.tabular),
                                     _ptr(lev), _ptr(theta), D, _ptr(rk), _ptr(state), T, W, N, _ptr(idx), _ptr(tm),
                                     _ptr(act), _ptr(rew), _ptr(dn), _ptr(cum))
    assert rc == 0
    np.testing.assert_array_equal(idx, otr["idx"].transpose(0, 2, 1))
    np.testing.assert_array_equal(tm, otr["time"].transpose(0, 2, 1))
    np.testing.assert_array_equal(act, otr["action"].transpose(0, 2, 1))
    np.testing.assert_array_equal(rew, otr["reward"].transpose(0, 2, 1))
    np.testing.assert_array_equal(dn.astype(bool), otr["done"].transpose(0, 2, 1))
    np.testing.assert_array_equal(cum, ocum.reshape(-1))
    np.testing.assert_array_equal(state, _soa(ost, spec.max_n_objs))
    # GAE on the same trajectory with a random linear value critic
    vc = np.random.RandomState(1).randn(N, D).astype(np.float32)
    adv = np.zeros((N * W, T), np.float32)
    tgt = np.zeros_like(adv)
    cpu.lib().toued_cpu_gae(_ptr(vc), D, _ptr(idx), _ptr(tm), _ptr(rew), _ptr(dn), T, W, N, 0.99, 0.95, _ptr(adv),
                            _ptr(tgt))
    for a in range(N):
        v = ometa.linear_logits(torch.tensor(vc[a][:, None], dtype=torch.float64), idx[a].T, tm[a].T)[..., 0]
        ra, ta = ometa.gae(v, torch.tensor(rew[a].T, dtype=torch.float64),
                           torch.tensor(dn[a].T.astype(np.float64)), 0.99, 0.95)
        np.testing.assert_allclose(adv[a * W:(a + 1) * W], ra.numpy(), rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(tgt[a * W:(a + 1) * W], ta.numpy(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("mode,lifetime", [("dense", 100), ("all_shortlife", 100), ("dense", 0)])
def test_cpu_a2c_update_matches_oracle(mode, lifetime):
    """toued_cpu_a2c_update (the C3 CPU baseline's update, agents/a2c.py:19-76) against oracle/a2c.py a2c_step in
    float64: parameter changes within 1e-4 relative L2 (float32 sums), losses within 1e-4; lifetime 0 discards."""
    N, W, T = 3, 16, 20
    spec = olv.env_spec(mode)
    keys = jr.split(jr.PRNGKey(15), N)
    p, lt = olv.reset_env_params(keys, mode)
    lt = np.full_like(lt, lifetime)
    lev = np.ascontiguousarray(olv.pack_levels(p, lt, spec))
    D = spec.obs_dim
    rs = np.random.RandomState(3)
    theta = (rs.randn(N, D, 5) * 3).astype(np.float32)
    vc = (rs.randn(N, D) * 0.5).astype(np.float32)
    st0 = oro.batch_reset(spec, jr.split(jr.PRNGKey(16), N), p, W)
    otr, _, _ = oro.batch_rollout(spec, jr.split(jr.PRNGKey(17), N), theta, p, st0, T)
    idx = np.ascontiguousarray(otr["idx"].transpose(0, 2, 1)).astype(np.int32)
    tm = np.ascontiguousarray(otr["time"].transpose(0, 2, 1)).astype(np.int32)
    act = np.ascontiguousarray(otr["action"].transpose(0, 2, 1)).astype(np.uint8)
    rew = np.ascontiguousarray(otr["reward"].transpose(0, 2, 1)).astype(np.float32)
    dn = np.ascontiguousarray(otr["done"].transpose(0, 2, 1)).astype(np.uint8)
    th1, vc1 = theta.copy(), vc.copy()
    step = np.zeros(N, np.int32)
    loss = np.zeros((N, 2), np.float32)
    hyp = ometa.Hypers()
    cpu.lib().toued_cpu_a2c_update(_ptr(th1), _ptr(vc1), _ptr(step), _ptr(lev), D, _ptr(idx), _ptr(tm), _ptr(act),
                                   _ptr(rew), _ptr(dn), T, W, N, hyp.gamma, hyp.gae_lambda, 0.01, 40.0, 4.0, 0.5,
                                   _ptr(loss))
    from oracle import a2c as oa2c
    for a in range(N):
        traj = {"idx": otr["idx"][a], "time": otr["time"][a], "action": otr["action"][a].astype(np.int64),
                "reward": otr["reward"][a], "done": otr["done"][a].astype(bool)}
        t_ref, v_ref, s_ref, al, cl = oa2c.a2c_step(torch.from_numpy(theta[a].astype(np.float64)),
                                                    torch.from_numpy(vc[a][:, None].astype(np.float64)), 0,
                                                    lifetime, traj, hyp, 40.0, 4.0, 0.5)
        assert int(step[a]) == s_ref
        assert abs(loss[a, 0] - al) <= 1e-4 * max(1.0, abs(al)) and abs(loss[a, 1] - cl) <= 1e-4 * max(1.0, abs(cl))
        dt_ref, dv_ref = t_ref.numpy() - theta[a], v_ref.numpy()[:, 0] - vc[a]
        dt, dv = th1[a].astype(np.float64) - theta[a], vc1[a].astype(np.float64) - vc[a]
        if lifetime == 0:
            assert not dt.any() and not dv.any()
        else:
            assert np.linalg.norm(dt - dt_ref) <= 1e-4 * np.linalg.norm(dt_ref), a
            assert np.linalg.norm(dv - dv_ref) <= 1e-4 * np.linalg.norm(dv_ref), a
