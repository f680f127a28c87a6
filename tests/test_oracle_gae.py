"""The float32 GAE restatement (oracle/meta.py gae_f32, util/metrics.py:17-38): known answers and the float64
recurrence."""
import numpy as np
import torch

from oracle import meta as ometa


def test_gae_f32_known_answers():
    T = 6
    # constant reward 1, zero value, no done: adv_t = sum_{k < T-t} (gamma lambda)^k
    a, t = ometa.gae_f32(np.zeros(T + 1), np.ones(T), np.zeros(T, bool), 0.99, 0.95)
    c = 0.99 * 0.95
    np.testing.assert_allclose(a, [(1 - c ** (T - i)) / (1 - c) for i in range(T)], rtol=1e-6)
    np.testing.assert_array_equal(a, t)
    # done at every step: adv_t = r_t - v_t (no bootstrap, no carry)
    v = np.arange(T + 1, dtype=np.float32)
    r = np.full(T, 2.0, np.float32)
    a, t = ometa.gae_f32(v, r, np.ones(T, bool), 0.99, 0.95)
    np.testing.assert_array_equal(a, r - v[:-1])
    np.testing.assert_array_equal(t, r)


def test_gae_f32_matches_float64():
    rs = np.random.RandomState(0)
    v = rs.randn(4, 64, 21).astype(np.float32)
    r = rs.randn(4, 64, 20).astype(np.float32)
    d = rs.rand(4, 64, 20) < 0.1
    a, t = ometa.gae_f32(v, r, d, 0.99, 0.95)
    a64, t64 = ometa.gae(torch.from_numpy(v).double(), torch.from_numpy(r).double(), torch.from_numpy(d).double(),
                         0.99, 0.95)
    np.testing.assert_allclose(a, a64.numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(t, t64.numpy(), rtol=1e-5, atol=1e-5)
