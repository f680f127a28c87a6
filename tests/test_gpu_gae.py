"""toued_gae (util/metrics.py:17-38) on the GPU: bit-exact against the float32 restatement with the reference's
operation order (oracle/meta.py gae_f32), within 1e-5 of the float64 recurrence (oracle/meta.py gae), over the
batched layout, the reference's single-worker call, ragged sizes (T = 1, W = 1, N = 0) and all-done / never-done
episodes."""
import numpy as np
import pytest
import torch

from oracle import meta as ometa

pytestmark = pytest.mark.gpu


def _case(N, T, W, p_done, seed, scale=1.0):
    rs = np.random.RandomState(seed)
    v = (rs.randn(N, T + 1, W) * scale).astype(np.float32)
    r = (rs.randn(N, T, W) * scale).astype(np.float32)
    d = (rs.rand(N, T, W) < p_done).astype(np.uint8)
    return v, r, d


@pytest.mark.parametrize("N,T,W,p_done", [(5, 20, 64, 0.1), (3, 1, 64, 0.5), (7, 20, 1, 0.2), (2, 33, 96, 0.0),
                                          (2, 20, 64, 1.0), (0, 20, 64, 0.1), (512, 20, 64, 0.05)])
def test_gae_bitexact(N, T, W, p_done):
    from toued.metrics import gae
    v, r, d = _case(N, T, W, p_done, seed=N * 100 + T)
    adv, tgt = gae(torch.from_numpy(v).cuda(), torch.from_numpy(r).cuda(), torch.from_numpy(d).cuda(), 0.99, 0.95)
    torch.cuda.synchronize()
    # oracle in the reference's per-worker layout [.., T]
    va, ta = ometa.gae_f32(v.transpose(0, 2, 1), r.transpose(0, 2, 1), d.transpose(0, 2, 1), 0.99, 0.95)
    np.testing.assert_array_equal(adv.cpu().numpy(), va.transpose(0, 2, 1))
    np.testing.assert_array_equal(tgt.cpu().numpy(), ta.transpose(0, 2, 1))
    if N:
        a64, t64 = ometa.gae(torch.from_numpy(v.transpose(0, 2, 1)).double(), torch.from_numpy(r.transpose(0, 2, 1)).double(),
                             torch.from_numpy(d.transpose(0, 2, 1)).double(), 0.99, 0.95)
        np.testing.assert_allclose(adv.cpu().numpy(), a64.numpy().transpose(0, 2, 1), rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(tgt.cpu().numpy(), t64.numpy().transpose(0, 2, 1), rtol=1e-5, atol=1e-5)


def test_gae_single_worker_call_and_constant_reward():
    """The reference's own call shape (value [T+1], reward/done [T]); constant reward 1, zero value, no done: the
    closed form adv_t = sum_k (gamma lambda)^k over the remaining steps (target = adv)."""
    from toued.metrics import gae
    T = 20
    v = torch.zeros(T + 1, device="cuda")
    r = torch.ones(T, device="cuda")
    d = torch.zeros(T, dtype=torch.uint8, device="cuda")
    adv, tgt = gae(v, r, d, 0.99, 0.95)
    c = np.float32(0.99 * 0.95)
    ref = np.zeros(T, np.float32)
    g = np.float32(0.0)
    for t in reversed(range(T)):
        g = np.float32(np.float32(1.0) + c * g)
        ref[t] = g
    np.testing.assert_array_equal(adv.cpu().numpy(), ref)
    np.testing.assert_array_equal(tgt.cpu().numpy(), ref)
    closed = np.array([(1 - float(c) ** (T - t)) / (1 - float(c)) for t in range(T)])
    np.testing.assert_allclose(adv.cpu().numpy(), closed, rtol=1e-5)
