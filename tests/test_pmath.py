"""Accuracy of the portable f32 exp/log shared by the oracle and the HIP kernels."""
import numpy as np

from oracle import pmath


def test_exp_ulp():
    x = np.random.RandomState(0).uniform(-87, 88, 200000).astype(np.float32)
    e = pmath.exp(x)
    ref = np.exp(x.astype(np.float64))
    ulp = np.abs(e - ref) / np.spacing(ref.astype(np.float32)).astype(np.float64)
    assert ulp.max() <= 1.5


def test_exp_edges():
    out = pmath.exp(np.float32([0.0, -104.0, 89.0, np.nan, -87.5, -100.0]))
    assert out[0] == 1.0 and out[1] == 0.0 and np.isinf(out[2]) and np.isnan(out[3])
    assert 0 < out[5] < np.finfo(np.float32).tiny  # subnormal result kept
    np.testing.assert_allclose(out[4], np.exp(-87.5), rtol=1e-6)


def test_log_ulp():
    y = np.exp(np.random.RandomState(1).uniform(-80, 80, 200000)).astype(np.float32)
    l = pmath.log(y)
    ref = np.log(y.astype(np.float64))
    ulp = np.abs(l - ref) / np.spacing(np.abs(ref).astype(np.float32))
    assert ulp.max() <= 1.0


def test_log_edges():
    out = pmath.log(np.float32([0.0, -1.0, np.inf, 1.0, 1e-42]))
    assert np.isneginf(out[0]) and np.isnan(out[1]) and np.isposinf(out[2]) and out[3] == 0.0
    np.testing.assert_allclose(out[4], np.log(np.float64(np.float32(1e-42))), rtol=1e-6)
