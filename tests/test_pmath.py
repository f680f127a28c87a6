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


def _exp_le0(x):
    """numpy restatement of common.h pexp_le0 (the softmax-argument exp of the env chains)."""
    F = np.float32
    with np.errstate(over="ignore", under="ignore", invalid="ignore"):
        k = np.rint(x * pmath._LOG2E).astype(F)
        r = x - k * pmath._LN2_HI
        r = r - k * pmath._LN2_LO
        p = pmath._C[7]
        for i in (6, 5, 4, 3, 2, 1, 0):
            p = p * r + pmath._C[i]
        ki = np.fmax(k, F(-200)).astype(np.int32)
        k1 = ki >> 1
        k2 = ki - k1
        v = (p * pmath._pow2(k1)) * pmath._pow2(k2)
        v = np.where(x < pmath._EXP_LO, F(0.0), v)
        return np.where(np.isnan(x), x, v).astype(F)


def test_exp_le0_is_exp_on_nonpositive_arguments():
    # pexp_le0 drops pexp's overflow test and exponent clamps for x <= 0: bit-identical there (strided over every
    # negative float32 bit pattern, plus both signs of zero, -inf, NaN and the cut-over region)
    bits = np.arange(0x80000000, 0x100000000, 97, dtype=np.uint64).astype(np.uint32)
    x = np.concatenate([bits.view(np.float32),
                        np.float32([0.0, -0.0, -np.inf, np.nan, -103.972084, -103.97208, -103.9721, -87.33655]),
                        np.linspace(-110, 0, 200001, dtype=np.float32)])
    a, b = _exp_le0(x), pmath.exp(x)
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), x[~same][:10]
