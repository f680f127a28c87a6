"""Portable float32 transcendental functions — numpy side (test oracle).

The HIP kernels implement the *same* sequences of correctly rounded float32
operations in ``to-ued_amd/csrc/pmath.h`` (compiled with -ffp-contract=off), so
the oracle and the GPU produce bit-identical results for every quantity that
steers discrete decisions (softmax -> action sampling, Gumbel top-k, level
generation).  numpy float32 elementwise arithmetic is IEEE-754 round-to-nearest
with subnormals preserved, exactly like gfx950's default f32 mode.

Relative to XLA-CPU's own exp/log (what the reference runs) these differ by at
most a couple of ulp — that is the documented float tolerance.

exp: Cody-Waite range reduction + degree-7 Taylor polynomial + 2-step ldexp.
log: the classic musl/FreeBSD ``logf`` reduction (s = f/(2+f), odd series).
"""
from __future__ import annotations

import numpy as np

F = np.float32

_LOG2E = F(1.44269504088896341)
_LN2_HI = F(0.693145751953125)        # 0x3f317200, 15 significant bits
_LN2_LO = F(1.428606765330187045e-06)  # 0x35bfbe8e
_EXP_HI = F(88.72283905206835)
_EXP_LO = F(-103.972084)


def _inv_fact(i: int) -> np.float32:
    import math
    return F(1.0 / math.factorial(i))


_C = [_inv_fact(i) for i in range(8)]


def _pow2(k):
    """2**k as float32 for integer array k in [-126, 127] (exact)."""
    k = np.asarray(k, dtype=np.int32)
    return ((k + 127).astype(np.uint32) << np.uint32(23)).view(np.float32)


def exp(x):
    x = np.asarray(x, dtype=F)
    with np.errstate(over="ignore", under="ignore", invalid="ignore"):
        k = np.rint(x * _LOG2E).astype(F)
        r = x - k * _LN2_HI
        r = r - k * _LN2_LO
        p = _C[7]
        for i in (6, 5, 4, 3, 2, 1, 0):
            p = p * r + _C[i]
        ki = np.clip(k, -200, 200).astype(np.int32)
        k1 = ki // 2
        k2 = ki - k1
        res = (p * _pow2(np.clip(k1, -126, 127))) * _pow2(np.clip(k2, -126, 127))
        res = np.where(x > _EXP_HI, F(np.inf), res)
        res = np.where(x < _EXP_LO, F(0.0), res)
        res = np.where(np.isnan(x), x, res)
    return res.astype(F)


_LG1 = F(0.66666662693)   # 0xaaaaaa.0p-24
_LG2 = F(0.40000972152)   # 0xccce13.0p-25
_LG3 = F(0.28498786688)   # 0x91e9ee.0p-25
_LG4 = F(0.24279078841)   # 0xf89e26.0p-26
_SQRT2 = F(1.41421356237)


def log(x):
    x = np.asarray(x, dtype=F)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        sub = (x > 0) & (x < np.finfo(F).tiny)
        xs = np.where(sub, x * F(8388608.0), x)          # * 2^23 for subnormals
        bits = xs.view(np.uint32)
        e = ((bits >> np.uint32(23)) & np.uint32(0xFF)).astype(np.int32) - 127
        e = np.where(sub, e - 23, e)
        m = ((bits & np.uint32(0x7FFFFF)) | np.uint32(0x3F800000)).view(F)
        big = m > _SQRT2
        m = np.where(big, m * F(0.5), m)
        e = np.where(big, e + 1, e)
        f = m - F(1.0)
        s = f / (F(2.0) + f)
        z = s * s
        w = z * z
        t1 = w * (_LG2 + w * _LG4)
        t2 = z * (_LG1 + w * _LG3)
        R = t2 + t1
        hfsq = F(0.5) * f * f
        dk = e.astype(F)
        res = dk * _LN2_HI - ((hfsq - (s * (hfsq + R) + dk * _LN2_LO)) - f)
        res = np.where(x == 0, F(-np.inf), res)
        res = np.where(x < 0, F(np.nan), res)
        res = np.where(np.isinf(x) & (x > 0), F(np.inf), res)
        res = np.where(np.isnan(x), x, res)
    return res.astype(F)


# erf / erfinv are only used by the agent-parameter initialiser (truncated
# normal), whose parity is unpinned (flax init RNG derivation).
# Giles' single-precision erfinv approximation (the one XLA uses for f32).
def erfinv(x):
    x = np.asarray(x, dtype=F)
    with np.errstate(divide="ignore", invalid="ignore"):
        w = -log((F(1.0) - x) * (F(1.0) + x))
        small = w < F(5.0)
        ws = w - F(2.5)
        p1 = F(2.81022636e-08)
        for c in (3.43273939e-07, -3.5233877e-06, -4.39150654e-06, 0.00021858087,
                  -0.00125372503, -0.00417768164, 0.246640727, 1.50140941):
            p1 = F(c) + p1 * ws
        wl = np.sqrt(np.maximum(w, F(0.0))).astype(F) - F(3.0)
        p2 = F(-0.000200214257)
        for c in (0.000100950558, 0.00134934322, -0.00367342844, 0.00573950773,
                  -0.0076224613, 0.00943887047, 1.00167406, 2.83297682):
            p2 = F(c) + p2 * wl
        p = np.where(small, p1, p2)
        res = p * x
        res = np.where(np.abs(x) == F(1.0), x * F(np.inf), res)
    return res.astype(F)


def erf(x):
    """float32 erf via float64 (only used for two constants of the initialiser)."""
    import math
    x = np.asarray(x, dtype=np.float64)
    return np.vectorize(math.erf)(x).astype(F)
