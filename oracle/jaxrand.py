"""numpy restatement of jax 0.4.13's threefry PRNG (``jax.random``) — test oracle.

Reference call sites: environments/rollout.py:41,49,61,63,64;
environments/gridworld/gridworld.py:76,88,100,116,161,171;
environments/gridworld/configs.py:23,32,36,49,86,100-126;
environments/level_sampler.py:94-408; meta/train.py:41-197.
jax itself (setup/requirements-cpu.txt:1-2, jax==0.4.13) is not installed, so
this follows jax's published algorithm (jax/_src/prng.py, jax/_src/random.py,
non-partitionable threefry, x32 mode) and is pinned by the Random123 KATs.

Keys are uint32 arrays of shape [..., 2].  Every function is vectorised over
leading key dimensions.  Float transcendental functions use the portable
``oracle.pmath`` implementations that the HIP kernels share.
"""
from __future__ import annotations

import numpy as np

from . import pmath

U32 = np.uint32
_ROT = (np.array([13, 15, 26, 6], dtype=np.uint32), np.array([17, 29, 16, 24], dtype=np.uint32))


def _rotl(v, r):
    return ((v << U32(r)) | (v >> U32(32 - r))).astype(np.uint32)


def threefry2x32(k0, k1, x0, x1):
    """threefry2x32-20 block (jax/_src/prng.py `_threefry2x32_lowering`)."""
    k0 = np.asarray(k0, dtype=np.uint32)
    k1 = np.asarray(k1, dtype=np.uint32)
    x0 = np.asarray(x0, dtype=np.uint32)
    x1 = np.asarray(x1, dtype=np.uint32)
    with np.errstate(over="ignore"):
        ks = (k0, k1, (k0 ^ k1 ^ U32(0x1BD11BDA)).astype(np.uint32))
        x0 = (x0 + ks[0]).astype(np.uint32)
        x1 = (x1 + ks[1]).astype(np.uint32)
        for i in range(5):
            for r in _ROT[i % 2]:
                x0 = (x0 + x1).astype(np.uint32)
                x1 = _rotl(x1, int(r))
                x1 = (x0 ^ x1).astype(np.uint32)
            x0 = (x0 + ks[(i + 1) % 3]).astype(np.uint32)
            x1 = (x1 + ks[(i + 2) % 3] + U32(i + 1)).astype(np.uint32)
    return x0, x1


def PRNGKey(seed: int) -> np.ndarray:
    """jax.random.PRNGKey for a 32-bit seed: [seed >> 32 (=0 in x32), seed & 0xffffffff]."""
    return np.array([0, np.uint32(np.int64(seed) & 0xFFFFFFFF)], dtype=np.uint32)


def threefry_2x32(key, count: int) -> np.ndarray:
    """threefry_2x32(key, iota(count)) -> uint32[..., count].

    Odd counts are padded with a trailing 0 counter (jax/_src/prng.py
    `threefry_2x32`); counters are split into halves X0=iota[:n], X1=iota[n:].
    """
    key = np.asarray(key, dtype=np.uint32)
    lead = key.shape[:-1]
    odd = count % 2
    n = (count + odd) // 2
    ctr = np.arange(count + odd, dtype=np.uint32)
    if odd:
        ctr[-1] = 0
    x0 = np.broadcast_to(ctr[:n], lead + (n,))
    x1 = np.broadcast_to(ctr[n:], lead + (n,))
    k0 = key[..., 0:1]
    k1 = key[..., 1:2]
    y0, y1 = threefry2x32(k0, k1, x0, x1)
    out = np.concatenate([y0, y1], axis=-1)
    return out[..., :count] if odd else out


def random_bits(key, shape) -> np.ndarray:
    """_threefry_random_bits_original(key, 32, shape)."""
    shape = tuple(shape)
    size = int(np.prod(shape)) if shape else 1
    key = np.asarray(key, dtype=np.uint32)
    bits = threefry_2x32(key, size)
    return bits.reshape(key.shape[:-1] + shape)


def split(key, num: int = 2) -> np.ndarray:
    """jax.random.split: threefry_2x32(key, iota(2*num)).reshape(num, 2)."""
    key = np.asarray(key, dtype=np.uint32)
    bits = threefry_2x32(key, 2 * num)
    return bits.reshape(key.shape[:-1] + (num, 2))


def fold_in(key, data: int) -> np.ndarray:
    key = np.asarray(key, dtype=np.uint32)
    y0, y1 = threefry2x32(key[..., 0], key[..., 1], U32(0), U32(np.int64(data) & 0xFFFFFFFF))
    return np.stack([y0, y1], axis=-1)


def bits_to_unit_float(bits) -> np.ndarray:
    """(bits >> 9) | 0x3F800000 reinterpreted as f32, minus 1.0 -> [0, 1)."""
    b = (np.asarray(bits, dtype=np.uint32) >> U32(9)) | U32(0x3F800000)
    return b.view(np.float32) - np.float32(1.0)


def uniform(key, shape=(), minval=0.0, maxval=1.0) -> np.ndarray:
    """jax.random.uniform (float32): max(lo, f*(hi-lo)+lo) with no FMA contraction."""
    lo = np.float32(minval)
    hi = np.float32(maxval)
    f = bits_to_unit_float(random_bits(key, shape))
    return np.maximum(lo, (f * (hi - lo)) + lo).astype(np.float32)


def bernoulli(key, p, shape=None) -> np.ndarray:
    p = np.asarray(p, dtype=np.float32)
    if shape is None:
        shape = p.shape
    return uniform(key, shape) < p


def randint(key, shape, minval: int, maxval: int) -> np.ndarray:
    """jax.random.randint (int32): two bit draws from split(key), modular combine."""
    key = np.asarray(key, dtype=np.uint32)
    ks = split(key, 2)
    hi_b = random_bits(ks[..., 0, :], shape)
    lo_b = random_bits(ks[..., 1, :], shape)
    span = np.uint32(maxval - minval) if maxval > minval else np.uint32(1)
    mult = np.uint32((2 ** 16) % int(span))
    mult = np.uint32((int(mult) * int(mult)) % int(span))
    with np.errstate(over="ignore"):
        off = ((hi_b % span) * mult + (lo_b % span)).astype(np.uint32) % span
    return (np.int32(minval) + off.astype(np.int32)).astype(np.int32)


def sort_key_val_stable(keys, vals):
    order = np.argsort(keys, axis=-1, kind="stable")
    return np.take_along_axis(vals, order, axis=-1)


def _num_shuffle_rounds(size: int) -> int:
    return int(np.ceil(3 * np.log(max(1, size)) / np.log(np.iinfo(np.uint32).max)))


def shuffle(key, x) -> np.ndarray:
    """jax.random._shuffle along the last axis: repeated stable sort by random bits."""
    key = np.asarray(key, dtype=np.uint32)
    x = np.asarray(x)
    x = np.broadcast_to(x, key.shape[:-1] + x.shape[-1:]).copy()
    for _ in range(_num_shuffle_rounds(x.shape[-1])):
        ks = split(key, 2)
        key, sub = ks[..., 0, :], ks[..., 1, :]
        sort_keys = random_bits(sub, x.shape[-1:])
        x = sort_key_val_stable(sort_keys, x)
    return x


def permutation(key, n_or_x):
    if np.ndim(n_or_x) == 0:
        return shuffle(key, np.arange(int(n_or_x), dtype=np.int32))
    return shuffle(key, n_or_x)


def gumbel(key, shape) -> np.ndarray:
    """-log(-log(uniform(minval=tiny, maxval=1)))."""
    u = uniform(key, shape, minval=np.finfo(np.float32).tiny, maxval=1.0)
    return -pmath.log(-pmath.log(u))


def cumsum_assoc(p) -> np.ndarray:
    """jnp.cumsum lowered by jax 0.4.13 on CPU: lax.associative_scan order.

    For n=5: [a, a+b, (a+b)+c, (a+b)+(c+d), ((a+b)+(c+d))+e].
    Implemented generically by the same recursive odd/even scheme.
    """
    p = np.asarray(p, dtype=np.float32)

    def scan(e):
        n = e.shape[-1]
        if n < 2:
            return e
        reduced = e[..., 0:-1:2] + e[..., 1::2]
        odd = scan(reduced)
        if n % 2 == 0:
            even = odd[..., :-1] + e[..., 2::2]
        else:
            even = odd + e[..., 2::2]
        even = np.concatenate([e[..., 0:1], even], axis=-1)
        out = np.empty_like(e)
        out[..., 0::2] = even
        out[..., 1::2] = odd
        return out

    return scan(p)


def choice_p_replace(key, p, shape=()) -> np.ndarray:
    """choice(key, n, shape, replace=True, p=p) (jax/_src/random.py `choice`):
    ``searchsorted(cumsum(p), cumsum(p)[-1]*(1-uniform(key, shape)), side='left')``.

    The left insertion point into a non-decreasing array is the count of
    elements strictly below the query.  ``shape=()`` draws one index per key
    (p: [..., n]); ``shape=(m,)`` draws m indices from a single key (p: [n]).
    """
    c = cumsum_assoc(p)
    u = uniform(key, shape)
    if shape == ():
        r = c[..., -1] * (np.float32(1.0) - u)
        return np.sum(c < r[..., None], axis=-1).astype(np.int32)
    r = c[-1] * (np.float32(1.0) - u)
    return np.sum(c[None, :] < r[:, None], axis=-1).astype(np.int32)


def choice_p_noreplace(key, p, k: int) -> np.ndarray:
    """choice(key, n, (k,), replace=False, p=p): Gumbel top-k, stable argsort(-g - log p)[:k]."""
    p = np.asarray(p, dtype=np.float32)
    g = -gumbel(key, p.shape[-1:]) - pmath.log(p)
    order = np.argsort(g, axis=-1, kind="stable")
    return order[..., :k].astype(np.int32)


def choice_noreplace(key, n: int, k: int) -> np.ndarray:
    """choice(key, arange(n), (k,), replace=False) with p=None: permutation(key, arr)[:k]."""
    return permutation(key, np.arange(n, dtype=np.int32))[..., :k]


def choice_replace_uniform(key, n: int, shape=()) -> np.ndarray:
    """choice(key, arange(n), shape, replace=True) with p=None: randint(key, shape, 0, n)."""
    return randint(key, shape, 0, n)


def erf_inv(x) -> np.ndarray:
    return pmath.erfinv(np.asarray(x, dtype=np.float32))


def normal(key, shape) -> np.ndarray:
    lo = np.nextafter(np.float32(-1.0), np.float32(0.0))
    u = uniform(key, shape, minval=lo, maxval=1.0)
    return (np.float32(np.sqrt(2.0)) * erf_inv(u)).astype(np.float32)


def truncated_normal(key, lower, upper, shape) -> np.ndarray:
    """jax.random.truncated_normal: sqrt2*erfinv(U(erf(l/sqrt2), erf(u/sqrt2))), clipped open."""
    sqrt2 = np.float32(np.sqrt(2.0))
    a = pmath.erf(np.float32(lower) / sqrt2)
    b = pmath.erf(np.float32(upper) / sqrt2)
    u = uniform(key, shape, minval=a, maxval=b)
    out = sqrt2 * erf_inv(u)
    lo = np.nextafter(np.float32(lower), np.float32(np.inf))
    hi = np.nextafter(np.float32(upper), np.float32(-np.inf))
    return np.clip(out, lo, hi).astype(np.float32)
