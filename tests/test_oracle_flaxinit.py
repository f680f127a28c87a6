"""oracle/flaxinit.py (flax 0.6.11 init restated) on CPU: key derivation, initialiser distributions, and the
product's host-side hash agreeing with the oracle's.  Parity unpinned (no flax output offline)."""
import hashlib

import numpy as np

from oracle import flaxinit
from oracle import jaxrand as jr
from oracle.lpg import layout


def test_static_hash_encoding():
    # names as utf-8, the params counter as minimal big-endian bytes, no separator (flax_fix_rng_separator off)
    want = int.from_bytes(hashlib.sha1(b"LPGGRU_0GRUCell_0hn\x01").digest()[:4], "big")
    assert flaxinit.static_hash(("LPGGRU_0", "GRUCell_0", "hn", 1)) == want
    assert flaxinit.static_hash(("Dense_0", 1)) != flaxinit.static_hash(("Dense_0", 2))
    assert flaxinit.static_hash(("a", 256)) == int.from_bytes(hashlib.sha1(b"a\x01\x00").digest()[:4], "big")


def test_param_key_is_one_fold_in():
    rng = jr.PRNGKey(3)
    k = flaxinit.param_key(rng, ("MLP_0", "Dense_1", 1))
    assert np.array_equal(k, jr.fold_in(rng, flaxinit.static_hash(("MLP_0", "Dense_1", 1))))
    assert np.array_equal(flaxinit.param_key(rng, ()), rng)


def test_product_hash_matches_oracle():
    from toued.agents import DENSE0_HASH, flax_static_hash
    from toued.lpg import FLAX_PARAM_PATHS
    assert DENSE0_HASH == flaxinit.static_hash(("Dense_0", 1))
    assert FLAX_PARAM_PATHS == flaxinit.LPG_PARAM_PATHS
    for _, path in FLAX_PARAM_PATHS.values():
        assert flax_static_hash(path + (1,)) == flaxinit.static_hash(path + (1,))


def test_lpg_init_distributions():
    F = 5
    eta = flaxinit.lpg_init(jr.PRNGKey(1), F)
    off = 0
    parts = {}
    for name, shape in layout(F).items():
        n = int(np.prod(shape))
        parts[name] = eta[off:off + n].reshape(shape)
        off += n
    assert off == eta.size
    for name, p in parts.items():
        if name.endswith("_b"):
            assert not p.any(), name
        elif name in ("hn_w", "hr_w", "hz_w"):
            q = p.astype(np.float64)
            np.testing.assert_allclose(q.T @ q, np.eye(256), atol=1e-5)
        else:
            bound = 2.0 * float(flaxinit.lecun_std(p.shape[0]))
            assert np.abs(p).max() < bound * (1 + 1e-6), name
    # different gates draw different matrices (distinct module paths)
    assert not np.allclose(parts["hr_w"], parts["hz_w"])
    # lecun std of the 256-fan-in y head (truncated normal variance = std^2 * .7737)
    assert abs(parts["y_w"].std() / (flaxinit.lecun_std(256) * np.sqrt(0.77374)) - 1) < 0.1
