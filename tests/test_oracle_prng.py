"""Pins the oracle's jax.random restatement (oracle/jaxrand.py) to published vectors.

* Random123 threefry2x32-20 known-answer tests (also in jax's random_test).
* jax.random.split(PRNGKey(0)) as printed in the JAX documentation.
* uniform/normal draws from PRNGKey(0)/PRNGKey(42) as printed in the JAX docs.
"""
import numpy as np

from oracle import jaxrand as jr


def test_threefry_kat():  # (also in tests/golden/prng_kat.json)
    cases = [((0, 0), (0, 0), (0x6B200159, 0x99BA4EFE)),
             ((0xFFFFFFFF, 0xFFFFFFFF), (0xFFFFFFFF, 0xFFFFFFFF), (0x1CB996FC, 0xBB002BE7)),
             ((0x13198A2E, 0x03707344), (0x243F6A88, 0x85A308D3), (0xC4923A9C, 0x483DF7A0))]
    for k, x, y in cases:
        out = jr.threefry2x32(k[0], k[1], x[0], x[1])
        assert (int(out[0]), int(out[1])) == y


def test_split_prngkey0():
    ks = jr.split(jr.PRNGKey(0))
    assert ks.tolist() == [[4146024105, 967050713], [2718843009, 1272950319]]


def test_published_draws():
    assert np.float32(jr.uniform(jr.PRNGKey(0))) == np.float32(0.41845703)
    assert np.float32(jr.normal(jr.PRNGKey(0), ())) == np.float32(-0.20584226)
    assert np.float32(jr.normal(jr.PRNGKey(42), ())) == np.float32(-0.18471177)


def test_prngkey_x32():
    assert jr.PRNGKey(7).tolist() == [0, 7]
    assert jr.PRNGKey(-1).tolist() == [0, 0xFFFFFFFF]


def test_split_batched_matches_single():
    keys = jr.split(jr.PRNGKey(3), 5)
    b = jr.split(keys, 3)
    for i in range(5):
        assert np.array_equal(b[i], jr.split(keys[i], 3))


def test_odd_count_padding():
    # threefry_2x32 with an odd count pads a 0 counter; element j<n comes from block j output 0
    k = jr.PRNGKey(11)
    bits5 = jr.random_bits(k, (5,))
    y = [jr.threefry2x32(k[0], k[1], b, (b + 3) if b + 3 < 5 else 0) for b in range(3)]
    assert bits5.tolist() == [int(y[0][0]), int(y[1][0]), int(y[2][0]), int(y[0][1]), int(y[1][1])]


def test_cumsum_assoc_order():
    p = np.float32([0.1, 0.2, 0.3, 0.15, 0.25])
    c = jr.cumsum_assoc(p)
    a, b, cc, d, e = p
    assert c.tolist() == [a, a + b, (a + b) + cc, (a + b) + (cc + d), ((a + b) + (cc + d)) + e]
    # generic n against the recursive definition for even/odd lengths
    for n in (1, 2, 3, 4, 7, 8, 13):
        x = np.random.RandomState(n).rand(n).astype(np.float32)
        np.testing.assert_allclose(jr.cumsum_assoc(x), np.cumsum(x), rtol=1e-6)


def test_randint_span_and_range():
    keys = jr.split(jr.PRNGKey(5), 2000)
    v = jr.randint(keys, (), 0, 7)
    assert v.min() == 0 and v.max() == 6
    counts = np.bincount(v, minlength=7)
    assert counts.min() > 200


def test_permutation_rounds():
    assert jr._num_shuffle_rounds(100) == 1
    assert jr._num_shuffle_rounds(512) == 1
    assert jr._num_shuffle_rounds(4000) == 2
    p = jr.permutation(jr.PRNGKey(0), 100)
    assert sorted(p.tolist()) == list(range(100))


def test_choice_replace_matches_definition():
    keys = jr.split(jr.PRNGKey(9), 1000)
    p = np.random.RandomState(0).dirichlet(np.ones(5), size=1000).astype(np.float32)
    a = jr.choice_p_replace(keys, p)
    c = jr.cumsum_assoc(p)
    u = jr.uniform(keys, ())
    r = c[:, -1] * (np.float32(1) - u)
    ref = np.array([np.searchsorted(c[i], r[i], side="left") for i in range(1000)])
    assert np.array_equal(a, ref)


def test_gumbel_topk_is_sample_without_replacement():
    keys = jr.split(jr.PRNGKey(1), 300)
    p = np.zeros((300, 10), np.float32)
    p[:, :6] = 1.0
    idx = jr.choice_p_noreplace(keys, p, 4)
    assert idx.max() < 6
    assert all(len(set(r)) == 4 for r in idx.tolist())
