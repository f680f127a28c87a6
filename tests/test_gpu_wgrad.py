"""GPU check of the weight-gradient reduction kernel (csrc/wgrad.hip, toued_wgrad).

C[ra][rb] = A[ra x K] . B[rb x K]^T is the f32 reduction behind every LPG weight gradient (the jax.vjp of
models/lpg.py's GRU and heads, meta/meta.py:177-181).  Checked against a float64 torch product on the
same f32 operands over the shapes the LPG backward uses, ragged tiles (rb not a multiple of 128, ra not a
multiple of 16), strided rows, K = 0 and a single 32-k slab.  Tolerance: |C - C64| <= 2e-6 * sqrt(K) *
(|A| . |B|^T) elementwise (f32 accumulation over K terms), and bit-identical repeat runs (the split-K
partials are summed in a fixed order).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def run(ra, rb, K, lda=None, ldb=None, seed=0):
    from toued import _lib as L
    lda = K if lda is None else lda
    ldb = K if ldb is None else ldb
    g = torch.Generator(device="cuda").manual_seed(seed)
    Ab = torch.randn(max(ra, 1), max(lda, 4), generator=g, device="cuda")
    Bb = torch.randn(max(rb, 1), max(ldb, 4), generator=g, device="cuda")
    C = torch.full((ra, rb), float("nan"), device="cuda")
    need = int(L.lib().toued_wgrad_workspace_floats(ra, rb, K))
    work = torch.empty(max(need, 1), device="cuda")
    L.call("toued_wgrad", ra, rb, K, L.ptr(Ab), lda, L.ptr(Bb), ldb, L.ptr(C), L.ptr(work), work.numel(),
           L.stream_ptr())
    torch.cuda.synchronize()
    A = Ab[:ra, :K].double()
    B = Bb[:rb, :K].double()
    return C, A @ B.t(), A.abs() @ B.abs().t(), (Ab, Bb, work)


@pytest.mark.parametrize("ra,rb,K", [(262, 768, 32 * 700), (6, 256, 32 * 900), (9, 257, 32 * 640),
                                     (1, 1, 32), (17, 129, 96), (272, 130, 32 * 37), (16, 128, 32 * 5000),
                                     (100, 300, 32 * 333)])
def test_wgrad_matches_float64(ra, rb, K):
    C, ref, mag, _ = run(ra, rb, K)
    err = (C.double() - ref).abs()
    tol = 2e-6 * math.sqrt(K) * mag + 1e-30
    assert torch.isfinite(C).all()
    assert (err <= tol).all(), float((err / tol).max())


def test_wgrad_strided_rows_and_determinism():
    from toued import _lib as L
    ra, rb, K, lda, ldb = 40, 200, 32 * 300, 32 * 300 + 64, 32 * 300 + 12
    C, ref, mag, (Ab, Bb, work) = run(ra, rb, K, lda, ldb, seed=3)
    err = (C.double() - ref).abs()
    assert (err <= 2e-6 * math.sqrt(K) * mag).all()
    C2 = torch.empty_like(C)
    L.call("toued_wgrad", ra, rb, K, L.ptr(Ab), lda, L.ptr(Bb), ldb, L.ptr(C2), L.ptr(work), work.numel(),
           L.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(C, C2)


def test_wgrad_small_strided_rows_and_determinism():
    # ra <= 16 (the register-ring stream): row pitches past K, a partial last column tile, a ragged slab count
    from toued import _lib as L
    ra, rb, K, lda, ldb = 9, 257, 32 * 411, 32 * 411 + 36, 32 * 411 + 8
    C, ref, mag, (Ab, Bb, work) = run(ra, rb, K, lda, ldb, seed=5)
    err = (C.double() - ref).abs()
    assert (err <= 2e-6 * math.sqrt(K) * mag).all()
    C2 = torch.empty_like(C)
    L.call("toued_wgrad", ra, rb, K, L.ptr(Ab), lda, L.ptr(Bb), ldb, L.ptr(C2), L.ptr(work), work.numel(),
           L.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(C, C2)


def test_wgrad_empty_k_and_errors():
    from toued import _lib as L
    C = torch.full((3, 5), 7.0, device="cuda")
    A = torch.zeros(3, 4, device="cuda")
    L.call("toued_wgrad", 3, 5, 0, L.ptr(A), 4, L.ptr(A), 4, L.ptr(C), None, 0, L.stream_ptr())
    torch.cuda.synchronize()
    assert torch.count_nonzero(C) == 0
    with pytest.raises(Exception, match="multiple of 32"):
        L.call("toued_wgrad", 3, 5, 33, L.ptr(A), 36, L.ptr(A), 36, L.ptr(C), L.ptr(A), 12, L.stream_ptr())
    with pytest.raises(Exception, match="workspace"):
        L.call("toued_wgrad", 3, 5, 64, L.ptr(A), 64, L.ptr(A), 64, L.ptr(C), L.ptr(A), 1, L.stream_ptr())


def test_wgrad_ldc_and_rowsum_build_the_head_block():
    """The backward's head block [9][257] = DH . [relu(h_out); 1]^T as toued_gru_bwd_small builds it: the 256 unit
    columns by toued_wgrad_ldc (row stride 257), the bias column by toued_rowsum_into (DH's row sums), against
    float64; the ldc result bit-identical to toued_wgrad's columns and the other entries of the block untouched."""
    from toued import _lib as L
    ra, rb, K = 9, 256, 32 * 2000 + 32 * 7
    g = torch.Generator(device="cuda").manual_seed(11)
    A = torch.randn(ra, K, generator=g, device="cuda")
    B = torch.randn(rb, K, generator=g, device="cuda")
    blk = torch.full((ra + 1, rb + 1), float("nan"), device="cuda")
    need = max(int(L.lib().toued_wgrad_workspace_floats(ra, rb, K)), int(L.lib().toued_rowsum_workspace_floats(ra, K)))
    work = torch.empty(need, device="cuda")
    L.call("toued_wgrad_ldc", ra, rb, K, L.ptr(A), K, L.ptr(B), K, L.ptr(blk), rb + 1, L.ptr(work), need,
           L.stream_ptr())
    L.call("toued_rowsum_into", ra, K, L.ptr(A), K, L.ptr(blk) + 4 * rb, rb + 1, L.ptr(work), need, L.stream_ptr())
    C = torch.empty(ra, rb, device="cuda")
    L.call("toued_wgrad", ra, rb, K, L.ptr(A), K, L.ptr(B), K, L.ptr(C), L.ptr(work), need, L.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(blk[:ra, :rb], C)
    assert torch.isnan(blk[ra]).all()                      # the row past the block is not written
    Ad, Bd = A.double(), B.double()
    ref, mag = Ad @ Bd.t(), Ad.abs() @ Bd.abs().t()
    assert ((C.double() - ref).abs() <= 2e-6 * math.sqrt(K) * mag).all()
    rs, rmag = Ad.sum(1), Ad.abs().sum(1)
    assert ((blk[:ra, rb].double() - rs).abs() <= 2e-6 * math.sqrt(K) * rmag).all()


def _col_exp(B):
    """the backward's per-column exponent: 2^e * max_j |B[j][m]| < 2^14 (127 for an all-zero column)"""
    mx = B.abs().amax(dim=0)
    _, e = torch.frexp(mx)
    ce = (14 - e).clamp(-126, 126)
    return torch.where(mx > 0, ce, torch.full_like(ce, 127)).to(torch.int8).contiguous()


@pytest.mark.parametrize("K,spread", [(32 * 700, 12.0), (32 * 2000, 3.0), (32 * 37, 20.0)])
def test_wgrad_bfp_matches_float64(K, spread):
    """toued_wgrad_bfp (block-floating-point fp16 pairs) on the LPG shape: rows 0..255 bounded by 1 (the GRU
    carry), feature rows of magnitudes 1e-3..1e3 (one all-zero), B columns spread over `spread` decades (one
    all-zero): the same f32-class bound as the bf16-triple kernel, and deterministic."""
    from toued import _lib as L
    ra, rb = 262, 768
    g = torch.Generator(device="cuda").manual_seed(int(K + spread))
    A = torch.empty(ra, K, device="cuda")
    A[:256].uniform_(-1, 1, generator=g)
    A[256:] = torch.randn(6, K, generator=g, device="cuda") * torch.tensor([1e-3, 1.0, 1e3, 7.0, 0.0, 1.0],
                                                                            device="cuda")[:, None]
    A[261] = 1.0
    B = torch.randn(rb, K, generator=g, device="cuda")
    B *= torch.pow(10.0, -spread * torch.rand(K, generator=g, device="cuda"))[None, :]
    B[:, 5] = 0.0
    CE = _col_exp(B)
    C = torch.full((ra, rb), float("nan"), device="cuda")
    work = torch.empty(int(L.lib().toued_wgrad_bfp_workspace_floats(ra, rb, K)), device="cuda")
    L.call("toued_wgrad_bfp", ra, rb, K, L.ptr(A), K, 256, L.ptr(B), K, L.ptr(CE), L.ptr(C), L.ptr(work),
           work.numel(), L.stream_ptr())
    torch.cuda.synchronize()
    ref = A.double() @ B.double().t()
    mag = A.double().abs() @ B.double().abs().t()
    err = (C.double() - ref).abs()
    assert torch.isfinite(C).all()
    assert (err <= 2e-6 * math.sqrt(K) * mag + 1e-300).all(), float((err / (mag + 1e-300)).max())
    rel = float((err.norm() / ref.norm()))
    assert rel < 2e-6, rel
    C2 = torch.empty_like(C)
    L.call("toued_wgrad_bfp", ra, rb, K, L.ptr(A), K, 256, L.ptr(B), K, L.ptr(CE), L.ptr(C2), L.ptr(work),
           work.numel(), L.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(C, C2)
    # B in 32-column slab blocks of 256 rows (the fused backward's DG layout): the same products, the same result
    Bs = B.view(rb // 256, 256, K // 32, 32).permute(0, 2, 1, 3).contiguous()
    C3 = torch.full_like(C, float("nan"))
    L.call("toued_wgrad_bfp_slab", ra, rb, K, L.ptr(A), K, 256, L.ptr(Bs), K, 2, L.ptr(CE), L.ptr(C3), L.ptr(work),
           work.numel(), L.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(C, C3)
    # and A's rows 0..255 in slab blocks too (the split-precision GRU pair's h_in), alone and with B's
    As = torch.cat([A[:256].view(256, K // 32, 32).permute(1, 0, 2).reshape(256, K), A[256:]]).contiguous()
    for layout, b in ((1, B), (3, Bs)):
        C4 = torch.full_like(C, float("nan"))
        L.call("toued_wgrad_bfp_slab", ra, rb, K, L.ptr(As), K, 256, L.ptr(b), K, layout, L.ptr(CE), L.ptr(C4),
               L.ptr(work), work.numel(), L.stream_ptr())
        torch.cuda.synchronize()
        assert torch.equal(C, C4), layout
