"""LPG model on MI355X: flat parameter layout, initialisation, MFMA GRU forward/backward.

models/lpg.py:11-96 (LPG, LPGGRU) + meta/meta.py:10-30 (create_lpg_train_state).
The parameters are one flat f32 vector in jax ``tree_flatten`` order of the
flax param dict (the layout evosax's ParameterReshaper ravels, and the one
oracle/lpg.py uses):

  Dense_0 {bias[1], kernel[H,1]}  Dense_1 {bias[Y], kernel[H,Y]}
  LPGGRU_0/GRUCell_0: hn{bias,kernel[H,H]} hr{kernel} hz{kernel} in{bias,kernel[F,H]} ir{..} iz{..}
  MLP_0: Dense_0 {bias[E], kernel[Y,E]}  Dense_1 {bias[1], kernel[E,1]}

F = 5 input features, 7 with --lifetime_conditioning.  H = 256 (lpg_gru_width),
Y = 8 (lpg_target_width), E = 16 (lpg_embedding_net_width) are what the HIP
kernels are built for.
"""
from __future__ import annotations

import ctypes
import os
import math
from collections import OrderedDict

import numpy as np
import torch

from . import _lib, prng

H, Y, E = 256, 8, 16
_OFF_ORDER = ("pi_b", "pi_w", "y_b", "y_w", "hn_b", "hn_w", "hr_w", "hz_w", "in_b", "in_w", "ir_b", "ir_w",
              "iz_b", "iz_w", "e1_b", "e1_w", "e2_b", "e2_w")


def layout(F: int) -> "OrderedDict[str, tuple]":
    L = OrderedDict()
    L["pi_b"], L["pi_w"] = (1,), (H, 1)
    L["y_b"], L["y_w"] = (Y,), (H, Y)
    L["hn_b"], L["hn_w"], L["hr_w"], L["hz_w"] = (H,), (H, H), (H, H), (H, H)
    L["in_b"], L["in_w"], L["ir_b"], L["ir_w"], L["iz_b"], L["iz_w"] = (H,), (F, H), (H,), (F, H), (H,), (F, H)
    L["e1_b"], L["e1_w"], L["e2_b"], L["e2_w"] = (E,), (Y, E), (1,), (E, 1)
    return L


class LPGLayout:
    def __init__(self, F: int, kernel_test: bool = False):
        # the model's input width is 5, or 7 with lifetime conditioning (models/lpg.py:38-85); the GRU kernels take
        # 1..7 (the augmented k-step holds x and the bias row in 8), which the kernel tests use for the edges of the
        # fused small products' A table -- only through kernel_test=True, so a wrong width fails on the product path
        if kernel_test:
            if not 1 <= F <= 7:
                raise ValueError(f"LPG input width F={F}: the GRU kernels take 1..7")
        elif F not in (5, 7):
            raise ValueError(f"LPG input width F={F}: the model defines 5, or 7 with lifetime conditioning")
        self.F = F
        self.shapes = layout(F)
        self.offsets = {}
        off = 0
        for k, s in self.shapes.items():
            self.offsets[k] = off
            off += int(np.prod(s))
        self.size = off
        self.off_array = np.array([self.offsets[k] for k in _OFF_ORDER], np.int32)
        self._c_off = (ctypes.c_int * len(_OFF_ORDER))(*self.off_array.tolist())

    def view(self, flat: torch.Tensor, name: str) -> torch.Tensor:
        o = self.offsets[name]
        s = self.shapes[name]
        return flat[o:o + int(np.prod(s))].view(s)

    @property
    def c_offsets(self):
        return self._c_off


# create_lpg_train_state (meta/meta.py:21-22): the flax module path of each weight (models/lpg.py:38-85 --
# MLP_0 embedding, LPGGRU_0/GRUCell_0 gates under nn.scan with split_rngs={"params": False}, Dense_0/Dense_1
# heads) and its initialiser (flax 0.6.11 Dense: lecun_normal kernel, zero bias; GRUCell: lecun_normal input
# kernels, orthogonal recurrent kernels, zero biases).  Every kernel is its module's first param (counter 1).
_GRU_PATH = ("LPGGRU_0", "GRUCell_0")
FLAX_PARAM_PATHS = {
    "pi_w": ("lecun", ("Dense_0",)), "y_w": ("lecun", ("Dense_1",)),
    "hn_w": ("orth", _GRU_PATH + ("hn",)), "hr_w": ("orth", _GRU_PATH + ("hr",)),
    "hz_w": ("orth", _GRU_PATH + ("hz",)), "in_w": ("lecun", _GRU_PATH + ("in",)),
    "ir_w": ("lecun", _GRU_PATH + ("ir",)), "iz_w": ("lecun", _GRU_PATH + ("iz",)),
    "e1_w": ("lecun", ("MLP_0", "Dense_0")), "e2_w": ("lecun", ("MLP_0", "Dense_1")),
}


def flax_init_lpg_params(lpg_rng: torch.Tensor, F: int) -> torch.Tensor:
    """``lpg_model.init(lpg_rng, ...)["params"]`` (meta/meta.py:21-22) as the flat f32 eta on lpg_rng's device.

    Per-weight keys: fold_in(lpg_rng, sha1(path + counter)) (flax lazy RNG, toued.agents.flax_static_hash).
    lecun_normal kernels are drawn by the truncated-normal table kernel (toued_init_tables); the orthogonal
    recurrent kernels draw normal(key, (256, 256)) on the device (toued_normal) and take the sign-fixed QR
    factor Q * sign(diag R) (jax/_src/nn/initializers.py orthogonal) -- one 256x256 float64 QR per gate at
    start-up, on the host."""
    from .agents import TN_HI, TN_LO, flax_static_hash
    dev = lpg_rng.device
    out = torch.zeros(LPGLayout(F).size, dtype=torch.float32, device=dev)
    lay = LPGLayout(F)
    key = lpg_rng.reshape(1, 2).contiguous()
    for name, shape in layout(F).items():
        if name.endswith("_b"):
            continue
        kind, path = FLAX_PARAM_PATHS[name]
        pk = prng.fold_in(key, flax_static_hash(path + (1,))).contiguous()
        dst = lay.view(out, name)
        if kind == "orth":
            n = shape[0]
            a = torch.empty(n * n, dtype=torch.float32, device=dev)
            _lib.call("toued_normal", _lib.ptr(pk), 1, n * n, _lib.ptr(a), _lib.stream_ptr())
            q, r = torch.linalg.qr(a.reshape(n, n).cpu().double())
            dst.copy_((q * torch.sign(torch.diagonal(r))[None, :]).float())
        else:
            fan_in, cols = shape
            std = float(np.float32(np.sqrt(np.float32(1.0 / fan_in))) / np.float32(0.87962566103423978))
            tab = torch.empty((fan_in, cols), dtype=torch.float32, device=dev)
            _lib.call("toued_init_tables", _lib.ptr(pk), 1, cols, fan_in, TN_LO, TN_HI, std, _lib.ptr(tab),
                      _lib.stream_ptr())
            dst.copy_(tab)
    return out


def init_lpg_params(seed: int, F: int, device=None) -> torch.Tensor:
    """Random LPG parameters with flax's init distributions (lecun-normal kernels, orthogonal recurrent
    kernels, zero biases) seeded from numpy -- a test utility for arbitrary eta; the training driver uses
    flax_init_lpg_params (the reference's own values).  Runs on the host, then lives on the GPU."""
    rs = np.random.RandomState(seed)
    parts = []
    for k, s in layout(F).items():
        if k.endswith("_b"):
            parts.append(np.zeros(s))
        elif k in ("hn_w", "hr_w", "hz_w"):
            q, r = np.linalg.qr(rs.randn(H, H))
            parts.append(q * np.sign(np.diag(r))[None, :])
        else:
            std = math.sqrt(1.0 / s[0]) / 0.87962566103423978
            parts.append(np.clip(rs.randn(*s), -2, 2) * std)
    flat = np.concatenate([p.ravel() for p in parts]).astype(np.float32)
    dev = torch.device(device) if device is not None else torch.device("cuda")
    return torch.from_numpy(flat).to(dev)


def quad_blocks_to_rows(flat: torch.Tensor, M: int) -> torch.Tensor:
    """[256][M] rows of an array in 32-column unit-quad blocks [M/32][64][32][4] (the split-precision GRU pair's saves:
    element (u, m) at (m >> 5) * 8192 + ((u >> 2) * 32 + (m & 31)) * 4 + (u & 3), gru.hip quad_soff)."""
    return flat.view(M // 32, 64, 32, 4).permute(1, 3, 0, 2).reshape(256, M)


class LPGGRU:
    """MFMA GRU forward/backward over K x R rows (csrc/gru.hip) with saved activations.

    Saved tensors are [256][M] with M = K*T*R columns ordered (k, t, r): the exact
    operand layout of the weight-gradient GEMMs.
    """

    def __init__(self, lay: LPGLayout, R: int, T: int, K: int, W: int, device, fused: bool | None = None):
        self.lay, self.R, self.T, self.K, self.W = lay, R, T, K, W
        self.M = K * T * R
        L = _lib.lib()
        dev = device
        f32 = torch.float32
        self.fwdA = torch.empty(int(L.toued_gru_packed_floats(0)), dtype=f32, device=dev)
        self.bwdA = torch.empty(int(L.toued_gru_packed_floats(1)), dtype=f32, device=dev)
        M = self.M
        # h_in saved as rows 0..255 of an augmented [264, M] operand whose rows 256..256+F-1 hold the
        # GRU inputs X (written by the LPG-input kernel) and row 256+F is all ones: one GEMM against the
        # gate cotangents then yields dW_h, dW_i and the biases together.
        self.A = torch.zeros((H + 8, M), dtype=f32, device=dev)
        self.A[H + lay.F].fill_(1.0)
        self.X = self.A[H:H + lay.F].view(lay.F, K, T, R)
        self.S = torch.empty((4, H, M), dtype=f32, device=dev)          # r, z, n (f32 fallback only), hn
        # the split-precision pair keeps h_in (A's first 256 rows' region) in 32-column slab blocks [M/32][256][32] and
        # r, z, hn in 32-column unit-quad blocks [M/32][64][32][4] (gru.hip slab_soff / quad_soff; hin_rows(),
        # a_rows(), s_rows() give rows); A's rows 256.. (x, ones) stay rows
        self.slab = bool(L.toued_gru_slab_saves(R))
        self.hin_slab = self.slab and bool(L.toued_gru_hin_slab())
        # the small weight-gradient products fused into the backward (toued_gru_bwd_fused) where the lockstep kernel
        # runs and F <= 6: then dn_pre, relu(h_out) and the head cotangents never reach HBM (TOUED_BWD_FUSED=0: the
        # unfused kernel + toued_gru_bwd_small)
        fits = bool(L.toued_gru_bwd_fused_fits(R, lay.F))
        self.fused = (fits and os.environ.get("TOUED_BWD_FUSED", "1") != "0") if fused is None else (fused and fits)
        # dr_pre, dz_pre, d(hn) (+ dn_pre when unfused); fused: each gate in 32-column slab blocks [M/32][256][32]
        # (toued_gru_bwd_fused -> toued_wgrad_bfp_slab), else [256][M] rows -- dg_rows() gives rows either way
        self.DG = torch.empty((3 if self.fused else 4, H, M), dtype=f32, device=dev)
        if self.fused:
            self.RH = self.DH = None
        else:
            self.RH = torch.zeros((H + 1, M), dtype=f32, device=dev)    # relu(h_out) + ones row
            self.RH[H].fill_(1.0)
            self.DH = torch.empty((9, M), dtype=f32, device=dev)        # head cotangents
        self._last_bwd = None
        self.keep_inputs = False   # tests: keep copies of the backward's inputs for relu_out()
        self.dX3 = torch.empty((K, T, R), dtype=f32, device=dev)
        self.dX4 = torch.empty((K, T, R), dtype=f32, device=dev)
        # weight-gradient reductions (csrc/wgrad.hip): outputs and the per-K-chunk partial-sum workspace
        # G and GI share one buffer so that their scatter into the flat gradient is one gather + one index_add
        ng, ngi = (H + lay.F + 1) * 3 * H, 8 * H + 9 * (H + 1)
        self._ggi = torch.empty(ng + ngi, dtype=f32, device=dev)
        self.G = self._ggi[:ng].view(H + lay.F + 1, 3 * H)
        # the backward's small products: [8][256] ([X; 1; 0] . dn^T) then [9][257] (DH . [relu(h_out); 1]^T)
        self.GI = self._ggi[ng:]
        self._scatter = None   # (src, dst) index pairs of the weight-gradient blocks into eta's flat layout
        # per-column cotangent exponents from the lockstep backward -> the block-floating-point fp16 reduction
        # (toued_wgrad_bfp, 3 products); else (or TOUED_WGRAD_X6=1) the bf16-triple reduction (toued_wgrad)
        self.bfp = bool(L.toued_gru_bwd_col_exp(R)) and os.environ.get("TOUED_WGRAD_X6") != "1" and \
            os.environ.get("TOUED_WGRAD_F32") != "1"
        self.CE = torch.empty(M if self.bfp else 0, dtype=torch.int8, device=dev)
        need = max(int(L.toued_wgrad_workspace_floats(H + lay.F + 1, 3 * H, M)),
                   int(L.toued_wgrad_bfp_workspace_floats(H + lay.F + 1, 3 * H, M)),
                   int(L.toued_gru_bwd_fused_work_floats(R, K)) if self.fused else int(L.toued_gru_bwd_small_work_floats(M)))
        self.wg_work = torch.empty(max(need, 1), dtype=f32, device=dev)

    def hin_rows(self):
        """The saved h_in as [256][M] rows (a copy of its slab blocks on the split-precision pair)."""
        H, M = 256, self.M
        if not self.hin_slab:
            return self.A[:H]
        return self.A[:H].reshape(-1).view(M // 32, H, 32).permute(1, 0, 2).reshape(H, M)

    def a_rows(self):
        """The main reduction's A operand [h_in; x; 1; pad] as [264][M] rows (a copy when h_in is in slab blocks)."""
        return torch.cat([self.hin_rows(), self.A[256:]]) if self.hin_slab else self.A

    def hin_block(self, k: int):
        """Update k's saved h_in (for --debug_nans): a [256][T*R] column block of the rows, or its contiguous slab
        blocks."""
        c0, n = k * self.T * self.R, self.T * self.R
        return self.A.view(-1)[256 * c0:256 * (c0 + n)] if self.hin_slab else self.A[:256, c0:c0 + n]

    def s_rows(self, i: int):
        """Saved array i (0 r, 1 z, 2 n, 3 hn) as [256][M] rows (a copy of its unit-quad blocks for r, z, hn)."""
        if not self.slab or i == 2:
            return self.S[i]
        return quad_blocks_to_rows(self.S[i].reshape(-1), self.S.shape[2])

    def dg_rows(self):
        """The gate cotangents as [gates][256][M] rows: DG itself (unfused), or a row-major copy of the fused
        backward's slab blocks (tests, comparison paths)."""
        if not self.fused:
            return self.DG
        g, H, M = self.DG.shape
        return self.DG.view(g, M // 32, H, 32).permute(0, 2, 1, 3).reshape(g, H, M)

    def _scatter_indices(self, dev):
        """(src into G|GI, dst into eta) for the blocks the backward accumulates, the same element pairs as the
        per-parameter views: hr_w <- G[0:H, 0:H], ..., heads <- GI[8H:] viewed [9][H+1] transposed."""
        lay, F = self.lay, self.lay.F
        ng = (H + F + 1) * 3 * H
        Gi = torch.arange(ng).view(H + F + 1, 3 * H)
        GIi = ng + torch.arange(8 * H + 9 * (H + 1))
        Gn = GIi[:8 * H].view(8, H)
        heads = GIi[8 * H:].view(9, H + 1).t()
        blocks = [("hr_w", Gi[0:H, 0:H]), ("hz_w", Gi[0:H, H:2 * H]), ("hn_w", Gi[0:H, 2 * H:3 * H]),
                  ("ir_w", Gi[H:H + F, 0:H]), ("iz_w", Gi[H:H + F, H:2 * H]), ("ir_b", Gi[H + F, 0:H]),
                  ("iz_b", Gi[H + F, H:2 * H]), ("hn_b", Gi[H + F, 2 * H:3 * H]), ("in_w", Gn[0:F]), ("in_b", Gn[F]),
                  ("pi_w", heads[0:H, 0:1]), ("y_w", heads[0:H, 1:9]), ("pi_b", heads[H, 0:1]), ("y_b", heads[H, 1:9])]
        src, dst = [], []
        for name, t in blocks:
            n = int(np.prod(lay.shapes[name]))
            assert t.numel() == n, (name, t.shape, lay.shapes[name])
            src.append(t.reshape(-1))
            dst.append(lay.offsets[name] + torch.arange(n))
        return torch.cat(src).to(dev, torch.int32), torch.cat(dst).to(dev, torch.int32)

    def pack(self, eta: torch.Tensor):
        _lib.call("toued_gru_pack", _lib.ptr(eta), self.lay.c_offsets, self.lay.F, _lib.ptr(self.fwdA),
                  _lib.ptr(self.bwdA), _lib.stream_ptr())

    def forward(self, k: int, X: torch.Tensor, done_k: torch.Tensor, eta: torch.Tensor, pi_hat: torch.Tensor,
                y_hat: torch.Tensor):
        """X: [F, K, T, R] (feature stride M); done_k: u8 [N, T, W]; pi_hat [K,T,R]; y_hat [K,T,8,R]."""
        R, T, M = self.R, self.T, self.M
        col = k * T * R
        Xk = X[:, k]
        S = self.S
        # this update's first column: [256][M] rows (the f32 pair) or its first slab block (the split-precision pair)
        sc = H * col if self.slab else col
        _lib.call("toued_gru_fwd", R, T, self.W, self.lay.F, _lib.ptr(X) + 4 * col, M, 1, _lib.ptr(done_k),
                  _lib.ptr(self.fwdA), _lib.ptr(eta), self.lay.c_offsets, _lib.ptr(pi_hat[k]), _lib.ptr(y_hat[k]),
                  _lib.ptr(self.A) + 4 * (sc if self.hin_slab else col), _lib.ptr(S) + 4 * (0 * H * M + sc),
                  _lib.ptr(S) + 4 * (1 * H * M + sc), _lib.ptr(S) + 4 * (2 * H * M + col),
                  _lib.ptr(S) + 4 * (3 * H * M + sc), M, _lib.stream_ptr())
        del Xk

    def relu_out(self) -> torch.Tensor:
        """relu(h_out) [256][M] of the last backward (tests: the relu decisions the backward took).  On the fused path
        the backward keeps it on chip, so the unfused kernel recomputes it from the same saves into scratch buffers
        (the same gate maths, so the same decisions)."""
        if not self.fused:
            return self.RH[:H]
        if self._last_bwd is None:
            raise RuntimeError("relu_out: set keep_inputs = True before the backward (the fused path keeps no relu rows)")
        done_all, eta, y_hat, d_pi_hat, d_y_hat = self._last_bwd
        M, dev, f32 = self.M, self.A.device, torch.float32
        DG4 = torch.empty((4, H, M), dtype=f32, device=dev)
        RH = torch.empty((H, M), dtype=f32, device=dev)
        DH = torch.empty((9, M), dtype=f32, device=dev)
        dX = torch.empty((2, M), dtype=f32, device=dev)
        CE = torch.empty(M, dtype=torch.int8, device=dev)
        S = self.S
        _lib.call("toued_gru_bwd", self.R, self.T, self.W, self.K, _lib.ptr(done_all), done_all[0].numel(),
                  _lib.ptr(self.bwdA), _lib.ptr(eta), self.lay.c_offsets, _lib.ptr(y_hat), _lib.ptr(d_pi_hat),
                  _lib.ptr(d_y_hat), _lib.ptr(self.A), _lib.ptr(S[0]), _lib.ptr(S[1]), _lib.ptr(S[2]), _lib.ptr(S[3]),
                  M, _lib.ptr(DG4), _lib.ptr(RH), _lib.ptr(DH), _lib.ptr(dX[0]), _lib.ptr(dX[1]), _lib.ptr(CE),
                  _lib.stream_ptr())
        return RH

    def backward(self, done_all: torch.Tensor, eta: torch.Tensor, y_hat: torch.Tensor, d_pi_hat: torch.Tensor,
                 d_y_hat: torch.Tensor, X: torch.Tensor, grad: torch.Tensor, timers=None, after_bwd=None,
                 before_main_wgrad=None):
        """done_all: u8 [K(+1), N, T, W] (first K slots used).  Accumulates d(loss)/d(eta) into ``grad``
        (all parameters except the embedding MLP, which needs dX3/dX4 -> agent-side kernel).  ``after_bwd()`` is
        called right after the recurrent backward kernel is enqueued, before the weight-gradient reductions;
        ``before_main_wgrad()`` right before the main one (after the small products)."""
        R, T, K, M = self.R, self.T, self.K, self.M
        S = self.S
        stride_k = done_all[0].numel()
        ws, wn = _lib.ptr(self.wg_work), self.wg_work.numel()
        if self.keep_inputs:   # relu_out() recomputes from these after the caller has moved on (Adam updates eta)
            self._last_bwd = (done_all.clone(), eta.clone(), y_hat.clone(), d_pi_hat.clone(), d_y_hat.clone())
        tok = timers.start("gru_bwd") if timers is not None else None
        if self.fused:
            # the recurrent backward with GI (both small products) reduced from its per-workgroup partials
            _lib.call("toued_gru_bwd_fused", R, T, self.W, K, _lib.ptr(done_all), stride_k, _lib.ptr(self.bwdA),
                      _lib.ptr(eta), self.lay.c_offsets, _lib.ptr(y_hat), _lib.ptr(d_pi_hat), _lib.ptr(d_y_hat),
                      _lib.ptr(self.A), _lib.ptr(S[0]), _lib.ptr(S[1]), _lib.ptr(S[3]), M, _lib.ptr(self.DG),
                      _lib.ptr(self.dX3), _lib.ptr(self.dX4), _lib.ptr(self.CE), _lib.ptr(self.GI), ws, wn,
                      _lib.stream_ptr())
        else:
            _lib.call("toued_gru_bwd", R, T, self.W, K, _lib.ptr(done_all), stride_k, _lib.ptr(self.bwdA),
                      _lib.ptr(eta), self.lay.c_offsets, _lib.ptr(y_hat), _lib.ptr(d_pi_hat), _lib.ptr(d_y_hat),
                      _lib.ptr(self.A), _lib.ptr(S[0]), _lib.ptr(S[1]), _lib.ptr(S[2]), _lib.ptr(S[3]), M,
                      _lib.ptr(self.DG), _lib.ptr(self.RH), _lib.ptr(self.DH), _lib.ptr(self.dX3), _lib.ptr(self.dX4),
                      _lib.ptr(self.CE) if self.bfp else None, _lib.stream_ptr())
        if timers is not None:
            timers.stop(tok)
        if after_bwd is not None:
            after_bwd()
        if timers is not None:
            tok = timers.start("wgrad_gemm")
        lay = self.lay
        F = lay.F
        DG = self.DG
        # weight-gradient reductions over M = K*T*R on MFMA (csrc/wgrad.hip, deterministic split-K):
        #   [h_in; X; 1] (262 x M) . [dr; dz; dhn]^T  -> dW_h (rows 0..255), dW_ir/dW_iz (X rows), biases (ones row)
        #   GI: [X; 1] . dn^T -> dW_in, b_in;   DH . [relu(h_out); 1]^T -> head kernels and biases
        G = self.G
        st = _lib.stream_ptr()
        if not self.fused:
            _lib.call("toued_gru_bwd_small", M, _lib.ptr(self.A), _lib.ptr(DG), _lib.ptr(self.RH), _lib.ptr(self.DH),
                      _lib.ptr(self.GI), ws, wn, st)
        if before_main_wgrad is not None:
            before_main_wgrad()
        tok_main = timers.start("wgrad_main") if timers is not None else None
        if self.bfp and self.slab and os.environ.get("TOUED_WGRAD_NW4") != "1":
            # h_in in slab blocks (layout bit 0); the fused backward's DG too (bit 1), the unfused one's in rows
            _lib.call("toued_wgrad_bfp_slab", H + F + 1, 3 * H, M, _lib.ptr(self.A), M, H, _lib.ptr(DG), M,
                      (1 if self.hin_slab else 0) | (2 if self.fused else 0), _lib.ptr(self.CE), _lib.ptr(G), ws, wn,
                      st)
        else:
            # (comparison paths on the split-precision pair: row-major copies of the slab blocks)
            A, B = self.a_rows(), self.dg_rows()
            if self.bfp:
                _lib.call("toued_wgrad_bfp", H + F + 1, 3 * H, M, _lib.ptr(A), M, H, _lib.ptr(B), M,
                          _lib.ptr(self.CE), _lib.ptr(G), ws, wn, st)
            else:
                _lib.call("toued_wgrad", H + F + 1, 3 * H, M, _lib.ptr(A), M, _lib.ptr(B), M, _lib.ptr(G), ws, wn, st)
        if tok_main is not None:
            timers.stop(tok_main)
        # every block of G (dW_h, dW_i, biases) and GI (dW_in, b_in, head kernels and biases) into eta's layout:
        # one gather + one index_add over precomputed indices (each target element once) instead of 14 launches
        if self._scatter is None:
            self._scatter = self._scatter_indices(grad.device)
        src, dst = self._scatter
        _lib.call("toued_gather_add", _lib.ptr(grad), _lib.ptr(self._ggi), _lib.ptr(src), _lib.ptr(dst), src.numel(),
                  _lib.stream_ptr())
        if timers is not None:
            timers.stop(tok)
