"""jax.random key plumbing on the GPU (threefry keys as int32[..., 2] tensors).

Keys carry the uint32 bit patterns of jax's threefry keys in int32 storage.
All derivations run on device through the C ABI (csrc/prng.hip).
"""
from __future__ import annotations

import torch

from . import _lib


def PRNGKey(seed: int, device=None) -> torch.Tensor:
    """jax.random.PRNGKey(seed) -> int32[2] = [0, seed & 0xffffffff] (x32 mode)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    lo = int(seed) & 0xFFFFFFFF
    lo = lo - (1 << 32) if lo >= (1 << 31) else lo
    return torch.tensor([0, lo], dtype=torch.int32, device=dev)


def split(keys: torch.Tensor, num: int = 2) -> torch.Tensor:
    """jax.random.split over a batch: keys [..., 2] -> [..., num, 2]."""
    lead = keys.shape[:-1]
    flat = keys.reshape(-1, 2).contiguous()
    out = torch.empty((flat.shape[0], num, 2), dtype=torch.int32, device=keys.device)
    _lib.call("toued_split", _lib.ptr(flat), flat.shape[0], num, _lib.ptr(out), _lib.stream_ptr())
    return out.reshape(lead + (num, 2))


def split_planar(keys: torch.Tensor, num: int = 2) -> torch.Tensor:
    """split with the num axis first: keys [n, 2] -> [num, n, 2] (out[j] = split(keys, num)[:, j], contiguous)."""
    flat = keys.reshape(-1, 2).contiguous()
    out = torch.empty((num, flat.shape[0], 2), dtype=torch.int32, device=keys.device)
    _lib.call("toued_split_planar", _lib.ptr(flat), flat.shape[0], num, _lib.ptr(out), _lib.stream_ptr())
    return out


def fold_in(keys: torch.Tensor, data: int) -> torch.Tensor:
    lead = keys.shape[:-1]
    flat = keys.reshape(-1, 2).contiguous()
    out = torch.empty_like(flat)
    _lib.call("toued_fold_in", _lib.ptr(flat), flat.shape[0], int(data) & 0xFFFFFFFF, _lib.ptr(out),
              _lib.stream_ptr())
    return out.reshape(lead + (2,))


def random_bits(keys: torch.Tensor, m: int) -> torch.Tensor:
    """jax.random.bits(key, (m,)) per key -> int32 bit patterns [..., m]."""
    lead = keys.shape[:-1]
    flat = keys.reshape(-1, 2).contiguous()
    out = torch.empty((flat.shape[0], m), dtype=torch.int32, device=keys.device)
    _lib.call("toued_random_bits", _lib.ptr(flat), flat.shape[0], m, _lib.ptr(out), _lib.stream_ptr())
    return out.reshape(lead + (m,))


def uniform(keys: torch.Tensor, m: int = 1, minval: float = 0.0, maxval: float = 1.0) -> torch.Tensor:
    lead = keys.shape[:-1]
    flat = keys.reshape(-1, 2).contiguous()
    out = torch.empty((flat.shape[0], m), dtype=torch.float32, device=keys.device)
    _lib.call("toued_uniform", _lib.ptr(flat), flat.shape[0], m, float(minval), float(maxval), _lib.ptr(out),
              _lib.stream_ptr())
    return out.reshape(lead + (m,))


def to_uint32_numpy(keys: torch.Tensor):
    return keys.detach().cpu().numpy().view("uint32")


def from_uint32_numpy(arr, device=None) -> torch.Tensor:
    import numpy as np
    a = np.ascontiguousarray(arr, dtype=np.uint32).view(np.int32)
    return torch.from_numpy(a.copy()).to(device if device is not None else torch.device("cuda"))
