"""ctypes binding of libtoued_hip.so (the C ABI declared in include/toued.h).

The product path has no CPU fallback: if the library is missing or a call
fails, ``ToUEDError`` is raised.  Device buffers are torch tensors; the
current torch HIP stream is passed to every call.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch

LIB_PATH = Path(os.environ.get("TOUED_LIB", Path(__file__).resolve().parent / "libtoued_hip.so"))


class ToUEDError(RuntimeError):
    pass


class EnvSpecC(ctypes.Structure):
    _fields_ = [("max_grid", ctypes.c_int), ("n_max", ctypes.c_int), ("n_types", ctypes.c_int),
                ("tabular", ctypes.c_int)]


_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_U = ctypes.c_uint32
_L = ctypes.c_long

# name -> argtypes (restype int unless listed in _RESTYPES)
_SIGS = {
    "toued_split": [_P, _I, _I, _P, _P],
    "toued_split_planar": [_P, _I, _I, _P, _P],
    "toued_fold_in": [_P, _I, _U, _P, _P],
    "toued_random_bits": [_P, _I, _I, _P, _P],
    "toued_uniform": [_P, _I, _I, _F, _F, _P, _P],
    "toued_normal": [_P, _I, _I, _P, _P],
    "toued_mode_program_bytes": [],
    "toued_level_gen": [_P, _P, _P, _P, _P, _I, _P],
    "toued_level_gen_masked": [_P, _P, _P, _P, _I, _P, _P],
    "toued_gw_reset": [EnvSpecC, _P, _I, _P, _P, _P, _P, _I, _P],
    "toued_gw_step": [EnvSpecC, _P, _I, _P, _P, _P, _P, _P, _P, _P, _I, _P],
    "toued_batch_reset": [EnvSpecC, _P, _P, _I, _I, _P, _P, _P, _P],
    "toued_batch_reset_masked": [EnvSpecC, _P, _P, _I, _I, _P, _P, _P, _P, _P],
    "toued_rollout": [EnvSpecC, _P, _P, _I, _P, _P, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P],
    "toued_eval_keys": [_P, _I, _I, _I, _P, _P],
    "toued_rollout_draws": [EnvSpecC, _P, _P, _I, _I, _I, _I, _P, _P, _P],
    "toued_rollout_env": [EnvSpecC, _P, _P, _I, _P, _I, _I, _I, _P, _L, _P, _P, _P, _P, _P, _P, _P],
    "toued_eval_draws": [EnvSpecC, _P, _I, _I, _I, _P, _P, _P],
    "toued_eval_returns": [EnvSpecC, _P, _P, _I, _P, _I, _I, _I, _P, _P, _P],
    "toued_meta_keys": [_P, _I, _I, _P, _P, _P, _P, _P],
    "toued_lpg_inputs": [_I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _L, _L, _L, _P],
    "toued_lpg_inputs_rows": [_I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _L, _L, _L,
                              _P],
    "toued_agent_grad": [_I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _F, _P, _P, _P, _P, _P, _P, _P],
    "toued_agent_apply": [_I, _I, _P, _P, _P, _P, _F, _F, _F, _P, _P, _P, _P, _P],
    "toued_entropy": [_I, _I, _I, _I, _P, _P, _P, _P, _P, _F, _F, _P, _P, _P],
    "toued_eval_loss": [_I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _F, _F, _P, _P, _P, _P],
    "toued_lpgloss_grad": [_I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P],
    "toued_clip_dot": [_I, _I, _P, _P, _P, _P, _P, _F, _F, _F, _P, _P],
    "toued_hvp": [_I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _F, _F, _F, _F, _F,
                  _P, _P, _P, _P, _P],
    "toued_embed_bwd": [_I, _I, _I, _I, _I, _P, _L, _I, _P, _L, _P, _P, _L, _P, _P, _L, _P, _P, _P, _P, _I, _P],
    "toued_init_tables": [_P, _I, _I, _I, _F, _F, _F, _P, _P],
    "toued_init_tables_masked": [_P, _I, _I, _I, _F, _F, _F, _P, _P, _P],
    "toued_adam": [_I, _P, _P, _P, _P, _F, _F, ctypes.c_double, ctypes.c_double, _F, _I, _P],
    "toued_gru_pack": [_P, _P, _I, _P, _P, _P],
    "toued_gru_packed_floats": [_I],
    "toued_gru_fwd": [_I, _I, _I, _I, _P, _L, _L, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _L, _P],
    "toued_gru_bwd": [_I, _I, _I, _I, _P, _L, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _L, _P, _P, _P, _P, _P,
                      _P, _P],
    "toued_gru_bwd_col_exp": [_I],
    "toued_gae": [_I, _I, _I, _P, _P, _P, _F, _F, _P, _P, _P],
    "toued_sort_keys2048": [_P, _P, _I, _I, _P],
    "toued_gru_bwd_fused_fits": [_I, _I],
    "toued_gru_bwd_fused_work_floats": [_I, _I],
    "toued_gru_bwd_fused": [_I, _I, _I, _I, _P, _L, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _L, _P, _P, _P, _P, _P,
                            _P, ctypes.c_size_t, _P],
    "toued_set_reserved_cus": [_I],
    "toued_wgrad_bfp_workspace_floats": [_I, _I, _L],
    "toued_wgrad_bfp": [_I, _I, _L, _P, _L, _I, _P, _L, _P, _P, _P, ctypes.c_size_t, _P],
    "toued_wgrad_bfp_slab": [_I, _I, _L, _P, _L, _I, _P, _L, _I, _P, _P, _P, ctypes.c_size_t, _P],
    "toued_gru_slab_saves": [_I],
    "toued_gru_hin_slab": [],
    "toued_gru_bwd_small_work_floats": [_L],
    "toued_gru_bwd_small": [_L, _P, _P, _P, _P, _P, _P, ctypes.c_size_t, _P],
    "toued_choice_cdf": [_P, _P, _I, _I, _P, _P],
    "toued_key_chain": [_P, _I, _I, _P, _P],
    "toued_a2c_grad": [_I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _F, _F, _F, _P, _P, _P, _P],
    "toued_value_critic_update": [_I, _I, _I, _I, _P, _P, _P, _P, _P, _F, _F, _F, _F, _P, _P, _P],
    "toued_a2c_apply": [_I, _I, _P, _P, _P, _P, _F, _F, _F, _P, _P, _P],
    "toued_a2c_update_fits": [_I, _I, _I],
    "toued_a2c_update": [_I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _F, _F, _F, _F, _F, _F, _P, _P, _P, _P],
    "toued_agent_update_fits": [_I, _I, _I],
    "toued_agent_update": [_I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _F, _F, _F, _F, _P, _P, _P, _P, _P],
    "toued_agent_step": [_I, _I, _I, _I] + [_P] * 11 + [_F] * 4 + [_P] * 7,
    "toued_agent_step_entropy": [_I, _I, _I, _I] + [_P] * 11 + [_F] * 4 + [_P] * 7,
    "toued_gather_add": [_P, _P, _P, _P, _I, _P],
    "toued_sum_rows_add": [_P, _I, _I, _P, _P],
    "toued_sample_random_keys": [_P, _I, _I, _I, _P, _P, _P, _U, _P, _P, _P],
    "toued_entropy_clip_hvp": [_I] * 5 + [_P] * 9 + [_F] * 2 + [_P] * 5 + [_F] * 3 + [_P] + [_F] * 3 + [_P] * 3,
    "toued_meta_metrics": [_I, _I, _P, _F, _P, _F, _F, _F, _F, _P, _P],
    "toued_entropy_clip": [_I, _I, _I, _I, _P, _P, _P, _P, _F, _F, _P, _P, _P, _P, _P, _F, _F, _F, _P, _P],
    "toued_a2c_chain_fits": [_I, _I, _I],
    "toued_a2c_chain_self_fits": [_I, _I, _I],
    "toued_device_error_check": [_P, _I],
    "toued_sync_check": [],
    "toued_nonfinite_count": [_P, _L, _P, _P],
    "toued_nonfinite_count_2d": [_P, _L, _L, _L, _P, _P],
    "toued_dbg_wgrad_visits": [_P, _I],
    "toued_eval_returns_cus": [_I],
    "toued_dbg_wgrad_last_ntiles": [],
    "toued_a2c_chain": [EnvSpecC, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _L, _F, _F, _F, _F, _F, _F, _P, _P, _P],
    "toued_a2c_chain_self": [EnvSpecC, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _F, _F, _F, _F, _F, _F, _P, _P, _P],
    "toued_gru_pack_fwd_multi": [_P, _L, _I, _P, _I, _P, _P],
    "toued_gru_fwd_multi": [_I, _I, _I, _I, _I, _P, _L, _L, _P, _P, _P, _L, _P, _P, _P, _P],
    "toued_es_ask": [_P, _L, _L, _L, _L, _P, _F, _P, _P],
    "toued_es_grad": [_P, _P, _F, _P, _I, _L, _P, _P],
    "toued_es_opt": [_L, _I, _P, _P, _F, _P, _P, _F, _F, _F, _F, _F, _F, _P],
    "toued_plr_reset_ids": [_I, _I, _P, _P, _P, _P, _P],
    "toued_plr_sample": [_I, _I, _P, _P, _P, _P, _I, _F, _F, _P, _P, _P, _P, _P],
    "toued_wgrad_workspace_floats": [_I, _I, _L],
    "toued_wgrad": [_I, _I, _L, _P, _L, _P, _L, _P, _P, ctypes.c_size_t, _P],
    "toued_wgrad_ldc": [_I, _I, _L, _P, _L, _P, _L, _P, _I, _P, ctypes.c_size_t, _P],
    "toued_rowsum_workspace_floats": [_I, _L],
    "toued_rowsum_into": [_I, _L, _P, _L, _P, _I, _P, ctypes.c_size_t, _P],
    "toued_last_error": [],
    "toued_abi_version": [],
    "toued_ctx_create": [],
    "toued_ctx_destroy": [_P],
    "toued_ctx_set_current": [_P],
    "toued_ctx_current": [],
}
_RESTYPES = {"toued_last_error": ctypes.c_char_p, "toued_ctx_create": ctypes.c_void_p,
             "toued_ctx_current": ctypes.c_void_p, "toued_mode_program_bytes": ctypes.c_size_t,
             "toued_gru_packed_floats": ctypes.c_size_t, "toued_wgrad_workspace_floats": ctypes.c_size_t,
             "toued_gru_bwd_small_work_floats": ctypes.c_size_t, "toued_wgrad_bfp_workspace_floats": ctypes.c_size_t,
             "toued_rowsum_workspace_floats": ctypes.c_size_t,
             "toued_gru_bwd_fused_work_floats": ctypes.c_size_t}

_lib = None


def lib():
    """Load the library once (raises ToUEDError if it is absent)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise ToUEDError(f"libtoued_hip.so not found at {LIB_PATH}; run `python to-ued_amd/build.py` "
                             "(there is no CPU fallback for the hot path)")
        L = ctypes.CDLL(str(LIB_PATH))
        for name, args in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        _lib = L
    return _lib


def exported_symbols():
    return list(_SIGS)


def ptr(t) -> int | None:
    if t is None:
        return None
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"expected a tensor, got {type(t)}")
    if not t.is_contiguous():
        raise ToUEDError("toued: tensor arguments must be contiguous")
    return t.data_ptr()


def stream_ptr():
    return torch.cuda.current_stream().cuda_stream


# --debug (util/jax.py:12-14): every ABI call is followed by a device synchronise and an error check, so an
# asynchronous kernel fault is reported at the call that launched it (toued.debug.configure)
_DEBUG_SYNC = False


def _capturing() -> bool:
    try:
        return torch.cuda.is_current_stream_capturing()
    except RuntimeError:     # no device: nothing can be capturing
        return False


def set_debug_sync(on: bool) -> None:
    global _DEBUG_SYNC
    _DEBUG_SYNC = bool(on)


def call(name: str, *args):
    fn = getattr(lib(), name)
    rc = fn(*args)
    if rc != 0:
        msg = lib().toued_last_error().decode(errors="replace")
        raise ToUEDError(f"{name} failed ({rc}): {msg}")
    if _DEBUG_SYNC and not _capturing():   # (a captured graph is checked at replay)
        if lib().toued_sync_check() != 0:
            msg = lib().toued_last_error().decode(errors="replace")
            raise ToUEDError(f"{name}: {msg} (--debug: checked after the call)")
    return rc


def check_device_errors(wait: bool = False) -> None:
    """Raise ToUEDError if a kernel set the device error word (a bounded wait that expired, toued.h
    toued_device_error_check).  wait=False never blocks: it reports the previous call's read-back and enqueues a new
    one on the current stream; wait=True synchronises with the current stream first."""
    call("toued_device_error_check", stream_ptr(), int(bool(wait)))


def env_spec_c(spec) -> EnvSpecC:
    return EnvSpecC(spec.max_grid_size, spec.max_n_objs, spec.max_n_obj_types, int(spec.tabular))
