"""toued — MI355X-native hot path of nmonette/TO-UED (GROOVE / LPG / TA-LPG).

Python host mirroring the reference's operator interfaces (gymnax GridWorld,
RolloutWrapper, LevelSampler, make_lpg_train_step, train.py flags) over the C
ABI of libtoued_hip.so (include/toued.h).  PyTorch provides device memory,
streams and torch.distributed; the computation is in the HIP kernels.
"""
from ._lib import ToUEDError, lib  # noqa: F401


def __getattr__(name):
    # the reference's meta/meta.py entry points, imported lazily (they pull in torch and the rollout machinery)
    if name in ("create_lpg_train_state", "make_lpg_train_step", "LpgTrainState", "ValueCriticStates"):
        from . import meta
        return getattr(meta, name)
    raise AttributeError(name)


__all__ = ["ToUEDError", "lib", "create_lpg_train_state", "make_lpg_train_step", "LpgTrainState",
           "ValueCriticStates"]
