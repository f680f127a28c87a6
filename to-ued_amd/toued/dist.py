"""One process per GPU over torch.distributed (RCCL on ROCm, gloo on CPU).

The agent axis is the only parallel axis: rank r owns agents
[r*N/world, (r+1)*N/world).  Every rank derives all N per-agent keys and keeps
its slice, so trajectories are identical at any world size.  The only
data-path collective is one all-reduce(SUM) of the flat LPG meta-gradient
(~0.8 MB) per outer step; the level sampler gathers per-agent scores.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class World:
    rank: int = 0
    size: int = 1
    local_rank: int = 0
    backend: str = ""

    @property
    def active(self) -> bool:
        return self.size > 1 and dist.is_available() and dist.is_initialized()

    def _staged(self, t: torch.Tensor) -> bool:
        # gloo (CPU tests, or several ranks sharing one GPU) moves device tensors through the host
        return self.backend == "gloo" and t.is_cuda

    def all_reduce_sum(self, t: torch.Tensor):
        if self.active:
            if self._staged(t):
                h = t.cpu()
                dist.all_reduce(h, op=dist.ReduceOp.SUM)
                t.copy_(h)
            else:
                dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t

    def all_gather_cat(self, t: torch.Tensor) -> torch.Tensor:
        if not self.active:
            return t
        src = t.contiguous().cpu() if self._staged(t) else t.contiguous()
        parts = [torch.empty_like(src) for _ in range(self.size)]
        dist.all_gather(parts, src)
        out = torch.cat(parts, dim=0)
        return out.to(t.device) if self._staged(t) else out

    def barrier(self):
        if self.active:
            dist.barrier()

    def agent_slice(self, n_total: int):
        if n_total % self.size:
            raise ValueError(f"num_agents={n_total} must divide evenly over {self.size} ranks")
        per = n_total // self.size
        return self.rank * per, (self.rank + 1) * per, n_total


def init_from_env(backend: str | None = None) -> World:
    """Initialise from torchrun's RANK/WORLD_SIZE/LOCAL_RANK (single process if absent)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1:
        return World()
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if backend is None:
        backend = os.environ.get("TOUED_DIST_BACKEND") or ("nccl" if torch.cuda.device_count() > 0 else "gloo")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and local >= ndev:
        # RCCL needs one device per rank: fail here with the cause instead of inside RCCL's communicator init
        raise RuntimeError(f"backend nccl (RCCL): local rank {local} has no GPU of its own ({ndev} visible); "
                           f"run at most {ndev} ranks per node, or TOUED_DIST_BACKEND=gloo to share devices")
    if ndev > 0:
        # one GPU per rank; ranks beyond the device count share devices (gloo only)
        torch.cuda.set_device(local % ndev)
    if not dist.is_initialized():
        dist.init_process_group(backend=backend)
    return World(rank, ws, local, backend)
