"""One process per GPU over torch.distributed (RCCL on ROCm, gloo for CPU tests).

The only collectives on the hot path: one flat gradient
all-reduce per minibatch (ppo.FlatGrads) and one 2-float (pos, count)
all-reduce for the belief-loss denominator; parameters are broadcast from
rank 0 once. Envs are sharded as contiguous blocks of the global env list,
so per-env RNG streams do not depend on the world size.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    group: Optional[object] = None  # None when world == 1

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def init_from_env(backend: Optional[str] = None) -> DistInfo:
    """Reads RANK/WORLD_SIZE/LOCAL_RANK (torchrun); no-op for a single process."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return DistInfo()
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if not dist.is_initialized():
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return DistInfo(rank=rank, world=world, local_rank=local, group=dist.group.WORLD)


def broadcast_module(module: torch.nn.Module, info: DistInfo) -> None:
    if info.world > 1:
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src=0, group=info.group)
