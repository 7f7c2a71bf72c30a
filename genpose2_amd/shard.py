"""Object sharding across GPUs (one process per GPU).

Objects are independent on the path except for two batch-wide scalars the reference computes
per call (F3): the PC sampler's mean score norm and RK45's error norm. The default semantics
are those of the reference called on each shard's sub-batch (the same batch-composition
dependence the reference has with --batch_size), so the data path needs no collective. The
one-time exchange is the packed-weight broadcast from rank 0 over RCCL (gloo on CPU tests).
"""
from __future__ import annotations

from typing import Iterable, Tuple

import torch


def shard_range(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block of ceil(total/world) objects for ``rank`` (last shard may be short)."""
    per = -(-total // world)
    lo = min(total, rank * per)
    return lo, min(total, lo + per)


def broadcast_tensors(tensors: Iterable[torch.Tensor], src: int = 0) -> None:
    import torch.distributed as dist
    for t in tensors:
        dist.broadcast(t, src=src)


def model_tensors(agent) -> list:
    """Device tensors holding an agent's packed weights, in a fixed order."""
    out = []
    if getattr(agent, "encoder", None) is not None:
        out.append(agent.encoder.wbuf)
        out += [agent.heads.up.t[k] for k in sorted(agent.heads.up.t)]
    if getattr(agent, "scale", None) is not None:
        out += [agent.scale.up.t[k] for k in sorted(agent.scale.up.t)]
    return out
