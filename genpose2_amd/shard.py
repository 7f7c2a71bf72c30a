"""Object sharding across GPUs (one process per GPU).

Objects are independent on the path except for two batch-wide scalars the reference computes
per call (F3): the PC sampler's mean score norm and RK45's error norm. The default semantics
are those of the reference called on each shard's sub-batch (the same batch-composition
dependence the reference has with --batch_size), so the data path needs no collective. The
exchanges are:

* once: the packed weights of every agent, broadcast from rank 0 (RCCL over xGMI; gloo on CPU);
* per evaluated batch: the per-object outputs (pred_pose, energy, aggregated 4x4, lengths;
  about 4.5 MB at config 4) gathered to rank 0 or to every rank -- one all_gather per output
  tensor, off the timed sampling loop;
* optional global-batch PC sampling (``GlobalBatch``): the shards together reproduce ONE
  reference call on the whole batch -- the Langevin grad_norm averages every shard's rows -- at the
  cost of one all-gather of the per-workgroup score-norm partials per step (a few hundred bytes,
  latency-bound).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Tuple

import numpy as np
import torch


def shard_range(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block of ceil(total/world) objects for ``rank`` (last shards may be short or empty)."""
    per = -(-total // world)
    lo = min(total, rank * per)
    return lo, min(total, lo + per)


@dataclass
class GlobalBatch:
    """This rank's block of one global-batch call: objects [lo, hi) of ``total`` (shard_range), at most
    ``per_max`` objects per shard, over the ranks of ``group`` (None: the default group)."""
    total: int
    lo: int
    hi: int
    per_max: int
    rank: int
    world: int
    group: object = None

    @staticmethod
    def of(total: int, group=None) -> "GlobalBatch":
        import torch.distributed as dist
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        lo, hi = shard_range(total, world, rank)
        if hi <= lo:
            raise ValueError(f"global-batch sampling needs every shard non-empty ({total} objects over {world} ranks)")
        return GlobalBatch(total, lo, hi, -(-total // world), rank, world, group)


class PartialsExchange:
    """The exchange callback of gp_pc_sample_global (``part``: 2 slots of ``n`` fp32 partials, slot
    ``step & 1``) and of gp_ode_auto_attempt_global (``part``: one slot of ``n`` fp64 partials), ``n / world``
    entries per shard: after each scoring launch (PC step, RK45 attempt), every shard's chunk of the slot the
    launch wrote reaches every rank before the next launch reads it. RCCL: an all-gather enqueued behind the
    launch on the current stream (torch orders the next launch after it). gloo: through host copies (tests)."""

    def __init__(self, part: torch.Tensor, n: int, gb: GlobalBatch):
        import torch.distributed as dist
        from . import _lib
        self.part, self.n, self.gb = part, n, gb
        self.slots = part.numel() // n
        if self.slots not in (1, 2) or part.numel() != self.slots * n or n % gb.world:
            raise ValueError(f"partials exchange: {part.numel()} entries for slots of {n} over {gb.world} shards")
        self.per = n // gb.world
        self.nccl = dist.get_backend(gb.group) == "nccl"
        self.chunk = torch.empty(self.per, dtype=part.dtype, device=part.device)
        self.error: Optional[BaseException] = None
        self.fn = _lib.PC_EXCHANGE_FN(self._call)   # kept alive with the object

    def slot(self, step: int) -> torch.Tensor:
        base = (step & 1) * self.n if self.slots == 2 else 0
        return self.part[base:base + self.n]

    def _call(self, ctx, step, slot_ptr, n, stream) -> int:
        import torch.distributed as dist
        try:
            slot = self.slot(step)
            assert n == self.n and slot_ptr == slot.data_ptr(), "exchange: unexpected partials slot"
            mine = slot[self.gb.rank * self.per:(self.gb.rank + 1) * self.per]
            if self.nccl:
                self.chunk.copy_(mine)
                dist.all_gather_into_tensor(slot, self.chunk, group=self.gb.group)
            else:
                got = [torch.empty(self.per, dtype=slot.dtype) for _ in range(self.gb.world)]
                dist.all_gather(got, mine.cpu(), group=self.gb.group)
                slot.copy_(torch.cat(got).to(slot.device))
            return 0
        except BaseException as e:   # noqa: BLE001 -- reported through the C return code, re-raised by the caller
            self.error = e
            return -1


def gather_shard_rows(local: torch.Tensor, gb: GlobalBatch, k: int) -> torch.Tensor:
    """The whole batch's (total * k, ...) rows from every rank's (hi - lo) * k rows of ``local``, in object
    order, on local's device: an all-gather of per_max-object chunks (the last shard zero-padded), then the
    padding dropped. RCCL on device tensors; gloo through host copies."""
    import torch.distributed as dist
    rows = (gb.hi - gb.lo) * k
    if local.shape[0] != rows:
        raise ValueError(f"gather_shard_rows: {local.shape[0]} rows for objects [{gb.lo}, {gb.hi}) x {k}")
    per = gb.per_max * k
    tail = tuple(local.shape[1:])
    nccl = dist.get_backend(gb.group) == "nccl"
    buf = torch.zeros((per,) + tail, dtype=local.dtype, device=local.device if nccl else "cpu")
    buf[:rows].copy_(local)
    if nccl:
        full = torch.empty((gb.world * per,) + tail, dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(full, buf, group=gb.group)
        chunks = full.view((gb.world, per) + tail)
    else:
        got = [torch.empty_like(buf) for _ in range(gb.world)]
        dist.all_gather(got, buf, group=gb.group)
        chunks = torch.stack(got)
    parts = []
    for r in range(gb.world):
        lo, hi = shard_range(gb.total, gb.world, r)
        parts.append(chunks[r, :(hi - lo) * k])
    return torch.cat(parts).to(local.device)


def broadcast_tensors(tensors: Iterable[torch.Tensor], src: int = 0) -> None:
    import torch.distributed as dist
    for t in tensors:
        dist.broadcast(t, src=src)


def broadcast_packed(tensors: Iterable[torch.Tensor], tables: Iterable[np.ndarray], src: int = 0,
                     device: Optional[torch.device] = None) -> List[np.ndarray]:
    """Broadcast an agent's packed buffers AND its host layer tables from ``src``; returns the tables
    as received. The tables hold the split-f16 exponents the encoder kernels read from the host
    (pack.split_exponent of the weight values), so a rank that broadcast only the buffers would keep
    exponents of its own initial weights and scale its levels wrongly. ``device``: where the table
    travels (the buffers' device under RCCL; CPU under gloo)."""
    import torch.distributed as dist
    broadcast_tensors(tensors, src)
    out = []
    for tab in tables:
        t = torch.from_numpy(np.ascontiguousarray(tab).copy())
        if device is not None:
            t = t.to(device)
        dist.broadcast(t, src=src)
        out.append(t.cpu().numpy().reshape(np.shape(tab)))
    return out


def model_tables(agent) -> List[np.ndarray]:
    """Host-side weight-derived state of an agent (the encoder's layer table), in a fixed order --
    the same order as ``packed_host_tables``."""
    enc = getattr(agent, "encoder", None)
    out = [enc.table] if enc is not None else []
    img = getattr(agent, "img_encoder", None) if getattr(agent, "pointwise", False) else None
    if img is not None:
        out.append(img.table)          # ImgEncoder host scalars (layer_attn.2 bias, the two branch gates)
    return out


def broadcast_agent(agent, src: int = 0) -> None:
    """Make every rank's agent hold ``src``'s weights: the device buffers (``model_tensors``) and the
    host layer tables (``model_tables``), then drop caches derived from the old weights. Call it
    after construction and again after ``load_ckpt`` on ``src``."""
    dev_ = agent.device if agent.device.type == "cuda" else None
    if dev_ is not None:
        # and every write into them (a checkpoint's upload on src, on whatever stream) has landed before
        # the collective copies them out
        torch.cuda.synchronize(dev_)
    tabs = broadcast_packed(model_tensors(agent), model_tables(agent), src, dev_)
    if tabs:
        agent.encoder.set_table(tabs[0])
    if len(tabs) > 1:
        agent.img_encoder.set_table(tabs[1])
    agent._pc_cache = {}
    if dev_ is not None:
        # one-time: every copy the collective made into (or out of) the weight buffers has landed
        # before any kernel of any stream reads them (gloo moves CUDA tensors on its own streams)
        torch.cuda.synchronize(dev_)


def packed_host_tables(kind: str, sd) -> List[np.ndarray]:
    """Host tables ``model_tables`` holds for an agent of ``kind`` built from ``sd``."""
    from . import pack
    if kind == "scale":
        return []
    if kind.endswith("_pointwise"):
        from . import arch
        from .img_encoder import pack_img_scalars
        return [pack.pack_encoder(sd, arch.fus_sa_branches())[1], pack_img_scalars(sd)]
    return [pack.pack_encoder(sd)[1]]


def model_tensors(agent) -> List[torch.Tensor]:
    """Device tensors holding an agent's packed weights, in a fixed order: the encoder buffer, then
    the head (or ScaleNet) buffers by name -- the same order as ``packed_host_tensors``."""
    out = []
    if getattr(agent, "encoder", None) is not None:
        out.append(agent.encoder.wbuf)
        if hasattr(agent.encoder, "t"):      # fused encoder (--dino pointwise): transformer / fusion blocks
            out += [agent.encoder.t[k] for k in sorted(agent.encoder.t)]
            out += [agent.img_encoder.t[k] for k in sorted(agent.img_encoder.t)]   # and the ImgEncoder
        out += [agent.heads.up.t[k] for k in sorted(agent.heads.up.t)]
    if getattr(agent, "scale", None) is not None:
        out += [agent.scale.up.t[k] for k in sorted(agent.scale.up.t)]
    return out


def packed_host_tensors(kind: str, sd) -> List[torch.Tensor]:
    """Host (CPU) tensors of exactly the buffers ``model_tensors`` holds on the device for an agent of
    ``kind`` built from state dict ``sd`` (genpose2_amd.pack), in the same order."""
    from . import pack
    if kind == "scale":
        p = pack.pack_scale(sd)
        return [torch.from_numpy(np.ascontiguousarray(p[k])) for k in sorted(p)]
    p = pack.pack_heads(sd)
    if kind.endswith("_pointwise"):
        from . import arch
        from .fus_encoder import pack_fus_blocks
        from .img_encoder import pack_img_encoder
        f = pack_fus_blocks(sd)
        im = pack_img_encoder(sd)
        enc = [torch.from_numpy(pack.pack_encoder(sd, arch.fus_sa_branches())[0])] + \
            [torch.from_numpy(f[k]) for k in sorted(f)] + [torch.from_numpy(im[k]) for k in sorted(im)]
    else:
        enc = [torch.from_numpy(pack.pack_encoder(sd)[0])]
    return enc + [torch.from_numpy(np.ascontiguousarray(p[k])) for k in sorted(p)]


def gather_outputs(outputs: Dict[str, Optional[torch.Tensor]], total: int, dst: Optional[int] = None
                   ) -> Optional[Dict[str, Optional[torch.Tensor]]]:
    """Reassemble per-object outputs sharded by ``shard_range``: every tensor's dim 0 is this rank's
    objects. Each tensor is padded to ceil(total/world) rows and all-gathered; the result (rows in
    object order, the padding dropped) is returned on every rank (dst=None) or on rank ``dst`` only
    (other ranks get None). None entries stay None. Works on RCCL (device tensors) and gloo (CPU)."""
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    per = -(-total // world)
    lo, hi = shard_range(total, world, rank)
    res: Dict[str, Optional[torch.Tensor]] = {}
    for name in sorted(outputs):
        t = outputs[name]
        if t is None:
            res[name] = None
            continue
        if t.shape[0] != hi - lo:
            raise ValueError(f"{name}: {t.shape[0]} rows on rank {rank}, shard holds {hi - lo} objects")
        buf = torch.zeros((per,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        buf[: hi - lo] = t
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf.contiguous())
        rows = [parts[r][: shard_range(total, world, r)[1] - shard_range(total, world, r)[0]] for r in range(world)]
        res[name] = torch.cat(rows, 0)
    if dst is not None and rank != dst:
        return None
    return res
