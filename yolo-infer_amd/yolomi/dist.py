"""Multi-GPU plumbing for batch-sharded inference.

One process per GPU.  At init rank 0 packs the model blob (BN-folded, NHWC packed weights + plan) and broadcasts it
over RCCL (xGMI) through the C-ABI (`rccl_broadcast_model` → ym_broadcast_weights; `broadcast_blob` is the same
exchange as one torch.distributed uint8 tensor, used by the gloo CPU tests).  Per batch,
rank r runs images [r*B_local, (r+1)*B_local) of the global batch on its own stream/graph; the only exchange is one
fp32 all-reduce (MAX) so that LoadTensor's /255 rule — a whole-batch decision in the reference — is taken over the
global batch, not per shard (`GlobalBatchMax`).  The reference itself is single-device for inference
(/root/reference/core/model.py:111-112).
"""
from __future__ import annotations

import hashlib
from typing import Optional, Tuple

import torch
import torch.distributed as dist


def broadcast_blob(blob: Optional[bytes], device: torch.device, src: int = 0) -> bytes:
    """Rank `src` passes its blob, the others None; everyone returns the same bytes."""
    rank = dist.get_rank()
    if rank == src:
        if blob is None:
            raise ValueError("source rank must provide the blob")
        n = torch.tensor([len(blob)], dtype=torch.int64, device=device)
    else:
        n = torch.zeros(1, dtype=torch.int64, device=device)
    dist.broadcast(n, src)
    if rank == src:
        buf = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(device)
    else:
        buf = torch.empty(int(n.item()), dtype=torch.uint8, device=device)
    dist.broadcast(buf, src)
    return blob if rank == src else bytes(buf.cpu().numpy())


def rccl_broadcast_model(make_model, blob: Optional[bytes], device: torch.device, root: int = 0):
    """The C-ABI path of the init-time weight broadcast (include/yolomi.h ym_broadcast_weights): the root's packed
    blob goes to every rank over RCCL (xGMI) straight into each rank's context.  The RCCL unique id travels over the
    default torch.distributed group; `make_model(**kw)` builds the rank's YOLO11Model (root: weights_blob=blob,
    others: weights_from=(comm, root)).  Collective: every rank calls it."""
    from . import lib as L
    rank, world = dist.get_rank(), dist.get_world_size()
    if rank == root and blob is None:
        raise ValueError("the root rank must provide the blob")
    uid = [L.rccl_unique_id() if rank == root else None]
    dist.broadcast_object_list(uid, src=root)
    comm = L.rccl_comm_init(device.index if device.index is not None else torch.cuda.current_device(), world, uid[0],
                            rank)
    try:
        if rank == root:
            model = make_model(weights_blob=blob)
            model.model.engine.broadcast_weights(comm, root)
        else:
            model = make_model(weights_from=(comm, root))
        torch.cuda.synchronize(device)
    finally:
        L.rccl_comm_destroy(comm)
    return model


def shard(global_batch: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous shard [start, stop) of a global batch; sizes differ by at most one image."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, extra = divmod(global_batch, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


class GlobalBatchMax:
    """LoadTensor's statistic over the GLOBAL batch for a batch-sharded rank: the shard's max (the engine's
    `ym_input_max` kernel) all-reduced with MAX over the process group, left in one persistent device float that
    `Engine.run(batch_max=...)` hands to the forward (stream-ordered: no host synchronisation).  `local_max` may be
    replaced (tests drive it on CPU with gloo)."""

    def __init__(self, engine=None, device: Optional[torch.device] = None, group=None):
        self.engine = engine
        self.group = group
        dev = device if device is not None else (engine.device if engine is not None else torch.device("cpu"))
        self.buf = torch.empty((1,), dtype=torch.float32, device=dev)

    def local_max(self, x: torch.Tensor) -> torch.Tensor:
        return self.engine.input_max(x, out=self.buf)

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        self.local_max(x)
        if dist.is_initialized() and dist.get_world_size(self.group) > 1:
            dist.all_reduce(self.buf, op=dist.ReduceOp.MAX, group=self.group)
        return self.buf


def enable_global_rule(model, group=None) -> GlobalBatchMax:
    """Make `model.predict` take the /255 decision over the global batch of this process group."""
    rule = GlobalBatchMax(model.model.engine, group=group)
    model.global_batch_max = rule
    return rule


def digest(blob: bytes) -> str:
    return hashlib.sha256(blob).hexdigest()
