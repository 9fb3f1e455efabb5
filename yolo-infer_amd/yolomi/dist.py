"""Multi-GPU plumbing for batch-sharded inference.

One process per GPU.  The only collective on the path is at init: rank 0 packs the model blob (BN-folded, NHWC
packed weights + plan) and broadcasts it as ONE uint8 tensor (RCCL over xGMI on MI355X when the process group is
`nccl`; gloo on CPU for tests).  Per batch there is no exchange: rank r runs images [r*B_local, (r+1)*B_local) of
the global batch on its own stream/graph.  The reference itself is single-device for inference
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


def shard(global_batch: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous shard [start, stop) of a global batch; sizes differ by at most one image."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, extra = divmod(global_batch, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def digest(blob: bytes) -> str:
    return hashlib.sha256(blob).hexdigest()
