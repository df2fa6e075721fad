"""Frame-sharded data parallelism over ranks (one process per GPU).

The hot path partitions cleanly: frames are independent and nothing carries
state across frames (BN in eval), so each rank runs the full two-stage pipeline
on its own contiguous shard of the global frame batch — no collective on the
data path.  Collectives exist only at the edges:
  * broadcast_array: rank 0's weights to every rank once at start (RCCL
    broadcast over xGMI when the group backend is 'nccl'; the reference's
    nn.DataParallel re-broadcasts all weights on every forward, yolov3/test.py:42-43);
  * gather_results: optional collection of fixed-size per-frame records
    (logits, detections padded to max_det, counts) on rank 0 (the DataParallel
    gather), for callers that need every result in one process.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def shard_range(global_batch: int, world: int, rank: int):
    """Contiguous shard of frames [start, start+count) for `rank`."""
    base, rem = divmod(global_batch, world)
    count = base + (1 if rank < rem else 0)
    start = rank * base + min(rank, rem)
    return start, count


def broadcast_array(arr, src: int = 0, device=None) -> np.ndarray:
    """Broadcast a float32 numpy array from `src` (other ranks pass None)."""
    rank = dist.get_rank()
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
    n = torch.tensor([arr.size if rank == src else 0], dtype=torch.int64, device=device)
    dist.broadcast(n, src)
    t = torch.from_numpy(np.ascontiguousarray(arr, np.float32)).to(device) if rank == src else \
        torch.empty(int(n.item()), dtype=torch.float32, device=device)
    dist.broadcast(t, src)
    return t.cpu().numpy()


def broadcast_state_dict(sd, shapes: dict, src: int = 0, device=None) -> dict:
    keys = sorted(shapes)
    flat = np.concatenate([np.asarray(sd[k], np.float32).reshape(-1) for k in keys]) if dist.get_rank() == src \
        else None
    flat = broadcast_array(flat, src, device)
    out, o = {}, 0
    for k in keys:
        c = int(np.prod(shapes[k]))
        out[k] = flat[o:o + c].reshape(shapes[k])
        o += c
    return out


def gather_results(tensors: dict, dst: int = 0):
    """Gather equally shaped per-rank tensors (e.g. logits [b,5], det [b,max_det,6],
    count [b]) to `dst`; returns {name: [world] list} on dst, None elsewhere.
    Ranks must hold the same shard size (pad the last shard)."""
    world = dist.get_world_size()
    rank = dist.get_rank()
    out = {} if rank == dst else None
    for k in sorted(tensors):
        t = tensors[k].contiguous()
        bufs = [torch.empty_like(t) for _ in range(world)] if rank == dst else None
        dist.gather(t, bufs, dst=dst)
        if rank == dst:
            out[k] = bufs
    return out
