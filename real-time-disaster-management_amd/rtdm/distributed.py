"""Frame-sharded data parallelism over ranks (one process per GPU).

The hot path partitions cleanly: frames are independent and nothing carries
state across frames (BN in eval), so each rank runs the full two-stage pipeline
on its own contiguous shard of the global frame batch — no collective on the
data path.  Collectives exist only at the edges:
  * broadcast_array: rank 0's weights to every rank once at start (RCCL
    broadcast over xGMI when the group backend is 'nccl'; the reference's
    nn.DataParallel re-broadcasts all weights on every forward, yolov3/test.py:42-43);
  * gather_records: per batch, each rank's flat output record (logits, probs,
    detections padded to max_det, indices, counts) to rank 0 in one gather (the
    DataParallel gather of io, yolov3/test.py:42-43, but of the post-NMS results);
    gather_results does the same field by field.
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


def gather_records(record: torch.Tensor, out: torch.Tensor | None = None, dst: int = 0):
    """One collective per batch: every rank's flat output record (TwoStagePipeline.record:
    logits, probs, detections, indices and counts of its frame shard) lands in row r of
    `out` [world, record.numel()] on `dst` (RCCL over xGMI with the 'nccl' backend: each rank
    sends on its own link to dst; a gather of ~77 KB per rank at b8 is latency-bound, so
    one message instead of one per field).  Ranks hold equal shard sizes.  Returns `out`
    on dst, None elsewhere."""
    rank = dist.get_rank()
    world = dist.get_world_size()
    flat = record.reshape(-1)
    if rank == dst:
        if out is None:
            out = torch.empty((world, flat.numel()), dtype=flat.dtype, device=flat.device)
        dist.gather(flat, list(out.unbind(0)), dst=dst)
        return out
    dist.gather(flat, None, dst=dst)
    return None


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
