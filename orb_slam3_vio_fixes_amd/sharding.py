"""Multi-GPU sharding of the hot path.

One process per GPU.  Frames (or keyframe-map shards) are split into
contiguous ranges; nothing in the data path is reduced across GPUs.  The only
collectives are a one-time broadcast of the vocabulary (and, for map-wide BoW
search, of the query frame) from rank 0, done with torch.distributed
(RCCL/"nccl" on GPU tensors, or gloo on CPU tensors in tests).
"""
from __future__ import annotations

import numpy as np


def shard(n: int, rank: int, world: int) -> range:
    """Contiguous block of [0, n) owned by `rank` (sizes differ by <= 1)."""
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def _bcast_array(a: np.ndarray | None, src: int, device, rank: int):
    import torch
    import torch.distributed as dist
    meta = torch.zeros(8, dtype=torch.int64, device=device)
    if rank == src:
        raw = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
        meta[0] = raw.size
        meta[1] = {np.dtype(np.uint8): 0, np.dtype(np.int32): 1, np.dtype(np.float64): 2,
                   np.dtype(np.float32): 3, np.dtype(np.uint32): 4}[np.dtype(a.dtype)]
        meta[2:2 + a.ndim] = torch.tensor(a.shape, dtype=torch.int64)
        meta[7] = a.ndim
    dist.broadcast(meta, src)
    m = meta.cpu().numpy()
    dt = [np.uint8, np.int32, np.float64, np.float32, np.uint32][int(m[1])]
    buf = torch.empty(int(m[0]), dtype=torch.uint8, device=device)
    if rank == src:
        buf.copy_(torch.from_numpy(raw))
    dist.broadcast(buf, src)
    shape = tuple(int(x) for x in m[2:2 + int(m[7])])
    return buf.cpu().numpy().view(dt).reshape(shape)


def broadcast_vocabulary(voc: dict | None, src: int = 0, device="cpu") -> dict:
    """Broadcast a vocabulary dict (synth.vocabulary layout) from `src` to all
    ranks; the only collective of the path."""
    import torch.distributed as dist
    rank = dist.get_rank()
    out = {}
    for key in ("first_child", "nchild", "node_desc", "word_id", "weight"):
        out[key] = _bcast_array(voc[key] if rank == src else None, src, device, rank)
    has_ci = _bcast_array(np.array([int(voc.get("child_idx") is not None)], np.int32) if rank == src else None,
                          src, device, rank)
    out["child_idx"] = _bcast_array(voc["child_idx"] if rank == src else None, src, device, rank) if has_ci[0] \
        else None
    out["nnodes"] = len(out["nchild"])
    dims = _bcast_array(np.array([voc["depth_levels"]], np.int32) if rank == src else None, src, device, rank)
    out["depth_levels"] = int(dims[0])
    return out


def broadcast_frame(kps: np.ndarray | None, desc: np.ndarray | None, src: int = 0, device="cpu"):
    """Per-query broadcast of a frame's keypoints (raw 28-B records) and descriptors."""
    import torch.distributed as dist
    from .abi import KEYPOINT_DTYPE
    rank = dist.get_rank()
    k = _bcast_array(kps.view(np.uint8).reshape(-1, 28) if rank == src else None, src, device, rank)
    d = _bcast_array(desc if rank == src else None, src, device, rank)
    return np.ascontiguousarray(k).view(KEYPOINT_DTYPE).reshape(-1), d
