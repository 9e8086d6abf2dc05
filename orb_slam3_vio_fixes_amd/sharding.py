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


_DTYPES = [np.uint8, np.int32, np.float64, np.float32, np.uint32]


def _bcast_tensor(a: np.ndarray | None, src: int, device, rank: int):
    """Broadcast an array from `src`; every rank gets a torch tensor of the
    same dtype and shape ON `device` (RCCL on GPU tensors, gloo on CPU ones).
    Nothing is copied back to the host."""
    import torch
    import torch.distributed as dist
    meta = torch.zeros(8, dtype=torch.int64, device=device)
    if rank == src:
        a = np.ascontiguousarray(a)
        meta[0] = a.nbytes
        meta[1] = [np.dtype(t) for t in _DTYPES].index(np.dtype(a.dtype))
        meta[2:2 + a.ndim] = torch.tensor(a.shape, dtype=torch.int64)
        meta[7] = a.ndim
    dist.broadcast(meta, src)
    m = meta.cpu().tolist()                  # 8 integers of metadata
    tdt = {np.uint8: torch.uint8, np.int32: torch.int32, np.float64: torch.float64, np.float32: torch.float32,
           np.uint32: torch.int32}[_DTYPES[int(m[1])]]
    shape = tuple(int(x) for x in m[2:2 + int(m[7])])
    buf = torch.empty(shape, dtype=tdt, device=device)
    if rank == src:
        buf.copy_(torch.from_numpy(a.view(np.int32) if a.dtype == np.uint32 else a))
    dist.broadcast(buf, src)
    return buf


def broadcast_vocabulary(voc: dict | None, src: int = 0, device="cpu") -> dict:
    """Broadcast a vocabulary dict (synth.vocabulary layout) from `src` to all
    ranks, once; the arrays stay as tensors on `device` (HBM for GPU ranks:
    orbv_transform_device descends it there).  The only collective of the
    path besides the per-query frame broadcast."""
    import torch.distributed as dist
    rank = dist.get_rank()
    out = {}
    for key in ("first_child", "nchild", "node_desc", "word_id", "weight"):
        out[key] = _bcast_tensor(voc[key] if rank == src else None, src, device, rank)
    hdr = np.array([int(voc.get("child_idx") is not None), int(voc["depth_levels"])], np.int32) if rank == src else None
    h = _bcast_tensor(hdr, src, device, rank).cpu().tolist()
    out["child_idx"] = _bcast_tensor(np.ascontiguousarray(voc["child_idx"], np.int32) if rank == src else None,
                                     src, device, rank) if h[0] else None
    out["nnodes"] = int(out["nchild"].shape[0])
    out["depth_levels"] = int(h[1])
    return out


def vocab_device_struct(v: dict):
    """orbv_vocab over the broadcast tensors (device pointers; keeps them alive)."""
    from . import abi
    keep = [v[k] for k in ("first_child", "nchild", "node_desc", "word_id", "weight")]
    ci = v.get("child_idx")
    s = abi.OrbvVocab(int(v["nnodes"]), int(v["depth_levels"]), *[t.data_ptr() for t in keep],
                      ci.data_ptr() if ci is not None else None)
    return abi.Keep(s, keep + ([ci] if ci is not None else []))


def broadcast_frame(kps: np.ndarray | None, desc: np.ndarray | None, src: int = 0, device="cpu"):
    """Per-query broadcast of a frame's keypoints (raw 28-B records) and
    descriptors; tensors on `device` ([n, 28] uint8 and [n, 32] uint8)."""
    import torch.distributed as dist
    rank = dist.get_rank()
    k = _bcast_tensor(kps.view(np.uint8).reshape(-1, 28) if rank == src else None, src, device, rank)
    d = _bcast_tensor(desc if rank == src else None, src, device, rank)
    return k, d


def keypoints_host(k) -> np.ndarray:
    """Broadcast keypoint records ([n, 28] uint8 tensor) as the 28-B structured array."""
    from .abi import KEYPOINT_DTYPE
    return np.ascontiguousarray(k.cpu().numpy()).view(KEYPOINT_DTYPE).reshape(-1)
