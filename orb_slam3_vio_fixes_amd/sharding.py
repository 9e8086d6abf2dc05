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
_VOCAB_KEYS = ("first_child", "nchild", "node_desc", "word_id", "weight", "child_idx")
_MAXDIM = 4


def _torch_dtype(code: int):
    import torch
    return {np.uint8: torch.uint8, np.int32: torch.int32, np.float64: torch.float64, np.float32: torch.float32,
            np.uint32: torch.int32}[_DTYPES[code]]


def _bcast_header(rows: list[list[int]] | None, nrows: int, src: int, device, rank: int) -> list[list[int]]:
    """ONE fixed-size int64 broadcast of `nrows` x 8 integers, read back to
    the host once: the metadata of everything that follows it."""
    import torch
    import torch.distributed as dist
    meta = torch.zeros((nrows, 8), dtype=torch.int64, device=device)
    if rank == src:
        meta.copy_(torch.tensor(rows, dtype=torch.int64))
    dist.broadcast(meta, src)
    return meta.cpu().tolist()


def _spec(a: np.ndarray | None) -> list[int]:
    """Header row of one array: present, dtype code, ndim, shape (<= 4 dims)."""
    if a is None:
        return [0] * 8
    a = np.asarray(a)
    assert a.ndim <= _MAXDIM, a.shape
    return [1, [np.dtype(t) for t in _DTYPES].index(a.dtype), a.ndim] + list(a.shape) + [0] * (_MAXDIM + 1 - a.ndim)


def _bcast_known(a: np.ndarray | None, spec: list[int], src: int, device, rank: int):
    """Broadcast one array whose header row every rank already holds: no
    metadata exchange and no host read."""
    import torch
    import torch.distributed as dist
    shape = tuple(int(x) for x in spec[3:3 + spec[2]])
    buf = torch.empty(shape, dtype=_torch_dtype(spec[1]), device=device)
    if rank == src:
        a = np.ascontiguousarray(a)
        buf.copy_(torch.from_numpy(a.view(np.int32) if a.dtype == np.uint32 else a))
    dist.broadcast(buf, src)
    return buf


def broadcast_vocabulary(voc: dict | None, src: int = 0, device="cpu") -> dict:
    """Broadcast a vocabulary dict (synth.vocabulary layout) from `src` to all
    ranks, once; the arrays stay as tensors on `device` (HBM for GPU ranks:
    orbv_transform_device descends it there).  One fixed-size header (every
    array's dtype and shape, the depth) is exchanged and read on the host
    once; the arrays follow with no further host round trip."""
    import torch.distributed as dist
    rank = dist.get_rank()
    rows = None
    if rank == src:
        arrs = {k: (None if voc.get(k) is None else np.ascontiguousarray(voc[k])) for k in _VOCAB_KEYS}
        if arrs["child_idx"] is not None:
            arrs["child_idx"] = arrs["child_idx"].astype(np.int32, copy=False)
        rows = [_spec(arrs[k]) for k in _VOCAB_KEYS] + [[int(voc["depth_levels"])] + [0] * 7]
    hdr = _bcast_header(rows, len(_VOCAB_KEYS) + 1, src, device, rank)
    out = {}
    for i, k in enumerate(_VOCAB_KEYS):
        out[k] = _bcast_known(arrs[k] if rank == src else None, hdr[i], src, device, rank) if hdr[i][0] else None
    out["nnodes"] = int(out["nchild"].shape[0])
    out["depth_levels"] = int(hdr[-1][0])
    return out


def vocab_device_struct(v: dict):
    """orbv_vocab over the broadcast tensors (device pointers; keeps them alive)."""
    from . import abi
    keep = [v[k] for k in ("first_child", "nchild", "node_desc", "word_id", "weight")]
    ci = v.get("child_idx")
    s = abi.OrbvVocab(int(v["nnodes"]), int(v["depth_levels"]), *[t.data_ptr() for t in keep],
                      ci.data_ptr() if ci is not None else None)
    return abi.Keep(s, keep + ([ci] if ci is not None else []))


class FrameChannel:
    """Per-query broadcast of a frame's keypoints (raw 28-B records) and
    descriptors from `src`.  The capacity is agreed once, when the channel is
    made; each query is then ONE broadcast of a fixed-size buffer
    [16-B header: n][cap x 28 keypoint bytes][cap x 32 descriptor bytes] and
    one 8-byte host read of n, which the caller needs anyway to size its
    launches (no per-array metadata exchange)."""

    def __init__(self, cap: int, src: int = 0, device="cpu"):
        import torch
        import torch.distributed as dist
        self.src, self.device, self.rank = src, device, dist.get_rank()
        c = torch.tensor([int(cap)], dtype=torch.int64, device=device)
        dist.broadcast(c, src)
        self.cap = int(c.cpu().item())
        self.buf = torch.zeros(16 + self.cap * 60, dtype=torch.uint8, device=device)
        self._host = np.zeros(16 + self.cap * 60, np.uint8) if self.rank == src else None

    def broadcast(self, kps: np.ndarray | None, desc: np.ndarray | None):
        """([n, 28] uint8, [n, 32] uint8) tensors on the channel's device.

        The returned tensors are views into the channel's one persistent
        buffer: they are valid until the next broadcast, which overwrites them
        in place (on the current stream).  A caller that keeps a frame past
        that, or reads it on another stream, must ``.clone()`` it first."""
        import torch
        import torch.distributed as dist
        cap = self.cap
        if self.rank == self.src:
            kb = np.ascontiguousarray(kps).view(np.uint8).reshape(-1, 28)
            n = len(kb)
            if n > cap:
                raise ValueError(f"frame of {n} keypoints exceeds the channel capacity {cap}")
            h = self._host
            h[:8] = np.array([n], np.int64).view(np.uint8)
            h[16:16 + n * 28] = kb.reshape(-1)
            h[16 + cap * 28:16 + cap * 28 + n * 32] = np.ascontiguousarray(desc, np.uint8).reshape(-1)
            self.buf.copy_(torch.from_numpy(h))
        dist.broadcast(self.buf, self.src)
        n = int(self.buf[:8].view(torch.int64).cpu().item())
        k = self.buf[16:16 + n * 28].view(n, 28)
        d = self.buf[16 + cap * 28:16 + cap * 28 + n * 32].view(n, 32)
        return k, d


def broadcast_frame(kps: np.ndarray | None, desc: np.ndarray | None, src: int = 0, device="cpu", cap: int = 0):
    """One-off form of FrameChannel (capacity from `cap`, or the sender's
    keypoint count): tensors on `device` ([n, 28] uint8 and [n, 32] uint8).
    A query loop keeps one FrameChannel instead."""
    import torch.distributed as dist
    if dist.get_rank() == src and not cap:
        cap = len(kps)
    return FrameChannel(cap, src, device).broadcast(kps, desc)


def keypoints_host(k) -> np.ndarray:
    """Broadcast keypoint records ([n, 28] uint8 tensor) as the 28-B structured array."""
    from .abi import KEYPOINT_DTYPE
    return np.ascontiguousarray(k.cpu().numpy()).view(KEYPOINT_DTYPE).reshape(-1)
