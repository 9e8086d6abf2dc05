"""Deterministic synthetic inputs.

No EuRoC / TUM-VI images and no ORBvoc.txt exist in the image, so every
workload is synthetic and seeded: u8 frames with full-range texture (random
rectangles and blobs of random intensity over a smooth illumination ramp,
additive noise sigma ~3, ~10 % flat patches so the minThFAST fallback and the
reflect-border paths are exercised), stereo right images shifted by a per-row
disparity field, a synthetic k-ary vocabulary and keyframe descriptor sets.
"""
from __future__ import annotations

import numpy as np


def frame_seed(config: int, index: int) -> int:
    return config * 1000 + index


def image(w: int, h: int, seed: int, n_shapes: int | None = None) -> np.ndarray:
    """One u8 image (h, w), deterministic in ``seed``.  Shapes are rendered in
    their bounding windows only, so a 752x480 frame takes a few ms."""
    rng = np.random.default_rng(seed)
    ang = rng.uniform(0, 2 * np.pi)
    xs = np.arange(w, dtype=np.float32)
    ys = np.arange(h, dtype=np.float32)
    img = (100.0 + 60.0 * (np.cos(ang) * xs[None, :] / w + np.sin(ang) * ys[:, None] / h)).astype(np.float32)
    n = n_shapes if n_shapes is not None else int(w * h / 900)
    kinds = rng.integers(0, 3, n)
    vals = rng.uniform(0, 255, n)
    cxs = rng.uniform(0, w, n)
    cys = rng.uniform(0, h, n)
    sizes = rng.uniform(0, 1, (n, 2))
    for kind, val, cx, cy, (s0, s1) in zip(kinds, vals, cxs, cys, sizes):
        if kind == 0:
            rw, rh = 3 + 37 * s0, 3 + 37 * s1
        elif kind == 1:
            rw = rh = 2 + 23 * s0
        else:
            rw = rh = 3 * (4 + 26 * s0)
        x0, x1 = max(0, int(cx - rw) - 1), min(w, int(cx + rw) + 2)
        y0, y1 = max(0, int(cy - rh) - 1), min(h, int(cy + rh) + 2)
        if x0 >= x1 or y0 >= y1:
            continue
        xx = xs[None, x0:x1] - cx
        yy = ys[y0:y1, None] - cy
        win = img[y0:y1, x0:x1]
        if kind == 0:
            m = (np.abs(xx) < rw) & (np.abs(yy) < rh)
            win[m] = val
        elif kind == 1:
            m = xx ** 2 + yy ** 2 < rw * rw
            win[m] = val
        else:
            r = rw / 3
            g = np.exp(-(xx ** 2 + yy ** 2) / (2 * r * r))
            win[:] = win * (1 - g) + val * g
    img += rng.normal(0, 3.0, size=img.shape).astype(np.float32)
    # ~10 % flat patches (no texture, no noise): exercises the minThFAST fallback
    for _ in range(max(1, int(0.10 * w * h / (48 * 48)))):
        x0, y0 = int(rng.integers(0, max(1, w - 48))), int(rng.integers(0, max(1, h - 48)))
        img[y0:y0 + 48, x0:x0 + 48] = rng.uniform(0, 255)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def stereo_pair(w: int, h: int, seed: int) -> tuple[np.ndarray, np.ndarray]:
    """Left image and a right image shifted by a 0-48 px per-row disparity."""
    left = image(w, h, seed)
    rng = np.random.default_rng(seed + 7_000_000)
    disp = np.clip(24 + 24 * np.sin(np.linspace(0, rng.uniform(1, 6), h)), 0, 48).astype(np.int64)
    right = np.empty_like(left)
    cols = np.arange(w)
    for y in range(h):
        right[y] = left[y, np.clip(cols + disp[y], 0, w - 1)]
    noise = rng.normal(0, 2.0, size=left.shape)
    right = np.clip(np.rint(right.astype(np.float64) + noise), 0, 255).astype(np.uint8)
    return left, right


def batch(w: int, h: int, nframes: int, config: int = 2, start: int = 0) -> np.ndarray:
    """(nframes, h, w) u8 stack of distinct seeded frames."""
    return np.stack([image(w, h, frame_seed(config, start + i)) for i in range(nframes)])


def vocabulary(k: int = 10, levels: int = 6, seed: int = 5, max_nodes: int | None = None):
    """Synthetic complete k-ary vocabulary of depth ``levels`` laid out breadth
    first (orbv_vocab): node 0 = root, TF-IDF-like random leaf weights.
    Children descriptors are perturbations of their parent so descents are
    stable.  Returns a dict of numpy arrays."""
    rng = np.random.default_rng(seed)
    counts = [k ** l for l in range(levels + 1)]
    nnodes = sum(counts)
    if max_nodes is not None and nnodes > max_nodes:
        raise ValueError("vocabulary too large")
    desc = np.zeros((nnodes, 32), np.uint8)
    first_child = np.zeros(nnodes, np.int32)
    nchild = np.zeros(nnodes, np.int32)
    word_id = np.full(nnodes, -1, np.int32)
    weight = np.zeros(nnodes, np.float64)
    desc[0] = rng.integers(0, 256, 32, dtype=np.uint8)
    start = 0
    nxt = 1
    for l in range(levels):
        for i in range(start, start + counts[l]):
            first_child[i] = nxt
            nchild[i] = k
            flip_p = 0.35 / (l + 1)
            for c in range(k):
                bits = np.unpackbits(desc[i])
                flips = rng.random(256) < flip_p
                desc[nxt + c] = np.packbits(bits ^ flips.astype(np.uint8))
            nxt += k
        start += counts[l]
    leaves = np.arange(start, nnodes)
    word_id[leaves] = np.arange(len(leaves), dtype=np.int32)
    weight[leaves] = rng.uniform(0.1, 5.0, len(leaves))
    return dict(nnodes=nnodes, depth_levels=levels, first_child=first_child, nchild=nchild,
                node_desc=desc, word_id=word_id, weight=weight)
