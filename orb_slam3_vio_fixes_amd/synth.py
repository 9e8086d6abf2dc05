"""Deterministic synthetic inputs.

No EuRoC / TUM-VI images and no ORBvoc.txt exist in the image, so every
workload is synthetic and seeded: u8 frames with full-range texture (random
rectangles and blobs of random intensity over a smooth illumination ramp,
additive integer noise sigma ~3, ~10 % flat patches so the minThFAST fallback and the
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
    # only IEEE basic arithmetic (no exp/sin/cos): bit-identical on every host CPU
    rng = np.random.default_rng(seed)
    gx, gy = rng.uniform(-1, 1, 2)
    xs = np.arange(w, dtype=np.float32)
    ys = np.arange(h, dtype=np.float32)
    img = (np.float32(100.0) + np.float32(60.0 * gx / w) * xs[None, :]
           + np.float32(60.0 * gy / h) * ys[:, None]).astype(np.float32)
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
            t = np.maximum(np.float32(0), np.float32(1) - (xx * xx + yy * yy) / np.float32(rw * rw))
            g = t * t * t
            win[:] = win * (1 - g) + np.float32(val) * g
    img += rng.integers(-5, 6, size=img.shape).astype(np.float32)   # ~sigma 3, exact on any host
    # ~10 % flat patches (no texture, no noise): exercises the minThFAST fallback
    for _ in range(max(1, int(0.10 * w * h / (48 * 48)))):
        x0, y0 = int(rng.integers(0, max(1, w - 48))), int(rng.integers(0, max(1, h - 48)))
        img[y0:y0 + 48, x0:x0 + 48] = rng.uniform(0, 255)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def right_view(left: np.ndarray, seed: int) -> np.ndarray:
    """Right image of a rectified pair: ``left`` shifted by a smooth 0-48 px
    per-row disparity (integer), plus independent sensor noise."""
    h, w = left.shape
    rng = np.random.default_rng(seed + 7_000_000)
    knots = rng.integers(0, 49, 9)
    disp = np.rint(np.interp(np.arange(h), np.linspace(0, h - 1, 9), knots)).astype(np.int64)
    cols = np.arange(w)
    right = left[np.arange(h)[:, None], np.clip(cols[None, :] + disp[:, None], 0, w - 1)]
    noise = rng.integers(-2, 3, size=left.shape)
    return np.clip(right.astype(np.int64) + noise, 0, 255).astype(np.uint8)


def stereo_pair(w: int, h: int, seed: int) -> tuple[np.ndarray, np.ndarray]:
    """Left image and a right image shifted by a 0-48 px per-row disparity."""
    left = image(w, h, seed)
    return left, right_view(left, seed)


def stereo_sequence(w: int, h: int, npairs: int, config: int = 3, start: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """(npairs, h, w) left frames of a panning camera (``sequence``) and their
    right views (``right_view``, seeded per frame)."""
    left = sequence(w, h, npairs, config=config, start=start)
    right = np.stack([right_view(left[i], frame_seed(config, start + i)) for i in range(npairs)])
    return left, right


def batch(w: int, h: int, nframes: int, config: int = 2, start: int = 0) -> np.ndarray:
    """(nframes, h, w) u8 stack of distinct seeded frames."""
    return np.stack([image(w, h, frame_seed(config, start + i)) for i in range(nframes)])


def sequence(w: int, h: int, nframes: int, config: int = 2, start: int = 0, step: float = 3.0) -> np.ndarray:
    """(nframes, h, w) u8 frames of a camera panning over one static scene:
    crops of a large seeded canvas along a smooth integer trajectory (a few px
    per frame), each with fresh integer sensor noise.  Consecutive frames share
    most of their content, so SearchForInitialization finds real matches."""
    seed = frame_seed(config, start)
    rng = np.random.default_rng(seed + 11_000_000)
    span = int(step * nframes) + 8
    canvas = image(w + span, h + span, seed).astype(np.int16)
    vx, vy = rng.uniform(0.3, 1.0, 2)
    norm = max(vx, vy)
    out = np.empty((nframes, h, w), np.uint8)
    for i in range(nframes):
        ox = int(round(i * step * vx / norm)) % (span - 4)
        oy = int(round(i * step * vy / norm)) % (span - 4)
        noise = rng.integers(-2, 3, size=(h, w), dtype=np.int16)
        out[i] = np.clip(canvas[oy:oy + h, ox:ox + w] + noise, 0, 255).astype(np.uint8)
    return out


def global_sequence(w: int, h: int, first: int, nframes: int, config: int = 2, step: float = 3.0,
                    span: int = 776) -> np.ndarray:
    """Frames [first, first + nframes) of ONE panning sequence whose frame g
    depends on g alone, so any partition of the frames over ranks (plus the
    halo frame a rank extracts across its seam) sees the same images: a fixed
    seeded canvas, a periodic integer trajectory on it, fresh integer sensor
    noise seeded by g."""
    seed = frame_seed(config, 0)
    rng = np.random.default_rng(seed + 12_000_000)
    canvas = image(w + span, h + span, seed).astype(np.int16)
    vx, vy = rng.uniform(0.3, 1.0, 2)
    norm = max(vx, vy)
    out = np.empty((nframes, h, w), np.uint8)
    for i in range(nframes):
        g = first + i
        ox = int(round(g * step * vx / norm)) % (span - 4)
        oy = int(round(g * step * vy / norm)) % (span - 4)
        noise = np.random.default_rng(seed * 7919 + g).integers(-2, 3, size=(h, w), dtype=np.int16)
        out[i] = np.clip(canvas[oy:oy + h, ox:ox + w] + noise, 0, 255).astype(np.uint8)
    return out


def vocabulary(k: int = 10, levels: int = 6, seed: int = 5):
    """Synthetic complete k-ary vocabulary of depth ``levels`` (the ORBvoc.txt
    shape is k=10, L=6: 1,111,111 nodes) laid out breadth first (orbv_vocab):
    node 0 = root, children of a node contiguous.  Each child descriptor is
    its parent's with every bit flipped with probability 2^-min(4, level+1)
    (AND of random bytes), so descents are stable; leaf weights are random
    TF-IDF-like values.  Vectorised per level; returns a dict of arrays."""
    rng = np.random.default_rng(seed)
    counts = [k ** l for l in range(levels + 1)]
    nnodes = sum(counts)
    desc = np.empty((nnodes, 32), np.uint8)
    first_child = np.zeros(nnodes, np.int32)
    nchild = np.zeros(nnodes, np.int32)
    word_id = np.full(nnodes, -1, np.int32)
    weight = np.zeros(nnodes, np.float64)
    desc[0] = rng.integers(0, 256, 32, dtype=np.uint8)
    start = 0
    for l in range(levels):
        n = counts[l]
        cstart = start + n
        first_child[start:start + n] = cstart + np.arange(n, dtype=np.int32) * k
        nchild[start:start + n] = k
        par = np.repeat(desc[start:start + n], k, axis=0)
        flips = rng.integers(0, 256, par.shape, dtype=np.uint8)
        for _ in range(min(4, l + 1) - 1):
            flips &= rng.integers(0, 256, par.shape, dtype=np.uint8)
        desc[cstart:cstart + n * k] = par ^ flips
        start = cstart
    nleaf = counts[levels]
    word_id[start:] = np.arange(nleaf, dtype=np.int32)
    weight[start:] = rng.uniform(0.1, 5.0, nleaf)
    return dict(nnodes=nnodes, depth_levels=levels, first_child=first_child, nchild=nchild,
                node_desc=desc, word_id=word_id, weight=weight)


def keyframe_map(kps: np.ndarray, desc: np.ndarray, node_of_feature: np.ndarray, ids, seed: int = 7,
                 per_kf: int | None = None, valid_frac: float = 1.0, near_frac: float = 1.0,
                 far_nodes: int = 30) -> dict:
    """A synthetic keyframe map around a query frame (config C5, SURVEY.md
    §8(d)), packed in the orbm_kf_map_device layout (kfmap.pack).  Keyframe i
    (ids: the map's keyframe ids, so any shard of the map is the same data)
    holds per_kf of the query's features (default: all; 5000 of a 5000-feature
    extractor's ~5008) with their node ids, descriptors with 2^-3, 2^-4 or 2^-5
    of their bits flipped, angles jittered (+30 degrees for every 7th keyframe,
    so the rotation filter drops matches), and MapPoints valid with
    probability valid_frac (1.0: all valid, as SURVEY §8(d) states C5).

    near_frac < 1 makes the relocalisation case (Tracking.cc:3609-3662) of a
    map mostly from elsewhere: a keyframe is "near" (as above) with
    probability near_frac, otherwise "far": per_kf features with unrelated
    random descriptors whose node ids come from a keyframe-specific set of
    far_nodes of the query's level-(L - levelsup) nodes and nodes the query
    does not hold (ids just past its largest), so it shares a minority of its
    nodes with the query and almost no match passes TH_LOW."""
    from . import kfmap
    n = len(kps)
    m = n if per_kf is None else min(per_kf, n)
    ids = list(ids)
    nkf = len(ids)
    out_k = np.empty((nkf, m), np.dtype(kps.dtype))
    kb = out_k.view(np.uint8).reshape(nkf, m, -1)            # rows as bytes: fast gathers
    kps_b = np.ascontiguousarray(kps).view(np.uint8).reshape(n, -1)
    out_d = np.empty((nkf, m, 32), np.uint8)
    out_v = np.ones((nkf, m), np.uint8)
    nodes, offs, idxs = [], [], []
    node_off, idx_off, nidx = [0], [], 0
    nid_all = np.asarray(node_of_feature, np.int64)
    # bit-flip masks at rates 2^-3, 2^-4, 2^-5 (AND of 3..5 random bytes); a
    # keyframe takes m consecutive rows of one pool from a random start
    prng = np.random.default_rng(seed)
    pools = []
    for ands in (3, 4, 5):
        p = np.frombuffer(prng.bytes(max(1 << 18, 2 * m) * 32), np.uint8).reshape(-1, 32).copy()
        for _ in range(ands - 1):
            p &= np.frombuffer(prng.bytes(p.size), np.uint8).reshape(-1, 32)
        pools.append(p)
    qnodes = np.unique(nid_all[nid_all >= 0])
    hi = int(qnodes.max()) + 1 if len(qnodes) else 1
    other = np.arange(hi, hi + max(len(qnodes), far_nodes), dtype=np.int64)   # nodes the query lacks
    for j, i in enumerate(ids):
        rng = np.random.default_rng(seed * 1_000_003 + int(i))
        sel = np.sort(rng.permutation(n)[:m])
        kk = out_k[j]
        kb[j] = kps_b[sel]
        far = near_frac < 1.0 and rng.random() >= near_frac
        if far:
            kk["angle"] = rng.uniform(0, 360, m).astype(np.float32)
            out_d[j] = np.frombuffer(rng.bytes(m * 32), np.uint8).reshape(m, 32)
            shared = rng.choice(qnodes, size=min(len(qnodes), far_nodes // 3), replace=False)
            pool = np.concatenate([shared, rng.choice(other, size=far_nodes - len(shared), replace=False)])
            nid_kf = pool[rng.integers(0, len(pool), m)]
        else:
            kk["angle"] = (kk["angle"] + rng.normal(0, 4, m).astype(np.float32) + (30 if i % 7 == 0 else 0)) % 360
            r = int(rng.integers(0, 3))
            s0 = int(rng.integers(0, len(pools[r]) - m + 1))
            np.bitwise_xor(desc[sel], pools[r][s0:s0 + m], out=out_d[j])
            nid_kf = nid_all[sel]
        if valid_frac < 1.0:
            out_v[j] = rng.random(m) < valid_frac
        n_ids, o, ix = kfmap.featvec_csr(nid_kf)
        nodes.append(n_ids)
        offs.append(o)
        idx_off.append(nidx)
        nidx += len(ix)
        idxs.append(ix)
        node_off.append(node_off[-1] + len(n_ids))
    cat = lambda a, dt: np.ascontiguousarray(np.concatenate(a) if a else np.zeros(0, dt), dt)
    return dict(kps=out_k.reshape(-1).view(np.uint8), desc=out_d.reshape(-1), valid=out_v.reshape(-1),
                kp_off=np.arange(nkf + 1, dtype=np.int64) * m, fv_node=cat(nodes, np.uint32),
                fv_off=cat(offs, np.int32), fv_idx=cat(idxs, np.uint32),
                fv_node_off=np.array(node_off, np.int64), fv_idx_off=np.array(idx_off, np.int64))
