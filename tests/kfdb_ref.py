"""Synthetic keyframe database and an independent Python restatement of
KeyFrameDatabase::DetectRelocalizationCandidates (src/KeyFrameDatabase.cc:733-845),
used to pin the oracle (tests/test_kfdb.py) and, through it, the GPU path."""
from __future__ import annotations

import numpy as np


def make_db(nkf: int, nwords: int, seed: int, words_per_kf=(80, 300), nmaps: int = 2):
    """Per-KF L1-normalised BowVectors over a Zipf-like word distribution,
    the inverted file in a random insertion order, random covisibility top-10
    lists, map ids, and a query sharing many words with a few keyframes."""
    rng = np.random.default_rng(seed)
    p = 1.0 / np.arange(1, nwords + 1) ** 0.9
    p /= p.sum()
    bows = []
    for _ in range(nkf):
        m = int(rng.integers(*words_per_kf))
        w = np.unique(rng.choice(nwords, m, p=p)).astype(np.int32)
        v = rng.uniform(0.05, 1.0, len(w))
        bows.append((w, v / np.abs(v).sum()))
    bow_off = np.zeros(nkf + 1, np.int32)
    for i, (w, _) in enumerate(bows):
        bow_off[i + 1] = bow_off[i] + len(w)
    bow_words = np.concatenate([b[0] for b in bows]).astype(np.int32)
    bow_vals = np.concatenate([b[1] for b in bows])
    inv = [[] for _ in range(nwords)]
    for kf in rng.permutation(nkf):                       # KeyFrameDatabase::add order
        for w in bows[kf][0]:
            inv[w].append(int(kf))
    inv_off = np.zeros(nwords + 1, np.int32)
    for w in range(nwords):
        inv_off[w + 1] = inv_off[w] + len(inv[w])
    inv_kf = np.array([k for lst in inv for k in lst], np.int32)
    cov = [rng.choice(nkf, min(10, nkf - 1), replace=False) for _ in range(nkf)]
    cov = [c[c != i][:10] for i, c in enumerate(cov)]
    cov_off = np.zeros(nkf + 1, np.int32)
    for i, c in enumerate(cov):
        cov_off[i + 1] = cov_off[i] + len(c)
    cov_kf = np.concatenate(cov).astype(np.int32)
    kf_map = rng.integers(0, nmaps, nkf).astype(np.int32)
    db = dict(nkf=nkf, nwords=nwords, bow_off=bow_off, bow_words=bow_words, bow_vals=bow_vals, inv_off=inv_off,
              inv_kf=inv_kf, cov_off=cov_off, cov_kf=cov_kf, kf_map=kf_map, bows=bows, inv=inv, cov=cov)
    return db


def make_query(db, seed: int):
    rng = np.random.default_rng(seed)
    base = db["bows"][int(rng.integers(db["nkf"]))][0]
    keep = base[rng.random(len(base)) < 0.8]
    extra = rng.integers(0, db["nwords"], 40)
    w = np.unique(np.concatenate([keep, extra])).astype(np.int32)
    v = rng.uniform(0.05, 1.0, len(w))
    return w, v / np.abs(v).sum()


def l1_score(qw, qv, w, v):
    d = dict(zip(w.tolist(), v.tolist()))
    s = 0.0
    for a, vi in zip(qw.tolist(), qv.tolist()):
        if a in d:
            wi = d[a]
            s += abs(vi - wi) - abs(vi) - abs(wi)
    return -s / 2.0


def detect(db, qw, qv, map_id, reloc_score):
    f32 = np.float32
    sharing, words = [], {}
    for w in qw.tolist():
        for kf in db["inv"][w]:
            if kf not in words:
                words[kf] = 0
                sharing.append(kf)
            words[kf] += 1
    if not sharing:
        return []
    max_common = max(words[k] for k in sharing)
    min_common = int(f32(max_common) * f32(0.8))
    scored = []
    for kf in sharing:
        if words[kf] > min_common:
            si = f32(l1_score(qw, qv, *db["bows"][kf]))
            reloc_score[kf] = si
            scored.append((si, kf))
    if not scored:
        return []
    acc, best_acc = [], f32(0)
    for si, kf in scored:
        best, accs, best_kf = si, si, kf
        for k2 in db["cov"][kf].tolist():
            if k2 not in words:
                continue
            accs = f32(accs + reloc_score[k2])
            if reloc_score[k2] > best:
                best_kf, best = k2, reloc_score[k2]
        acc.append((accs, best_kf))
        if accs > best_acc:
            best_acc = accs
    min_keep = f32(f32(0.75) * best_acc)
    out, seen = [], set()
    for s, kf in acc:
        if s > min_keep and db["kf_map"][kf] == map_id and kf not in seen:
            out.append(kf)
            seen.add(kf)
    return out
