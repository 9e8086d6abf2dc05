"""Independent Python restatements of the DBoW2 vocabulary side
(Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h, BowVector.cpp,
FeatureVector.cpp, ScoringObject.cpp) used to pin the library's host code:
saveToTextFile (:1428-1449, writer), loadFromTextFile (:1338-1424, a line
loop with per-line token streams), transform(features, v, fv, levelsup)
assembly and the L1 / L2 / chi-square / Bhattacharyya / dot-product scores."""
from __future__ import annotations

import math

import numpy as np


def save_text(path, voc: dict, k: int, scoring: int = 0, weighting: int = 0, trailing_newline: bool = True):
    """saveToTextFile: `k L  scoring weighting` then `parent leaf b0 .. b31  weight`
    per node 1..n-1 (std::endl after every line); weights in the default
    6-significant-digit stream format."""
    n = voc["nnodes"]
    lines = [f"{k} {voc['depth_levels']}  {scoring} {weighting}"]
    parent = np.zeros(n, np.int64)
    for i in range(n):
        c0, nc = voc["first_child"][i], voc["nchild"][i]
        for j in range(nc):
            c = voc["child_idx"][c0 + j] if voc.get("child_idx") is not None else c0 + j
            parent[c] = i
    for i in range(1, n):
        leaf = 1 if voc["nchild"][i] == 0 else 0
        d = " ".join(str(int(b)) for b in voc["node_desc"][i]) + " "
        lines.append(f"{parent[i]} {leaf} {d} {float(voc['weight'][i]):.6g}")
    txt = "\n".join(lines) + ("\n" if trailing_newline else "")
    with open(path, "w") as f:
        f.write(txt)


def _ints(tokens):
    """Stream-style int extraction over whitespace tokens: stops at the first
    failure; the failed target and all later ones read 0."""
    out, ok = [], True
    for t in tokens:
        if ok:
            try:
                out.append(int(t))
                continue
            except ValueError:
                ok = False
        out.append(0)
    return out


def load_text(path) -> dict | None:
    with open(path, "rb") as f:
        data = f.read().decode("latin-1")
    segs = data.split("\n")
    head = segs[0].split()
    hv = (_ints(head[:4]) + [0, 0, 0, 0])[:4]
    k, L, n1, n2 = hv
    if k < 0 or k > 20 or L < 1 or L > 10 or n1 < 0 or n1 > 5 or n2 < 0 or n2 > 3:
        return None
    nodes_parent, nodes_desc, nodes_w, nodes_leaf = [0], [bytes(32)], [0.0], [False]
    children = [[]]
    for seg in segs[1:]:
        tok = seg.split()
        nid = len(nodes_parent)
        fields = tok + [None] * (35 - len(tok))
        ok = True

        def take_int(t):
            nonlocal ok
            if not ok or t is None:
                ok = False
                return 0
            try:
                return int(t)
            except ValueError:
                ok = False
                return 0
        pid = take_int(fields[0])
        leaf = take_int(fields[1])
        dtoks = [fields[2 + i] if ok else None for i in range(32)]
        if any(t is None for t in dtoks):
            ok = False
        desc = []
        dok = True
        for t in dtoks:
            if dok and t is not None:
                try:
                    desc.append(int(t) & 0xff)
                    continue
                except ValueError:
                    dok = False
            dok = False
            desc.append(0)
        w = 0.0
        if ok and fields[34] is not None:
            try:
                w = float(fields[34])
            except ValueError:
                w = 0.0
        nodes_parent.append(pid)
        children[pid].append(nid)
        children.append([])
        nodes_desc.append(bytes(desc))
        nodes_w.append(w)
        nodes_leaf.append(leaf > 0)
    n = len(nodes_parent)
    word_id = np.zeros(n, np.int32)
    nw = 0
    for i in range(1, n):
        if nodes_leaf[i]:
            word_id[i] = nw
            nw += 1
    first, nch, cidx = np.zeros(n, np.int32), np.zeros(n, np.int32), []
    for i in range(n):
        first[i] = len(cidx)
        nch[i] = len(children[i])
        cidx += children[i]
    return dict(nnodes=n, depth_levels=L, k=k, scoring=n1, weighting=n2, nwords=nw, first_child=first,
                nchild=nch, child_idx=np.array(cidx, np.int32),
                node_desc=np.frombuffer(b"".join(nodes_desc), np.uint8).reshape(n, 32).copy(),
                word_id=word_id, weight=np.array(nodes_w, np.float64))


def bow_assemble(scoring, weighting, wid, w, nid):
    v, fv = {}, {}
    tf = weighting in (0, 1)
    for i, (a, b, c) in enumerate(zip(wid.tolist(), w.tolist(), nid.tolist())):
        if b > 0:
            if tf:
                v[a] = v.get(a, 0.0) + b
            elif a not in v:
                v[a] = b
            fv.setdefault(c, []).append(i)
    keys = sorted(v)
    must = scoring != 5
    if tf and v and not must:
        for kk in keys:
            v[kk] /= float(len(v))
    if must:
        norm = 0.0
        if scoring != 1:
            for kk in keys:
                norm += abs(v[kk])
        else:
            for kk in keys:
                norm += v[kk] * v[kk]
            norm = math.sqrt(norm)
        if norm > 0.0:
            for kk in keys:
                v[kk] /= norm
    return (np.array(keys, np.int32), np.array([v[kk] for kk in keys], np.float64),
            {kk: fv[kk] for kk in sorted(fv)})


LOG_EPS = math.log(2.220446049250313e-16)


def score(scoring, w1, v1, w2, v2):
    d2 = dict(zip(w2.tolist(), v2.tolist()))
    s = 0.0
    for a, vi in zip(w1.tolist(), v1.tolist()):
        if a not in d2:
            if scoring == 3 and vi != 0:
                s += vi * (math.log(vi) - LOG_EPS)
            continue
        if scoring == 3:
            wi = d2[a]
            if vi != 0 and wi != 0:
                s += vi * math.log(vi / wi)
            continue
        wi = d2[a]
        if scoring == 0:
            s += abs(vi - wi) - abs(vi) - abs(wi)
        elif scoring in (1, 5):
            s += vi * wi
        elif scoring == 2:
            if vi + wi != 0.0:
                s += vi * wi / (vi + wi)
        elif scoring == 4:
            s += math.sqrt(vi * wi)
    if scoring == 0:
        return -s / 2.0
    if scoring == 1:
        return 1.0 if s >= 1 else 1.0 - math.sqrt(1.0 - s)
    if scoring == 2:
        return 2.0 * s
    return s
