#!/usr/bin/env python3
"""Measurement of config C5 (BASELINE.json): a synthetic 1920x1080 frame with
5000 features, SearchByBoW(KF_i, F) against a 10,000-keyframe map resident in
HBM (relocalisation runs one ORBmatcher(0.75, true).SearchByBoW per candidate,
src/Tracking.cc:3641-3648; here every keyframe of the map in one launch,
orbm_search_by_bow_batch_device).

Query: HIP extraction (ORBextractor(5000, 1.2, 8, 20, 7)), node ids at
levelsup 4 from a full-size synthetic vocabulary (k=10, L=6, 1,111,111
nodes) by the GPU descent.  Map: 10,000 keyframes x 5000
descriptors, every MapPoint valid (synth.keyframe_map: 5000 of the query's
features per keyframe with their node ids, 2^-3..2^-5 of the descriptor bits
flipped, angles jittered; synthetic data, FeatureVectors are inputs of the
search, not recomputed).  Timed: K repetitions of the map-wide search on
one stream, bracketed by synchronisations.  CPU baseline and parity: the
oracle's SearchByBoW for EVERY keyframe of rank 0's shard (threads stated),
compared with the GPU's.  Multi-GPU (torch.distributed): the map is sharded
by keyframe id, the query is broadcast from rank 0 (sharding.py).
usage: python tools/bench_c5.py [--nkf 10000] [--per-kf 5000] [--reps 10] [--cpu-sample N (default: all)]"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))
import benchlib  # noqa: E402

W, H, NFEAT = 1920, 1080, 5000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nkf", type=int, default=10000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--per-kf", type=int, default=5000)
    ap.add_argument("--valid-frac", type=float, default=1.0,
                    help="share of keyframe features with a valid MapPoint (1.0: the stated C5 map)")
    ap.add_argument("--near-frac", type=float, default=1.0,
                    help="share of keyframes near the query (1.0: the stated map; e.g. 0.1: a relocalisation map "
                         "mostly from elsewhere, synth.keyframe_map)")
    ap.add_argument("--cpu-sample", type=int, default=-1, help="keyframes the oracle checks (-1: all)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); started here under torch.distributed.run when WORLD_SIZE is unset")
    ap.add_argument("--dump", default="", help="directory: each rank saves its shard's matches (tests)")
    args = ap.parse_args()
    from orb_slam3_vio_fixes_amd import launch
    rc = launch.ensure_ranks(args.gpus, __file__, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    res = run_c5(args)
    if res is not None:
        print(json.dumps(res), flush=True)


# algorithmic bytes the map-wide search reads per keyframe feature: its
# descriptor (32 B), its FeatureVector index (4 B) and its MapPoint flag (1 B)
KF_FEATURE_BYTES = 37


def run_c5(args):
    """Config C5 (see the module docstring); the JSON object on rank 0, None
    on the other ranks."""
    import torch
    import torch.distributed as dist
    from oracle import oracle as O
    from orb_slam3_vio_fixes_amd import abi, kfmap, orb, sharding, synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # RCCL; gloo (ORB_BENCH_BACKEND=gloo) when ranks share one GPU (tests)
        if os.environ.get("ORB_BENCH_BACKEND", "nccl") == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    if rank == 0:
        img = synth.image(W, H, 5000)
        ex = orb.ORBextractor(NFEAT, 1.2, 8, 20, 7, device=local)
        k, d, _ = ex(img, None, (0, 1000))
        vh = synth.vocabulary(10, 6, seed=55)
    else:
        k = d = vh = None
    if world > 1:
        # the vocabulary once, the query per query: RCCL broadcasts into HBM
        vt = sharding.broadcast_vocabulary(vh, 0, dev)
        # the query channel is made once (capacity agreed once); each query
        # is one fixed-size broadcast
        chan = sharding.FrameChannel(2 * NFEAT, 0, dev)
        kt, dt = chan.broadcast(k, d)
        k = sharding.keypoints_host(kt)
    else:
        vt = {key: torch.from_numpy(np.ascontiguousarray(vh[key])).to(dev)
              for key in ("first_child", "nchild", "node_desc", "word_id", "weight")}
        vt.update(nnodes=int(vh["nnodes"]), depth_levels=int(vh["depth_levels"]), child_idx=None)
        dt = torch.from_numpy(np.ascontiguousarray(d)).to(dev)
    d = dt.cpu().numpy()
    _, _, nid_t = orb.transform_device(sharding.vocab_device_struct(vt), dt, 4)
    nid = nid_t.cpu().numpy()
    ids = list(sharding.shard(args.nkf, rank, world))
    t0 = time.perf_counter()
    arrays = synth.keyframe_map(k, d, nid, ids, seed=7, per_kf=args.per_kf,
                                valid_frac=getattr(args, "valid_frac", 1.0),
                                near_frac=getattr(args, "near_frac", 1.0))
    m = kfmap.DeviceKeyframeMap(arrays=arrays)
    build_s = time.perf_counter() - t0
    nfeat_kf = int(arrays["kp_off"][-1])
    # the query frame resident in HBM before the timed region (keypoints,
    # descriptors, FeatureVector CSR, output rows), as after a device-side
    # extraction and transform; the per-query upload is timed separately below
    fr = m.prepare_frame(k, d, nid)
    for _ in range(args.warmup):
        match, nm = m.search_prepared(fr, 0.75, True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evs = []
    for _ in range(args.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        match, nm = m.search_prepared(fr, 0.75, True)
        e1.record()
        evs.append((e0, e1))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    tt = torch.tensor([el], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    el = float(tt.item())
    # the same searches with the frame uploaded from host memory in each query
    torch.cuda.synchronize()
    tu = time.perf_counter()
    for _ in range(args.reps):
        m.search_by_bow(k, d, nid, 0.75, True)
    torch.cuda.synchronize()
    upload_ms = (time.perf_counter() - tu) / args.reps * 1e3
    match, nm = m.search_prepared(fr, 0.75, True)
    torch.cuda.synchronize()
    if getattr(args, "dump", ""):
        os.makedirs(args.dump, exist_ok=True)
        np.savez(os.path.join(args.dump, f"rank{rank}.npz"), ids=np.asarray(ids, np.int64), nid=nid,
                 match=match.cpu().numpy(), nm=nm.cpu().numpy())
    kf_feat = nfeat_kf
    search_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    ach = kf_feat * KF_FEATURE_BYTES / (search_ms * 1e-3) / 1e9
    roof = {"kernel": "k_bow_init + k_bowk_* (map, fill, top-4 on MFMA, resolve) + k_bow_final (one map-wide search)", "bound": "hbm", "achieved": ach,
            "peak": benchlib.HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / benchlib.HBM_PEAK_GBS, "traffic": None,
            "bytes_per_launch": kf_feat * KF_FEATURE_BYTES, "ms_per_launch": search_ms,
            "bytes_per_unit": f"{KF_FEATURE_BYTES} B per keyframe feature (descriptor, FeatureVector index, "
                              "MapPoint flag), rank 0's shard"}
    res = {"metric": "C5 map-wide SearchByBoW: keyframe pairs/s (1920x1080, 5000 feat, 10k-KF map)",
           "value": args.nkf * args.reps / el, "unit": "keyframe-pairs/s", "queries_per_s": args.reps / el,
           "ms_per_query": el / args.reps * 1e3, "n_gpus": world, "nkf": args.nkf, "features": int(len(k)),
           "kf_features_total": nfeat_kf * world, "mappoints_valid_frac": float(arrays["valid"].mean()),
           "near_frac": getattr(args, "near_frac", 1.0), "data": "synthetic",
           "ms_per_query_with_frame_upload": upload_ms,
           "timed": "map-wide search, query frame resident in HBM (prepare_frame before the timed region)",
           "map_build_s_rank0": build_s, "mean_matches": float(nm.float().mean().item()),
           "scaling": "strong", "higher_is_better": True, "dtype": "u8", "roofline": roof}
    if rank == 0 and args.cpu_sample != 0:
        ns = len(ids) if args.cpu_sample < 0 else min(args.cpu_sample, len(ids))
        sub = arrays
        if ns < len(ids):   # the first ns keyframes of the shard
            e = int(arrays["kp_off"][ns])
            sub = dict(arrays, kp_off=arrays["kp_off"][:ns + 1], fv_node_off=arrays["fv_node_off"][:ns + 1],
                       fv_idx_off=arrays["fv_idx_off"][:ns], kps=arrays["kps"][:e * 28], desc=arrays["desc"][:e * 32],
                       valid=arrays["valid"][:e])
        f = abi.frame_struct(k, d, W, H)
        fv = abi.featvec_struct(nid)
        t0 = time.perf_counter()
        rmatch, rnm = O.search_by_bow_map(sub, f, fv, 0.75, True, nthreads=args.cpu_threads)
        dt = time.perf_counter() - t0
        mh, nh = match[:ns].cpu().numpy(), nm[:ns].cpu().numpy()
        bad = int(np.sum((rnm != nh) | np.any(rmatch != mh, axis=1)))
        res["cpu_baseline"] = {"value": ns / dt, "unit": "keyframe-pairs/s", "cores": args.cpu_threads,
                               "kind": "port", "sample": f"{'all' if ns == len(ids) else 'first'} {ns} keyframes of "
                                                         "rank 0's map shard, oracle SearchByBoW (threaded map loop)"}
        res["parity"] = {"keyframes_checked": ns, "keyframes_mismatched": bad,
                         "matches_total": int(rnm.sum())}
    if world > 1:
        dist.destroy_process_group()
    return res if rank == 0 else None


if __name__ == "__main__":
    main()
