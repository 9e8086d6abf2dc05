#!/usr/bin/env python3
"""Measurement of the SURVEY.md §8(f) row-1 workload (config C3): rectified
752x480 stereo pairs, ORBextractor(1200, 1.2, 8, 20, 7) with lapping {0, 0}
on left and right, Frame::ComputeStereoMatches (Frame.cc:811-981) on every
pair, SearchForInitialization(window 100, 0.9, checkOri) on consecutive left
frames (Tracking.cc:2459-2492).  One step = one batch of B pairs resident in
HBM (left and right frames extracted in one launch chain).  Prints one JSON
line with pairs/s, per-stage times (HIP events), a CPU-oracle baseline on a
bounded sample and the parity of that sample.

With --workload c4: 512x512 fisheye stereo pairs,
ORBextractor(1500) with lapping {0, 511}, the ComputeStereoFishEyeMatches
candidates (knnMatch k=2 + Lowe 0.7 over the lapping areas, Frame.cc:1126-1156);
the Kannala-Brandt triangulation of the candidates stays on the host.

Multi-GPU: one process per GPU under torch.distributed.run;
pairs are sharded by contiguous range of ONE global sequence (pair g depends
on g alone), --pairs per rank (weak scaling), no data-path collective; a
barrier brackets the timed region and its time is the max over ranks.  C3's
SearchForInitialization runs on consecutive LEFT frames, so every rank but the
last also extracts the next rank's first left frame (the seam halo, not
counted) and matches the pair across the seam; C4's pairs are independent.

usage: python tools/bench_stereo.py [--workload c3|c4] [--pairs 128] [--steps 10] [--warmup 2] [--dump DIR]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))
import benchlib  # noqa: E402

W, H, NFEAT, LAP = 752, 480, 1200, (0, 0)
FX, BASE = 435.2, 0.11            # EuRoC-like rectified rig
MBF = float(np.float32(BASE) * np.float32(FX))
SFI_AFTER_STAGE = 2    # orbx_set_stage_event: the matching starts once the next extraction's FAST pass is done


def cpu_baseline(left, right, threads):
    from oracle import oracle as O
    O.lib()                      # load (and build if stale) once, before the worker threads
    n = len(left)
    outs = [None] * n

    def work(t):
        el, er = O.OracleExtractor(NFEAT, 1.2, 8, 20, 7), O.OracleExtractor(NFEAT, 1.2, 8, 20, 7)
        for i in range(t, n, threads):
            kl, dl, _ = el(left[i], LAP)
            kr, dr, _ = er(right[i], LAP)
            outs[i] = (kl, O.compute_stereo_matches(el, er, kl, dl, kr, dr, BASE, MBF))
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as pool:
        list(pool.map(work, range(threads)))
    return n / (time.perf_counter() - t0), outs


def dist_init():
    """(world, rank, device index) of this process; initialises the process
    group for world > 1 (RCCL, or gloo with ORB_BENCH_BACKEND=gloo when ranks
    share one GPU in tests), as bench.py does."""
    import os
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = os.environ.get("ORB_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, local


def dist_time(t0_fn, world, dev):
    """Barrier + synchronize on both sides of the timed region; returns the
    max over ranks of the elapsed time (t0_fn runs the timed steps)."""
    import os
    import torch
    import torch.distributed as dist
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    t0_fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        nccl = os.environ.get("ORB_BENCH_BACKEND", "nccl") == "nccl"
        t = torch.tensor([dt], dtype=torch.float64, device=dev if nccl else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["c3", "c4"], default="c3")
    ap.add_argument("--pairs", type=int, default=128)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-sample", type=int, default=64)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); started here under torch.distributed.run when WORLD_SIZE is unset")
    ap.add_argument("--dump", default="", help="directory: each rank saves its last step's outputs (tests)")
    args = ap.parse_args()
    from orb_slam3_vio_fixes_amd import launch
    rc = launch.ensure_ranks(args.gpus, __file__, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    out = run_c4(args) if args.workload == "c4" else run_c3(args)
    if out is not None:
        print(json.dumps(out), flush=True)


def run_c3(args):
    """Config C3 (see the module docstring); returns the JSON object."""
    import torch
    from orb_slam3_vio_fixes_amd import capi, orb, synth
    world, rank, local = dist_init()
    dev = torch.device("cuda", local)
    P = args.pairs
    # pairs [rank P, (rank + 1) P) of one global sequence; the seam halo (the
    # next rank's first left frame) is extracted but not counted
    first = rank * P
    Px = P + (1 if rank < world - 1 else 0)
    left = synth.global_sequence(W, H, first, Px, config=3)
    right = np.stack([synth.right_view(left[i], synth.frame_seed(3, first + i)) for i in range(P)])
    frames = torch.from_numpy(np.concatenate([left, right])).to(dev)
    L = capi.lib()
    stream = torch.cuda.current_stream(dev)
    inv_w = float(np.float32(64) / np.float32(W))
    inv_h = float(np.float32(48) / np.float32(H))
    # Pipeline: step k's matching (ComputeStereoMatches, which reads the
    # extractor's device pyramid, and SearchForInitialization, which reads the
    # keypoints and descriptors) runs on two side streams while step k+1 extracts
    # on the main stream.  Two extractor handles and two output sets alternate;
    # step k+2 waits for step k's matching before it reuses them.
    sets = []
    for _ in range(2):
        ex = orb.ORBextractor(NFEAT, 1.2, 8, 20, 7)
        kps, desc, n, mono, cap = ex.extract_batch_device(frames, LAP)
        ur = torch.empty((P, cap), dtype=torch.float32, device=dev)
        sets.append({"ex": ex, "out": (kps, desc, n, mono), "cap": cap, "ur": ur, "dep": torch.empty_like(ur),
                     "sad": torch.empty((P, cap), dtype=torch.int32, device=dev),
                     "matches": torch.empty((Px - 1, cap), dtype=torch.int32, device=dev),
                     "nmatch": torch.empty(Px - 1, dtype=torch.int32, device=dev), "done": None})
    s_st, s_sfi = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    ev = []
    it = [0]
    # as in bench.py (C2): step k's matching is enqueued behind step k+1's
    # "FAST cells done" stage event (orbx_set_stage_event), so it shares the GPU
    # with the latency-bound quadtree / describe stages, not with the pyramid
    # and FAST passes whose times the roofline reports
    stage_ev = []
    for S in sets:
        e_ = torch.cuda.Event()
        e_.record(stream)                                    # creates the event
        capi.check(L.orbx_set_stage_event(S["ex"]._h, SFI_AFTER_STAGE, e_.cuda_event), "stage event")
        stage_ev.append(e_)
    pending = []

    def match(S, extracted, after, e):
        kps, desc, n, mono = S["out"]
        cap = S["cap"]
        for st_ in (s_st, s_sfi):
            st_.wait_event(extracted)
            if after is not None:
                st_.wait_event(after)
        if e is not None:
            e[2].record(s_st)
            e[4].record(s_sfi)
        capi.check(L.orbs_compute_stereo_matches_batch_device(S["ex"]._h, P, 0, Px, kps.data_ptr(), desc.data_ptr(),
                                                              n.data_ptr(), cap, BASE, MBF, S["ur"].data_ptr(),
                                                              S["dep"].data_ptr(), S["sad"].data_ptr(),
                                                              s_st.cuda_stream), "stereo")
        capi.check(L.orbm_search_for_initialization_batch_device(
            Px, kps.data_ptr(), desc.data_ptr(), n.data_ptr(), cap, 0.0, float(W), 0.0, float(H), inv_w, inv_h,
            100, 0.9, 1, S["matches"].data_ptr(), S["nmatch"].data_ptr(), s_sfi.cuda_stream), "sfi")
        if e is not None:
            e[3].record(s_st)
            e[5].record(s_sfi)
            ev.append(e)
        done = torch.cuda.Event()
        s_sfi.wait_stream(s_st)
        done.record(s_sfi)
        S["done"] = done

    def step(timed=False):
        i = it[0] % 2
        S = sets[i]
        it[0] += 1
        ex, (kps, desc, n, mono) = S["ex"], S["out"]
        e = [torch.cuda.Event(enable_timing=True) for _ in range(6)] if timed else None
        if S["done"] is not None:
            stream.wait_event(S["done"])                     # step k-2's matching released this set
        if timed:
            e[0].record(stream)
        ex.extract_batch_device(frames, LAP, out=(kps, desc, n, mono))
        if timed:
            e[1].record(stream)
        extracted = torch.cuda.Event()
        extracted.record(stream)
        while pending:                                       # the previous step's matching, behind this stage
            pS, pev, pe = pending.pop()
            match(pS, pev, stage_ev[i], pe)
        pending.append((S, extracted, e))

    def flush():
        while pending:
            pS, pev, pe = pending.pop()
            match(pS, pev, None, pe)

    for _ in range(args.warmup):
        step()
    flush()
    torch.cuda.synchronize()
    exs = [S["ex"] for S in sets]
    benchlib.profile_on(exs)

    def timed():
        for _ in range(args.steps):
            step(timed=True)
        flush()
    dt = dist_time(timed, world, dev)
    xst, calls = benchlib.profile_read(exs)
    if args.dump:
        S = sets[(it[0] - 1) % 2]                            # the last step's outputs, global pair indices
        Path(args.dump).mkdir(parents=True, exist_ok=True)
        np.savez(Path(args.dump) / f"rank{rank}.npz", first=first, pairs=P, frames=Px, world=world,
                 kps=S["out"][0].cpu().numpy(), desc=S["out"][1].cpu().numpy(), n=S["out"][2].cpu().numpy(),
                 ur=S["ur"].cpu().numpy(), dep=S["dep"].cpu().numpy(), matches=S["matches"].cpu().numpy(),
                 nmatch=S["nmatch"].cpu().numpy())
    if rank != 0:
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return None
    stage = {"extract_2B_images": float(np.mean([e[0].elapsed_time(e[1]) for e in ev])),
             "compute_stereo_matches_side_stream": float(np.mean([e[2].elapsed_time(e[3]) for e in ev])),
             "search_for_initialization_side_stream": float(np.mean([e[4].elapsed_time(e[5]) for e in ev]))}
    out = {"metric": "stereo pairs/s (752x480 L+R ORB extract, ComputeStereoMatches, SearchForInitialization)",
           "value": P * args.steps * world / dt, "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
           "dtype": "u8", "data": "synthetic",
           "config": {"workload": "C3: 752x480 rectified stereo, ORBextractor(1200,1.2,8,20,7), lapping {0,0}, "
                                  "mb 0.11 m, fx 435.2", "pairs_per_step_per_gpu": P,
                      "parallelism": f"pairs sharded over {world} GPU(s), halo left frame per seam"},
           "stage_ms": stage, "extract_stage_ms": xst,
           "roofline": benchlib.fast_roofline(sets[0]["ex"], W, H, xst, 2 * P * args.steps / max(1, calls))}
    if args.cpu_sample > 0 and world == 1:
        ns = min(args.cpu_sample, P)
        fps, outs = cpu_baseline(left[:ns], right[:ns], args.cpu_threads)
        S = sets[(it[0] - 1) % 2]                            # the last step's outputs
        urh, deph, nh = S["ur"].cpu().numpy(), S["dep"].cpu().numpy(), S["out"][2].cpu().numpy()
        bad = 0
        for i in range(ns):
            rk, (rur, rdep) = outs[i]
            if nh[i] != len(rk) or not np.array_equal(urh[i, :nh[i]].view(np.uint32), rur.view(np.uint32)) or \
                    not np.array_equal(deph[i, :nh[i]].view(np.uint32), rdep.view(np.uint32)):
                bad += 1
        out["cpu_baseline"] = {"value": fps, "unit": "pairs/s", "cores": args.cpu_threads, "kind": "port",
                               "sample": f"first {ns} pairs: oracle extraction of L and R + ComputeStereoMatches"}
        out["parity"] = {"pairs_checked": ns, "pairs_mismatched": bad,
                         "matched_fraction": float(np.mean([(o[1][0] >= 0).mean() for o in outs]))}
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return out


def run_c4(args):
    """Config C4 (see the module docstring); returns the JSON object."""
    import torch
    from oracle import oracle as O
    from orb_slam3_vio_fixes_amd import capi, orb, synth
    w = h = 512
    nf, lap = 1500, (0, 511)
    world, rank, local = dist_init()
    dev = torch.device("cuda", local)
    P = args.pairs
    # pairs [rank P, (rank + 1) P) of one global sequence (independent pairs: no halo)
    first = rank * P
    left = synth.global_sequence(w, h, first, P, config=4)
    right = np.stack([synth.right_view(left[i], synth.frame_seed(4, first + i)) for i in range(P)])
    frames = torch.from_numpy(np.concatenate([left, right])).to(dev)
    ex = orb.ORBextractor(nf, 1.2, 8, 20, 7)
    stream = torch.cuda.current_stream(dev)
    # knnMatch of step k (descriptors only) on a side stream while step k+1
    # extracts; two output sets alternate, step k+2 waits for step k's match
    sets = [list(ex.extract_batch_device(frames, lap)) + [None] for _ in range(2)]
    cap = sets[0][4]
    side = torch.cuda.Stream(dev)
    ev = []
    it = [0]
    L = capi.lib()
    # step k's knnMatch behind step k+1's "FAST cells done" stage event (C2's placement)
    stage_ev = []
    for _ in range(2):
        e_ = torch.cuda.Event()
        e_.record(stream)
        stage_ev.append(e_)
    pending = []
    res = [None]

    def match(S, extracted, after, e):
        kps, desc, n, mono = S[:4]
        side.wait_event(extracted)
        if after is not None:
            side.wait_event(after)
        with torch.cuda.stream(side):
            if e is not None:
                e[2].record(side)
            res[0] = orb.fisheye_stereo_candidates_batch_device(P, 0, P, desc, n, mono, cap)
            if e is not None:
                e[3].record(side)
                ev.append(e)
            done = torch.cuda.Event()
            done.record(side)
        S[5] = done

    def step(timed=False):
        i = it[0] % 2
        S = sets[i]
        it[0] += 1
        kps, desc, n, mono = S[:4]
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if timed else None
        if S[5] is not None:
            stream.wait_event(S[5])
        capi.check(L.orbx_set_stage_event(ex._h, SFI_AFTER_STAGE, stage_ev[i].cuda_event), "stage event")
        if timed:
            e[0].record(stream)
        ex.extract_batch_device(frames, lap, out=(kps, desc, n, mono))
        if timed:
            e[1].record(stream)
        extracted = torch.cuda.Event()
        extracted.record(stream)
        while pending:
            pS, pev, pe = pending.pop()
            match(pS, pev, stage_ev[i], pe)
        pending.append((S, extracted, e))

    def flush():
        while pending:
            pS, pev, pe = pending.pop()
            match(pS, pev, None, pe)

    for _ in range(args.warmup):
        step()
    flush()
    torch.cuda.synchronize()
    benchlib.profile_on([ex])

    def timed():
        for _ in range(args.steps):
            step(timed=True)
        flush()
    dt = dist_time(timed, world, dev)
    idx, _, l2r = res[0]
    xst, calls = benchlib.profile_read([ex])
    if args.dump:
        S = sets[(it[0] - 1) % 2]
        Path(args.dump).mkdir(parents=True, exist_ok=True)
        np.savez(Path(args.dump) / f"rank{rank}.npz", first=first, pairs=P, world=world,
                 kps=S[0].cpu().numpy(), desc=S[1].cpu().numpy(), n=S[2].cpu().numpy(), mono=S[3].cpu().numpy(),
                 idx=idx.cpu().numpy(), l2r=l2r.cpu().numpy())
    if rank != 0:
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return None
    stage = {"extract_2B_images": float(np.mean([e[0].elapsed_time(e[1]) for e in ev])),
             "fisheye_knn2_ratio_side_stream": float(np.mean([e[2].elapsed_time(e[3]) for e in ev]))}
    out = {"metric": "fisheye stereo pairs/s (512x512 L+R ORB extract, knnMatch(2) + ratio over the lapping areas)",
           "value": P * args.steps * world / dt, "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
           "dtype": "u8", "data": "synthetic",
           "config": {"workload": "C4: 512x512 fisheye stereo, ORBextractor(1500,1.2,8,20,7), lapping {0,511}",
                      "pairs_per_step_per_gpu": P, "parallelism": f"pairs sharded over {world} GPU(s)"},
           "stage_ms": stage, "extract_stage_ms": xst,
           "roofline": benchlib.fast_roofline(ex, w, h, xst, 2 * P * args.steps / max(1, calls))}
    if args.cpu_sample > 0 and world == 1:
        ns = min(args.cpu_sample, P)
        O.lib()
        S = sets[(it[0] - 1) % 2]                            # the last step's outputs
        dh, nh, mh, ih = S[1].cpu().numpy(), S[2].cpu().numpy(), S[3].cpu().numpy(), idx.cpu().numpy()
        t0 = time.perf_counter()
        bad = 0
        for p in range(ns):
            el, er = O.OracleExtractor(nf, 1.2, 8, 20, 7), O.OracleExtractor(nf, 1.2, 8, 20, 7)
            kl, dl, ml = el(left[p], lap)
            kr, dr, mr = er(right[p], lap)
            ri, _ = O.knn_match2(dl[ml:], dr[mr:])
            if nh[p] != len(kl) or not np.array_equal(ih[p, ml:nh[p]], np.where(ri >= 0, ri + mr, -1)):
                bad += 1
        fps = ns / (time.perf_counter() - t0)
        out["cpu_baseline"] = {"value": fps, "unit": "pairs/s", "cores": 1, "kind": "port",
                               "sample": f"first {ns} pairs: oracle extraction of L and R + knnMatch(2), one thread"}
        out["parity"] = {"pairs_checked": ns, "pairs_mismatched": bad}
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
