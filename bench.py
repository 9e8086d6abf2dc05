#!/usr/bin/env python3
"""Throughput bench of the ORB extract + match hot path on MI355X.

Metric (BASELINE.json): frames/s ORB extract+match (752x480, 1000 feat),
keypoints/descriptors bit-exact.  One step = one batch of B distinct
synthetic 752x480 frames of a panning camera (synth.global_sequence), resident in
HBM before the timed region; consecutive steps rotate through a ring of
--ring batches (default 4 x 256 frames = 370 MB, more than the 256 MB
Infinity Cache), so no step reads the frames the step before it read:
ORBextractor(1000, 1.2, 8, 20, 7) with vLappingArea {0, 1000} (Frame.cc:311)
on every frame, then ORBmatcher(0.9, true).SearchForInitialization(F[t],
F[t+1], prev = F[t] keypoints, window 100) on the B-1 consecutive pairs
(Tracking.cc:2459-2492).  Two steps are in flight (--overlap 2): consecutive steps alternate between two
extractor handles on two streams, so step k+1's pyramid and FAST run beside
step k's quadtree and describe, with four output sets in rotation.  Within
that, the matching of step k runs
on a second HIP stream while step k+1 extracts into a second output set,
started once step k+1's extraction has passed its pyramid stage
(orbx_set_stage_event; --sfi-after): its parallel top-K pass then runs beside
FAST and its latency-bound serial walk beside the quadtree and describe
(--no-pipeline serialises them); all K steps' work is inside the timed region.  Multi-GPU: one process per GPU, frames sharded
(weak scaling, no data-path collective); timing = max over ranks.

Extra objects on the JSON line:
  roofline     dominant kernel (k_fast_cells, the FAST pass) measured with HIP
               events on the extraction stream over a profiled pass after the
               timed region (--profile-steps, one step in flight: with two in
               flight each kernel shares the GPU with the other step's, so its
               launch time would not be its own; the timed steps carry no
               events);
               algorithmic bytes = every pyramid pixel read once
               (sum_l w_l*h_l per frame) x frames per launch.
               traffic = HBM bytes per launch of the same kernel from the committed
               rocprofv3 PMC summary (FETCH_SIZE x2 per the gfx950 note +
               WRITE_SIZE; tools/pmc_profile.sh, same command/config), and
               valu_roofline_frac = its VALU wave-instructions per launch (PMC)
               / (2 per CU per cycle x 256 CUs x the PMC clock x this run's
               launch time): the FAST pass is VALU-bound.
  stage_roofline  per stage (one kernel each): algorithmic bytes and their
               fraction of the HBM peak, the PMC bytes (FETCH_SIZE x2 +
               WRITE_SIZE of that kernel) over this run's launch time, and the
               VALU roofline fraction; the pyramid's algorithmic bytes are
               level 0 read once + levels 1..7 written once (sum(P)), with
               SURVEY §8(d)'s per-level figure (read P_0..P_6 + write
               P_1..P_7) beside it; describe's are the 43 x 43 raw patch read
               + 36 B written per keypoint; and the north-star pass (pyramid +
               FAST read bytes, R = 2*sum(P) - P_7 per frame).
  cpu_baseline the CPU oracle (oracle/, "port") on the host, rank 0, N=1,
               on a bounded sample of the same frames, threads stated; its
               outputs double as a parity check of the sampled frames.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

W, H, NFEAT, LAP = 752, 480, 1000, (0, 1000)
HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)
PMC_SUMMARY = ROOT / "profiles" / "pmc_summary_latest.csv"
METRIC = "frames/s ORB extract+match (752×480, 1000 feat) @1/2/4/8 GPU; bit-exact kp/desc"
STAGES = ["pyramid", "fast_cells", "quadtree", "describe", "assemble"]
STAGE_KERNEL = {"pyramid": "k_pyr_stream", "fast_cells": "k_fast_cells", "quadtree": "k_quadtree",
                "describe": "k_describe", "assemble": "k_assemble"}
PMC_FRAMES_PER_LAUNCH = 256     # tools/pmc_profile.sh runs the default config
CUS = 256
DESC_BYTES_PER_KP = 43 * 43 + 4 + 32   # k_describe: raw 43x43 patch read; angle + descriptor written


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without WORLD_SIZE in the environment bench.py starts them itself "
                         "under torch.distributed.run, with it WORLD_SIZE must equal --gpus")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="frames per step per GPU")
    ap.add_argument("--ring", type=int, default=4,
                    help="distinct input batches the steps rotate through (4 x 256 frames exceed the 256 MB "
                         "Infinity Cache, so every step reads cold frames)")
    ap.add_argument("--cpu-sample", type=int, default=256, help="frames in the CPU-baseline sample (0 = skip)")
    ap.add_argument("--parity-sample", type=int, default=4,
                    help="frames of every rank's last timed step checked against the oracle on its host when the "
                         "CPU baseline does not run (N > 1, or --cpu-sample 0); the mismatch counts are summed over "
                         "ranks onto rank 0's line")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the CPU-baseline pool (0 = the cores this process may run on, at most 16)")
    ap.add_argument("--no-host-api", dest="host_api", action="store_false",
                    help="skip the PCIe-inclusive drop-in latency leg")
    ap.add_argument("--no-profile", action="store_true", help="skip the profiled pass (no stage_ms / roofline)")
    ap.add_argument("--profile-steps", type=int, default=10,
                    help="steps of the profiled pass after the timed region: one step in flight, HIP events at "
                         "every stage boundary (the roofline's per-kernel launch times)")
    ap.add_argument("--pmc-summary", default=str(PMC_SUMMARY), help="rocprofv3 PMC summary (tools/pmc_summary.py)")
    ap.add_argument("--no-pipeline", dest="pipeline", action="store_false",
                    help="run SearchForInitialization on the extraction stream (no step overlap)")
    ap.add_argument("--streams", type=int, default=1, help="sub-batch streams per extractor (orbx_set_streams)")
    ap.add_argument("--overlap", type=int, default=2, choices=[1, 2],
                    help="batches in flight: 2 = consecutive steps alternate between two extractor handles "
                         "(own plan and scratch each) on two streams, so step k+1 extracts beside step k")
    ap.add_argument("--sfi-after", type=int, default=1,
                    help="pipeline: step k's SearchForInitialization waits until step k+1's extraction has passed this "
                         "stage (orbx_set_stage_event: 1 pyramid (default), 2 FAST, 3 quadtree; -1: starts at once)")
    ap.add_argument("--sets", type=int, default=4,
                    help="pipeline: output sets in rotation (2: step k+2 waits for step k's matching; "
                         "--overlap 2 wants 4)")
    ap.add_argument("--match-prio", type=int, default=0,
                    help="priority of the SearchForInitialization stream (torch.cuda.Stream priority: -1 = high)")
    ap.add_argument("--dump", default="", help="directory: each rank saves its last step's outputs (tests)")
    ap.add_argument("--workload", choices=["c2", "c3", "c4", "c5"], default="c2",
                    help="c2: the headline (this file); c3 stereo, c4 fisheye stereo (tools/bench_stereo.py), "
                         "c5 map-wide SearchByBoW (tools/bench_c5.py): one JSON line each, with its own roofline")
    ap.add_argument("--nkf", type=int, default=10000, help="c5: keyframes in the map")
    ap.add_argument("--per-kf", type=int, default=5000, help="c5: features per keyframe (of the query's ~5008)")
    ap.add_argument("--valid-frac", type=float, default=1.0,
                    help="c5: share of keyframe features with a valid MapPoint (the stated map: 1.0)")
    ap.add_argument("--near-frac", type=float, default=1.0,
                    help="c5: share of keyframes near the query (1.0: the stated map; 0.1: mostly far keyframes)")
    return ap.parse_args()


def other_workload(args):
    """BASELINE.json configs C3-C5 as their own JSON lines (not the headline)."""
    import types
    sys.path.insert(0, str(ROOT / "tools"))
    batch_given = any(a.startswith("--batch") for a in sys.argv)
    if args.workload in ("c3", "c4"):
        import bench_stereo
        a = types.SimpleNamespace(pairs=args.batch if batch_given else (128 if args.workload == "c3" else 64),
                                  steps=args.steps, warmup=args.warmup,
                                  cpu_sample=min(args.cpu_sample, 64 if args.workload == "c3" else 8),
                                  cpu_threads=args.cpu_threads or min(16, len(os.sched_getaffinity(0))),
                                  dump=args.dump)
        return bench_stereo.run_c3(a) if args.workload == "c3" else bench_stereo.run_c4(a)
    import bench_c5
    # the oracle checks every keyframe of rank 0's shard (a threaded map loop: a few seconds)
    a = types.SimpleNamespace(nkf=args.nkf, per_kf=args.per_kf, valid_frac=args.valid_frac, near_frac=args.near_frac,
                              reps=args.steps, warmup=args.warmup,
                              cpu_sample=-1 if args.cpu_sample > 0 else 0,
                              cpu_threads=args.cpu_threads or min(16, len(os.sched_getaffinity(0))))
    return bench_c5.run_c5(a)


def pmc_row(path, kernel):
    """Row of a tools/pmc_summary.py CSV for `kernel`, or None."""
    import csv
    try:
        with open(path) as fh:
            for row in csv.DictReader(fh):
                if kernel in row["kernel"]:
                    return row
    except OSError:
        pass
    return None


def level_sizes(ex):
    """Pixels of each pyramid level (ComputePyramid sizes, ORBextractor.cc:1174-1175)."""
    return [int(np.rint(np.float32(W) * np.float32(s))) * int(np.rint(np.float32(H) * np.float32(s)))
            for s in ex.GetInverseScaleFactors()]


def level_pixels(ex):
    return sum(level_sizes(ex))


def pmc_figures(row, ms, frames_per_launch):
    """PMC bytes and VALU roofline fraction of one kernel from its PMC summary
    row (per dispatch at PMC_FRAMES_PER_LAUNCH frames, scaled to this run's
    launch) over this run's launch time `ms`."""
    if not row or ms <= 0:
        return {}
    scale = frames_per_launch / PMC_FRAMES_PER_LAUNCH
    out = {}
    if row.get("fetch_MB_x2") and row.get("write_MB"):
        b = (float(row["fetch_MB_x2"]) + float(row["write_MB"])) * 1024 * 1024 * scale
        out["pmc_bytes_per_launch"] = b
        out["pmc_frac"] = b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS
    if row.get("valu_per_wave") and row.get("waves") and row.get("clock_GHz"):
        wi = float(row["valu_per_wave"]) * float(row["waves"]) * scale        # VALU wave-instructions per launch
        out["valu_roofline_frac"] = wi / (2 * CUS * float(row["clock_GHz"]) * 1e9 * ms * 1e-3)
    return out


def stage_roofline(ex, stage_ms, frames_per_launch, kps_per_frame, pmc_path):
    """Per stage: algorithmic bytes and their HBM fraction,
    PMC bytes and VALU fraction (pmc_figures).  Algorithmic bytes per frame:
    pyramid sum(P) (level 0 read once, levels 1..L-1 written once; SURVEY's
    per-level figure sum(P[:-1]) + sum(P[1:]) as survey_*), FAST sum(P) (every
    level pixel read once), describe (43 x 43 + 36) B per keypoint.  The
    north-star pass (pyramid + FAST) reads R = 2*sum(P) - P_{L-1} per frame."""
    P = level_sizes(ex)
    per_frame = {"pyramid": sum(P), "fast_cells": sum(P), "quadtree": None,
                 "describe": DESC_BYTES_PER_KP * kps_per_frame, "assemble": None}
    out = {}
    for k, b in per_frame.items():
        ms = float(stage_ms.get(k) or 0)
        if ms <= 0:
            continue
        e = {"kernel": STAGE_KERNEL[k], "ms": ms}
        if b is not None:
            gbs = b * frames_per_launch / (ms * 1e-3) / 1e9
            e.update({"bytes_per_launch": b * frames_per_launch, "achieved_GBs": gbs, "frac": gbs / HBM_PEAK_GBS})
        e.update(pmc_figures(pmc_row(pmc_path, STAGE_KERNEL[k]), ms, frames_per_launch))
        if k == "pyramid":
            sb = (sum(P[:-1]) + sum(P[1:])) * frames_per_launch
            e.update({"survey_bytes_per_launch": sb, "survey_frac": sb / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS})
        out[k] = e
    ms = float(stage_ms.get("pyramid") or 0) + float(stage_ms.get("fast_cells") or 0)
    if ms > 0:
        r = (2 * sum(P) - P[-1]) * frames_per_launch
        gbs = r / (ms * 1e-3) / 1e9
        out["north_star_pyramid_fast_read"] = {"bytes_per_launch": r, "ms": ms, "achieved_GBs": gbs,
                                               "frac": gbs / HBM_PEAK_GBS}
    return out


def cpu_baseline(frames_np, threads, lib_path):
    """The CPU oracle on the host: extraction + SearchForInitialization on the
    same consecutive pairs; frames spread over a pool of `threads` threads
    (ctypes releases the GIL).  Returns (frames/s, outputs, {pair: (nm, m12)})."""
    from oracle import oracle as O
    from orb_slam3_vio_fixes_amd import abi
    n = len(frames_np)
    exs = [O.OracleExtractor(NFEAT, 1.2, 8, 20, 7, lib_path=lib_path) for _ in range(threads)]
    outs = [None] * n

    def work(t):
        for i in range(t, n, threads):
            outs[i] = exs[t](frames_np[i], LAP)
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as pool:
        list(pool.map(work, range(threads)))

    def match(t):
        res = []
        for i in range(t, n - 1, threads):
            k1, d1, _ = outs[i]
            k2, d2, _ = outs[i + 1]
            prev = np.stack([k1["x"], k1["y"]], 1)
            nm, m12, _ = O.search_for_initialization(abi.frame_struct(k1, d1, W, H), abi.frame_struct(k2, d2, W, H),
                                                     prev, 100, 0.9, True, lib_path=lib_path)
            res.append((i, (nm, m12)))
        return res
    with ThreadPoolExecutor(threads) as pool:
        nms = dict(x for r in pool.map(match, range(threads)) for x in r)
    dt = time.perf_counter() - t0
    return n / dt, outs, nms


def parity_counts(snap, ns, outs, nms):
    """Mismatches of the first `ns` frames / `ns - 1` pairs of a device output
    snapshot (kps, desc, n, mono, nmatch, matches12) against the oracle's
    outputs `outs` / `nms` (cpu_baseline): every keypoint byte, descriptor,
    monoIndex, nmatches and the whole matches12 row."""
    from orb_slam3_vio_fixes_amd import orb
    kh, dh, nh, monoh, mh, m12h = (x.cpu().numpy() for x in snap)
    bad = 0
    for i in range(ns):
        rk, rd, rmono = outs[i]
        if nh[i] != len(rk) or monoh[i] != rmono or \
                not np.array_equal(orb.keypoints_from_device(kh[i][:nh[i]]).view(np.uint8), rk.view(np.uint8)) or \
                not np.array_equal(dh[i][:nh[i]], rd):
            bad += 1
    bad_m = 0
    for i in range(ns - 1):
        rnm, rm12 = nms[i]
        if mh[i] != rnm or not np.array_equal(m12h[i][:len(rm12)], rm12):
            bad_m += 1
    return bad, bad_m


def cpu_single_thread(frames_np, lib_path, seconds=4.0):
    """The reference's own threading model for a monocular stream: the
    Tracking thread extracts one image at a time (Frame.cc:418-425; a stereo
    frame runs its two images on two threads, Frame.cc:122-125) and matches it
    against the previous frame.  One thread, frames in order, for about
    `seconds`.  Returns (frames/s, frames done)."""
    from oracle import oracle as O
    from orb_slam3_vio_fixes_amd import abi
    ex = O.OracleExtractor(NFEAT, 1.2, 8, 20, 7, lib_path=lib_path)
    prev = None
    t0 = time.perf_counter()
    done = 0
    for img in frames_np:
        cur = ex(img, LAP)
        if prev is not None:
            k1, d1, _ = prev
            O.search_for_initialization(abi.frame_struct(k1, d1, W, H), abi.frame_struct(cur[0], cur[1], W, H),
                                        np.stack([k1["x"], k1["y"]], 1), 100, 0.9, True, lib_path=lib_path)
        prev = cur
        done += 1
        if time.perf_counter() - t0 > seconds:
            break
    return done / (time.perf_counter() - t0), done


def host_api_rates(frames_np, reps=200):
    """PCIe-inclusive rates of the Tracking thread's drop-in calls (host image
    in, host keypoints out): orbx_extract one image per call (Frame.cc:418-425)
    and orbx_extract_batch on a stereo pair per call (Frame.cc:122-125).  Not
    the metric (that is HBM-resident); the drop-in latency."""
    from orb_slam3_vio_fixes_amd import orb
    ex = orb.ORBextractor(NFEAT, 1.2, 8, 20, 7)
    imgs = [np.ascontiguousarray(f) for f in frames_np[:16]]
    for i in range(10):
        ex(imgs[i % len(imgs)], None, LAP)
    t0 = time.perf_counter()
    for i in range(reps):
        ex(imgs[i % len(imgs)], None, LAP)
    single = (time.perf_counter() - t0) / reps
    for i in range(5):
        ex.extract_batch([imgs[i % 16], imgs[(i + 1) % 16]], [LAP, LAP])
    t0 = time.perf_counter()
    for i in range(reps // 2):
        ex.extract_batch([imgs[i % 16], imgs[(i + 1) % 16]], [LAP, LAP])
    pair = (time.perf_counter() - t0) / (reps // 2)
    out = {"orbx_extract_ms": single * 1e3, "orbx_extract_frames_per_s": 1.0 / single,
           "orbx_extract_batch_stereo_pair_ms": pair * 1e3, "orbx_extract_batch_frames_per_s": 2.0 / pair,
           "calls": reps, "image": f"{W}x{H} u8, host memory, outputs copied back to host",
           "note": "PCIe-inclusive drop-in rate (one Tracking-thread call at a time); not the metric"}
    out["adapter"] = adapter_rates(frames_np[0], reps)
    return out


def adapter_rates(img, reps):
    """The drop-in ORBextractor adapter's true per-call cost (ORBextractor::
    operator() of adapters/orbslam3/ORBextractor.cc, compiled against the
    reference header into tests/native/bin/adapter_extractor by build()):
    with the eight mvImagePyramid host copies it makes by default, and with
    them off (ORBextractorSetHostPyramid: mono / RGB-D, or stereo matching on
    the device).  None when the binary was not built."""
    import subprocess
    import tempfile
    exe = ROOT / "tests" / "native" / "bin" / "adapter_extractor"
    if not exe.exists():
        return None
    with tempfile.TemporaryDirectory() as td:
        src = Path(td) / "img.u8"
        src.write_bytes(np.ascontiguousarray(img, np.uint8).tobytes())
        r = subprocess.run([str(exe), str(src), str(W), str(H), str(NFEAT), str(LAP[0]), str(LAP[1]), td, str(reps)],
                           capture_output=True, text=True, timeout=120)
        if r.returncode != 0:
            return {"error": r.stderr[-500:]}
        with_pyr, without, _ = (Path(td) / "time.txt").read_text().split()
    return {"ms_per_call_host_pyramid": float(with_pyr), "ms_per_call_no_host_pyramid": float(without),
            "frames_per_s_host_pyramid": 1e3 / float(with_pyr), "frames_per_s_no_host_pyramid": 1e3 / float(without),
            "calls": reps}


MATCHER_SEARCHES = ["search_for_initialization", "search_by_projection_last", "search_by_projection_mps",
                    "search_by_bow"]
MATCHER_OUT = {"search_for_initialization": "sfi", "search_by_projection_last": "last",
               "search_by_projection_mps": "mps", "search_by_bow": "bow"}
LATENCY_EXE = ROOT / "tests" / "native" / "bin" / "matcher_latency"


def matcher_inputs(frames_np, d):
    """The Tracking thread's per-frame matcher calls at their stated sizes,
    written as raw arrays into directory d for tests/native/matcher_latency:
    two consecutive 752x480 frames of the batch extracted by the GPU extractor
    (1000 features); SearchForInitialization(F1, F2); SearchByProjection(F2,
    LastFrame) with the last frame's ~1000 points projected onto F2's keypoints
    (1 px noise, 2 % descriptor bits flipped); SearchByProjection(F2, 3000
    local map points) (map points drawn from F2's keypoints, 2 px noise);
    SearchByBoW(KF = F1, F2) with level-2 vocabulary nodes (synthetic k = 10
    vocabulary) and 90 % of the keyframe's MapPoints valid."""
    from orb_slam3_vio_fixes_amd import abi, orb, synth
    d = Path(d)
    ex = orb.ORBextractor(NFEAT, 1.2, 8, 20, 7)
    k1, d1, _ = ex(np.ascontiguousarray(frames_np[0]), None, LAP)
    k2, d2, _ = ex(np.ascontiguousarray(frames_np[1]), None, LAP)
    rng = np.random.default_rng(11)
    meta = {"W": W, "H": H, "n1": len(k1), "n2": len(k2), "nlevels": 8}
    w = lambda name, a: np.ascontiguousarray(a).tofile(d / name)
    w("f1_kps.bin", k1.view(np.uint8)); w("f2_kps.bin", k2.view(np.uint8))
    w("f1_desc.bin", d1); w("f2_desc.bin", d2)
    w("scale.bin", np.asarray(ex.GetScaleFactors(), np.float32))
    # the last frame's points, projected near the current frame's keypoints
    nl = len(k2)
    flip = lambda a, p: np.where(rng.random(a.shape) < p, a ^ np.uint8(1 << int(rng.integers(0, 8))), a)
    w("last_valid.bin", (rng.random(nl) < 0.9).astype(np.uint8))
    w("last_u.bin", (k2["x"] + rng.normal(0, 1, nl)).astype(np.float32))
    w("last_v.bin", (k2["y"] + rng.normal(0, 1, nl)).astype(np.float32))
    w("last_ur.bin", np.full(nl, -1, np.float32))
    w("last_oct.bin", k2["octave"].astype(np.int32))
    w("last_ang.bin", ((k2["angle"] + rng.normal(0, 3, nl)) % 360).astype(np.float32))
    w("last_hobs.bin", np.ones(nl, np.uint8))
    w("last_desc.bin", flip(d2, 0.02))
    meta["nlast"] = nl
    # local map points
    nq = 3000
    src = rng.integers(0, len(k2), nq)
    qx = (k2["x"][src] + rng.normal(0, 2, nq)).astype(np.float32)
    w("mps_x.bin", qx); w("mps_y.bin", (k2["y"][src] + rng.normal(0, 2, nq)).astype(np.float32))
    w("mps_xr.bin", (qx - 20).astype(np.float32))
    w("mps_lvl.bin", k2["octave"][src].astype(np.int32))
    w("mps_vcos.bin", rng.uniform(0.99, 1.0, nq).astype(np.float32))
    w("mps_depth.bin", rng.uniform(0, 100, nq).astype(np.float32))
    w("mps_inview.bin", (rng.random(nq) < 0.9).astype(np.uint8))
    w("mps_hobs.bin", np.ones(nq, np.uint8))
    w("mps_desc.bin", flip(d2[src], 0.02))
    meta["nmps"] = nq
    # BoW: FeatureVectors at level 2 of a synthetic k = 10 vocabulary
    voc = abi.vocab_struct(synth.vocabulary(10, 3, seed=31))
    for tag, dd in (("fv1", d1), ("fv2", d2)):
        fv = abi.featvec_struct(orb.transform(voc, dd, 1)[2])
        node_ids, offsets, idx = fv.arrays
        w(f"{tag}_nodes.bin", node_ids); w(f"{tag}_off.bin", offsets); w(f"{tag}_idx.bin", idx)
        meta[f"{tag}_nodes"] = len(node_ids)
    w("kf_valid.bin", (rng.random(len(k1)) < 0.9).astype(np.uint8))
    (d / "meta.txt").write_text("".join(f"{k} {v}\n" for k, v in meta.items()))
    return {"frame_features": [len(k1), len(k2)], "last_frame_points": nl, "local_map_points": nq}


def run_latency(lib, prefix, d, reps):
    import subprocess
    r = subprocess.run([str(LATENCY_EXE), str(lib), prefix, str(d), str(reps)], capture_output=True, text=True,
                       timeout=300)
    if r.returncode != 0:
        raise RuntimeError(f"matcher_latency {prefix}: {r.stderr[-500:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


def host_api_matchers(frames_np, d, reps=200):
    """Per-call latency of the Tracking thread's matcher calls through the C
    ABI, from C++ (tests/native/matcher_latency: host inputs in, host outputs
    out, PCIe and every synchronisation included; no Python in the timed
    loop).  Not the metric: the drop-in latency."""
    from orb_slam3_vio_fixes_amd import capi
    if not LATENCY_EXE.exists():
        return None
    sizes = matcher_inputs(frames_np, d)
    gpu = run_latency(capi.LIB_PATH, "orbm", d, reps)
    return {"sizes": sizes, "calls": reps, "gpu": gpu,
            "note": "median per call from C++ through the C ABI, host arrays in and out (PCIe included)"}


def cpu_baseline_matchers(d, blk, reps=200):
    """CPU leg of host_api.matchers: the oracle's same entry points, one
    thread (the reference's per-call model), same inputs and harness; the
    outputs of every search compared with the GPU's (parity)."""
    from oracle import oracle as O
    lib_path, flags = O.fast_variant()
    cpu = run_latency(lib_path, "orbo", d, reps)
    blk["cpu_1thread"] = cpu
    blk["speedup_vs_1thread"] = {k: cpu[k]["median_us"] / blk["gpu"][k]["median_us"] for k in MATCHER_SEARCHES}
    same = lambda a, b: bool(np.array_equal(np.fromfile(Path(d) / a, np.int32), np.fromfile(Path(d) / b, np.int32)))
    blk["parity"] = {k: same(f"orbm_{MATCHER_OUT[k]}.bin", f"orbo_{MATCHER_OUT[k]}.bin") for k in MATCHER_SEARCHES}
    # the dframe forms (frames resident in HBM: the Tracking thread's frame as
    # the extraction leaves it, the keyframe since its creation)
    if all(f"{k}_dframe" in blk["gpu"] for k in MATCHER_SEARCHES):
        blk["speedup_vs_1thread_dframe"] = {k: cpu[k]["median_us"] / blk["gpu"][f"{k}_dframe"]["median_us"]
                                            for k in MATCHER_SEARCHES}
        blk["parity_dframe"] = {k: same(f"orbm_{MATCHER_OUT[k]}_dframe.bin", f"orbo_{MATCHER_OUT[k]}.bin")
                                for k in MATCHER_SEARCHES}
    blk["cpu_flags"] = flags


def main():
    args = parse()
    # --gpus N without a launcher: start N ranks as one child process (no
    # torch import, no GPU call in this process) and exit with its code
    from orb_slam3_vio_fixes_amd import launch
    rc = launch.ensure_ranks(args.gpus, __file__, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    if args.workload != "c2":
        res = other_workload(args)
        if res is not None:
            print(json.dumps(res), flush=True)
        return
    import torch
    import torch.distributed as dist
    from orb_slam3_vio_fixes_amd import capi, orb, synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # one process per GPU; the modulo only matters when rehearsing several
    # ranks on fewer GPUs (ORB_BENCH_BACKEND=gloo)
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    backend = os.environ.get("ORB_BENCH_BACKEND", "nccl")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    B = args.batch

    # distinct frames per rank (weak scaling), generated once, uploaded before
    # timing.  Seam halo: every rank but the last also
    # extracts the next rank's first frame, so SearchForInitialization covers
    # the pair across each shard seam and the job matches all N*B-1 pairs
    # with no data-path collective; the halo frame is not counted in `value`.
    Bx = B + (1 if rank < world - 1 else 0)
    # ring batch j of rank r holds global frames (j*world + r)*B ...: every
    # frame of the job is distinct, and the seam halo of batch j is frame 0
    # of rank r+1's batch j
    R = max(1, args.ring)
    ring_first = [(j * world + rank) * B for j in range(R)]
    ring_np = [synth.global_sequence(W, H, f0, Bx, config=2) for f0 in ring_first]
    ring = [torch.from_numpy(a).to(dev) for a in ring_np]
    frames_np, frames = ring_np[0], ring[0]
    exs = [orb.ORBextractor(NFEAT, 1.2, 8, 20, 7, device=local) for _ in range(args.overlap)]
    ex = exs[0]
    L = capi.lib()
    for e in exs:
        capi.check(L.orbx_set_streams(e._h, args.streams), "orbx_set_streams")
    stream = torch.cuda.current_stream(dev)
    # extraction stream of each handle (--overlap 2: the second on its own stream)
    xstreams = [stream] + [torch.cuda.Stream(dev) for _ in range(args.overlap - 1)]
    kps, desc, n, mono, cap = ex.extract_batch_device(frames, LAP)
    # --sets output sets (default 2): SearchForInitialization of step k runs on
    # its own stream while step k+1 extracts into another set; with more sets
    # step k+2 does not wait for step k's matching either (measured: no gain
    # at --overlap 1; --overlap 2 wants 4) (--no-pipeline: both on the
    # extraction stream)
    nsets = max(2, args.sets)
    outs = [(kps, desc, n, mono)] + [tuple(torch.empty_like(x) for x in (kps, desc, n, mono))
                                     for _ in range(nsets - 1)]
    outs_dev = outs
    # the matching stream at a higher priority (--match-prio -1): its kernels
    # are dispatched ahead of the extraction's as CUs free up, instead of
    # waiting for LDS behind a stream of small extraction blocks
    mstream = torch.cuda.Stream(dev, priority=args.match_prio) if args.pipeline else stream
    done = [None] * nsets                # match of set i finished (recorded on mstream)
    matches = torch.empty((Bx - 1, cap), dtype=torch.int32, device=dev)
    nmatch = torch.empty(Bx - 1, dtype=torch.int32, device=dev)
    inv_w = float(np.float32(64) / np.float32(W))
    inv_h = float(np.float32(48) / np.float32(H))

    match_events = []
    counter = [0]

    # --sfi-after k: the library records a per-set event when the extraction
    # passes stage k, and step k's matching is enqueued behind step k+1's
    # event, so it runs beside the latency-bound later stages, not beside FAST
    stage_ev = [None] * nsets
    if args.pipeline and args.sfi_after >= 0:
        for j in range(nsets):
            stage_ev[j] = torch.cuda.Event()
            stage_ev[j].record(stream)                  # creates the event
    pending = []                                        # (set, extracted event) whose match is not enqueued yet

    def match(i, extracted, after=None, timed=False):
        k_, d_, n_, m_ = outs[i]
        mstream.wait_event(extracted)
        if after is not None:
            mstream.wait_event(after)
        if timed:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(mstream)
        rc = L.orbm_search_for_initialization_batch_device(
            Bx, k_.data_ptr(), d_.data_ptr(), n_.data_ptr(), cap, 0.0, float(W), 0.0, float(H), inv_w, inv_h,
            100, 0.9, 1, matches.data_ptr(), nmatch.data_ptr(), mstream.cuda_stream)
        capi.check(rc, "SearchForInitialization batch")
        if timed:
            e1.record(mstream)
            match_events.append((e0, e1))
        done[i] = torch.cuda.Event()
        done[i].record(mstream)

    def step(timed=False, handle=None):
        i = counter[0] % nsets
        # --overlap 2: consecutive steps alternate handles (the profiled pass
        # pins handle 0: one step in flight)
        h = counter[0] % args.overlap if handle is None else handle
        frames = ring[counter[0] % R]                   # a different input batch than the step before
        counter[0] += 1
        k_, d_, n_, m_ = outs[i]
        xe, xs = exs[h], xstreams[h]
        if done[i] is not None:
            xs.wait_event(done[i])       # the match that read this set has finished
        if stage_ev[i] is not None:
            capi.check(L.orbx_set_stage_event(xe._h, args.sfi_after, stage_ev[i].cuda_event), "stage event")
        xe.extract_batch_device(frames, LAP, out=(k_, d_, n_, m_), stream=xs)
        extracted = torch.cuda.Event()
        extracted.record(xs)
        if stage_ev[i] is None:
            match(i, extracted, timed=timed)
            return
        while pending:                                  # the previous step's match, behind this step's stage
            pi, pev = pending.pop()
            match(pi, pev, after=stage_ev[i], timed=timed)
        pending.append((i, extracted))

    def flush(timed=False):
        while pending:
            pi, pev = pending.pop()
            match(pi, pev, timed=timed)

    for _ in range(args.warmup):
        step()
    flush()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # the timed steps carry no instrumentation: per-kernel times come from
    # the profiled pass below
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    flush()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # the last TIMED step's outputs (its output set, its ring batch and its
    # matching, which the final flush ran last), copied before the profiled
    # pass reuses the sets: the parity legs below check these
    snap_set, snap_slot = (counter[0] - 1) % nsets, (counter[0] - 1) % R
    own_cpu = world == 1 and args.cpu_sample > 0
    ns_snap = max(1, min(Bx, min(args.cpu_sample, B) if own_cpu else args.parity_sample))
    snap = tuple(x[:ns_snap].clone() for x in outs_dev[snap_set]) + \
        (nmatch[:ns_snap - 1].clone(), matches[:ns_snap - 1].clone())
    torch.cuda.synchronize()
    # profiled pass (after the timed region, not in `value`): --profile-steps
    # more steps of the same pipeline at ONE step in flight (handle 0 only;
    # step k's matching still beside step k+1's later stages), with HIP events
    # at every stage boundary on the extraction stream, so each kernel's
    # launch time is its own and not shared with the other handle's step
    stage_ms = np.zeros(len(STAGES), np.float32)
    prof = not args.no_profile and args.profile_steps > 0
    frames_per_launch = Bx
    if prof:
        for e in exs:
            L.orbx_set_profiling(e._h, 1)
        for _ in range(args.profile_steps):
            step(timed=True, handle=0)
        flush(timed=True)
        torch.cuda.synchronize()
        calls = 0
        for e in exs:
            sm = np.zeros(len(STAGES), np.float32)
            calls += L.orbx_get_profile(e._h, sm.ctypes.data, len(STAGES))
            L.orbx_set_profiling(e._h, 0)
            stage_ms += sm
        stage_ms /= max(1, calls)
        frames_per_launch = Bx * args.profile_steps / max(1, calls)  # each sub-batch range is one launch per stage
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    # every rank's own sample of its last timed step vs the oracle on its host
    # (N > 1, or no CPU baseline), the counts summed over ranks
    par = None
    if not own_cpu and args.parity_sample > 0:
        from oracle import oracle as O
        lib_path, _ = O.fast_variant()
        _, ro, rn = cpu_baseline(ring_np[snap_slot][:ns_snap], min(4, len(os.sched_getaffinity(0))), lib_path)
        bad, bad_m = parity_counts(snap, ns_snap, ro, rn)
        pt = torch.tensor([ns_snap, bad, ns_snap - 1, bad_m], dtype=torch.int64,
                          device=dev if backend == "nccl" else "cpu")
        if world > 1:
            dist.all_reduce(pt, op=dist.ReduceOp.SUM)
        fc, fm, pc, pm = (int(x) for x in pt.tolist())
        par = {"frames_checked": fc, "frames_mismatched": fm, "pairs_checked": pc, "pairs_mismatched": pm,
               "ranks": world, "source": f"first {ns_snap} frames / {ns_snap - 1} pairs of every rank's last timed "
                                         "step, oracle on the rank's host, counts summed over ranks",
               "compared": "keypoint count, all 28 keypoint bytes, 32 descriptor bytes, monoIndex, nmatches and the "
                           "full matches12"}

    last_slot = (counter[0] - 1) % R                    # the ring batch of the last step
    if args.dump:
        # the last step's outputs of this rank, with global frame / pair indices
        last = outs_dev[(counter[0] - 1) % nsets]
        Path(args.dump).mkdir(parents=True, exist_ok=True)
        np.savez(Path(args.dump) / f"rank{rank}.npz", first=ring_first[last_slot], frames=Bx, world=world,
                 kps=last[0].cpu().numpy(), desc=last[1].cpu().numpy(), n=last[2].cpu().numpy(),
                 mono=last[3].cpu().numpy(), nmatch=nmatch.cpu().numpy(), matches=matches.cpu().numpy())
    if rank == 0:
        total_frames = B * args.steps * world
        value = total_frames / elapsed
        # the roofline names the longest extraction kernel with algorithmic
        # bytes (the FAST pass or describe; stage_roofline has every stage)
        sr = stage_roofline(ex, dict(zip(STAGES, map(float, stage_ms))), frames_per_launch,
                            float(n.float().mean().item()), args.pmc_summary)
        dom = max(("fast_cells", "describe"), key=lambda k_: sr.get(k_, {}).get("ms", 0.0))
        d_ = sr.get(dom, {})
        roof = {"kernel": STAGE_KERNEL[dom], "bound": "hbm", "achieved": d_.get("achieved_GBs"), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": d_.get("frac"), "traffic": d_.get("pmc_bytes_per_launch"),
                "bytes_per_launch": d_.get("bytes_per_launch"), "ms_per_launch": d_.get("ms"),
                "frames_per_launch": frames_per_launch,
                "bytes_per_unit": ("sum of the pyramid level sizes per frame (every level pixel read once)"
                                   if dom == "fast_cells" else
                                   f"{DESC_BYTES_PER_KP} B per keypoint (43x43 raw patch read, angle + descriptor "
                                   "written)"),
                "traffic_source": (os.path.relpath(args.pmc_summary, ROOT) if d_.get("pmc_bytes_per_launch") else None),
                "time_source": (f"HIP events on the extraction stream over a profiled pass of {args.profile_steps} "
                                "steps after the timed region, one step in flight (the timed steps run "
                                f"{args.overlap} in flight, uninstrumented)"),
                "valu_roofline_frac": d_.get("valu_roofline_frac"),
                "second": {k_: sr.get(k_, {}).get("frac") for k_ in ("fast_cells", "describe") if k_ != dom}}
        out = {"metric": METRIC, "value": value, "unit": "frames/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
               "config": {"workload": "C2: 752x480 mono, ORBextractor(1000,1.2,8,20,7), lapping {0,1000}, "
                                      "+ SearchForInitialization(window 100, 0.9, checkOri) on consecutive frames",
                          "frames_per_step_per_gpu": B, "input_ring_batches": R,
                          "input_ring_MB": round(R * Bx * W * H / 2**20, 1), "streams": args.streams, "overlap": args.overlap,
                          "steps_in_flight": args.overlap, "pipeline": args.pipeline,
                          "profiled_pass_steps": args.profile_steps if prof else 0,
                          "sfi_after_stage": args.sfi_after if args.pipeline else None,
                          "output_sets": nsets if args.pipeline else 1,
                          "parallelism": f"frames sharded over {world} GPU(s), halo frame per seam"},
               "stage_ms": {**{k: float(v) for k, v in zip(STAGES, stage_ms)},
                            "search_for_initialization": (float(np.mean([a.elapsed_time(b) for a, b in match_events]))
                                                          if match_events else None)},
               "roofline": roof,
               "stage_roofline": sr,
               "world_size": dist.get_world_size() if world > 1 else 1,
               "backend": dist.get_backend() if world > 1 else None}
        if par is not None:
            out["parity"] = par
        if own_cpu:
            from oracle import oracle as O
            ns = ns_snap
            avail = len(os.sched_getaffinity(0))
            threads = args.cpu_threads or min(16, avail)
            lib_path, flags = O.fast_variant()
            frames_np = ring_np[snap_slot]             # the frames of the last timed step
            fps, outs, nms = cpu_baseline(frames_np[:ns], threads, lib_path)
            fps1, n1 = cpu_single_thread(frames_np[:ns], lib_path)
            # parity of the sampled frames (the CPU leg doubles as a checker)
            # against the snapshot of the last timed step (two in flight)
            bad, bad_m = parity_counts(snap, ns, outs, nms)
            nproc = os.cpu_count() or avail
            out["cpu_baseline"] = {"value": fps, "unit": "frames/s", "cores": threads, "kind": "port",
                                   "cores_available": avail, "host_cpus_nproc": nproc,
                                   "cores_note": ("all host cores this job may use: the pool's per-GPU CPU share "
                                                  f"({threads} threads; nproc reports {nproc} on the shared host). "
                                                  "all_cores_linear_estimate scales the measured per-thread rate to "
                                                  "nproc -- an upper bound, not a measurement"),
                                   "per_thread_fps": fps / threads,
                                   "all_cores_linear_estimate": fps / threads * nproc, "flags": flags,
                                   "library": os.path.relpath(lib_path, ROOT),
                                   "single_thread_fps": fps1, "single_thread_frames": n1,
                                   "sample": f"first {ns} frames of the step batch: extraction + SearchForInitialization "
                                             f"on {ns - 1} consecutive pairs by the oracle on a pool of {threads} "
                                             f"threads (value); single_thread_fps: the reference's model, one "
                                             f"Tracking thread extracting and matching frame after frame"}
            out["parity"] = {"frames_checked": ns, "frames_mismatched": bad, "pairs_checked": ns - 1,
                             "pairs_mismatched": bad_m, "ranks": 1,
                             "source": f"first {ns} frames / {ns - 1} pairs of the last timed step ({args.overlap} "
                                       "in flight), the CPU-baseline outputs",
                             "compared": "keypoint count, all 28 keypoint bytes, 32 descriptor "
                                         "bytes, monoIndex, nmatches and the full matches12"}
        if world == 1 and args.host_api:
            # side measurements (not the metric): a failure here is reported in
            # the line instead of losing it
            try:
                out["host_api"] = host_api_rates(frames_np)
            except Exception as e:          # noqa: BLE001
                out["host_api"] = {"error": f"{type(e).__name__}: {e}"[:300]}
            import tempfile
            with tempfile.TemporaryDirectory() as td:
                try:
                    mb = host_api_matchers(ring_np[0][:2], td)
                    if mb is not None and args.cpu_sample > 0:
                        cpu_baseline_matchers(td, mb)
                except Exception as e:      # noqa: BLE001
                    mb = {"error": f"{type(e).__name__}: {e}"[:300]}
                out["host_api"]["matchers"] = mb
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
