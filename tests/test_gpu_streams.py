"""orbx_set_streams: a batch split into frame ranges on private streams gives
exactly the single-stream results (and the oracle's)."""
import numpy as np
import pytest

from oracle import oracle as O
from orb_slam3_vio_fixes_amd import capi, orb, synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nsub", [2, 3])
def test_sub_batch_streams_identical(gpu_lib, nsub):
    import torch
    frames_np = synth.sequence(752, 480, 70, config=2, start=900)
    frames = torch.from_numpy(frames_np).cuda()
    ex1 = orb.ORBextractor(1000, 1.2, 8, 20, 7)
    exs = orb.ORBextractor(1000, 1.2, 8, 20, 7)
    capi.check(capi.lib().orbx_set_streams(exs._h, nsub), "orbx_set_streams")
    a = ex1.extract_batch_device(frames, (0, 1000))
    b = exs.extract_batch_device(frames, (0, 1000))
    torch.cuda.synchronize()
    n = a[2].cpu().numpy()
    assert np.array_equal(n, b[2].cpu().numpy())
    assert np.array_equal(a[3].cpu().numpy(), b[3].cpu().numpy())
    ka, kb = a[0].cpu().numpy(), b[0].cpu().numpy()
    da, db = a[1].cpu().numpy(), b[1].cpu().numpy()
    for i in range(len(n)):
        assert np.array_equal(ka[i, :n[i]], kb[i, :n[i]])
        assert np.array_equal(da[i, :n[i]], db[i, :n[i]])
    # the last frame of the last range against the oracle
    rk, rd, rm = O.OracleExtractor(1000, 1.2, 8, 20, 7)(frames_np[-1], (0, 1000))
    assert np.array_equal(orb.keypoints_from_device(ka[-1, :n[-1]]).view(np.uint8), rk.view(np.uint8))
    assert np.array_equal(db[-1, :n[-1]], rd)


def test_batched_search_scratch_beyond_lru_and_release(gpu_lib):
    """Both batched searches with per-stream scratch (SearchForInitialization
    over a device batch, map-wide SearchByBoW) on more streams than the
    scratch LRU keeps (kScratchSets = 16 sets: 20 streams x 2 kinds = 40), so
    sets are evicted -- each after an event wait on its own stream, not a
    device synchronisation -- while the other streams' work is in flight.
    Every stream's results equal the default stream's.  Then
    orbm_release_scratch(stream, 0) for one stream and (NULL, 1) for all, and a
    rerun on a fresh stream gives the same results again."""
    import ctypes as C
    import torch
    from orb_slam3_vio_fixes_amd import kfmap
    L = capi.lib()
    W, H = 752, 480
    frames = torch.from_numpy(synth.sequence(W, H, 6, config=2, start=1300)).cuda()
    ex = orb.ORBextractor(1000, 1.2, 8, 20, 7)
    kps, desc, n, mono, cap = ex.extract_batch_device(frames, (0, 1000))
    inv_w, inv_h = float(np.float32(64) / np.float32(W)), float(np.float32(48) / np.float32(H))
    # a small keyframe map from frame 0's features (host oracle-free: results are
    # compared across streams; the map search itself is pinned in test_gpu_c5)
    k0 = orb.keypoints_from_device(kps[0, :int(n[0])].cpu().numpy())
    d0 = desc[0, :int(n[0])].cpu().numpy()
    rng = np.random.default_rng(3)
    nid = rng.integers(0, 40, len(k0)).astype(np.int32)
    kfs = []
    for i in range(6):
        sel = np.sort(rng.choice(len(k0), size=len(k0) * 3 // 4, replace=False))
        kd = d0[sel].copy()
        kd[rng.random(kd.shape) < 0.05] ^= np.uint8(0x04)
        kfs.append((k0[sel].copy(), kd, (rng.random(len(sel)) < 0.9).astype(np.uint8), nid[sel]))
    m = kfmap.DeviceKeyframeMap(kfs)
    # one prepared query frame (own output rows) per run
    frs = [m.prepare_frame(k0, d0, nid) for _ in range(22)]
    torch.cuda.synchronize()

    def run(stream):
        fr = frs.pop()
        with torch.cuda.stream(stream):
            mt = torch.full((5, cap), -7, dtype=torch.int32, device="cuda")
            nm = torch.zeros(5, dtype=torch.int32, device="cuda")
            capi.check(L.orbm_search_for_initialization_batch_device(
                6, kps.data_ptr(), desc.data_ptr(), n.data_ptr(), cap, 0.0, float(W), 0.0, float(H), inv_w, inv_h,
                100, 0.9, 1, mt.data_ptr(), nm.data_ptr(), stream.cuda_stream), "sfi batch")
            bm, bn = m.search_prepared(fr, 0.75, True, stream=stream)
        return mt, nm, bm, bn

    torch.cuda.synchronize()
    ref = [x.cpu().numpy() for x in run(torch.cuda.current_stream())]
    torch.cuda.synchronize()
    assert ref[1].min() > 50 and ref[3].min() > 50
    streams = [torch.cuda.Stream() for _ in range(20)]
    outs = [run(s) for s in streams]              # issued back to back: evictions while others run
    torch.cuda.synchronize()
    for o in outs:
        for a, b in zip(ref, o):
            assert np.array_equal(a, b.cpu().numpy())
    capi.check(L.orbm_release_scratch(C.c_void_p(streams[3].cuda_stream), 0), "release one")
    capi.check(L.orbm_release_scratch(None, 1), "release all")
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    again = run(s)
    torch.cuda.synchronize()
    for a, b in zip(ref, again):
        assert np.array_equal(a, b.cpu().numpy())
    capi.check(L.orbm_release_scratch(C.c_void_p(s.cuda_stream), 0), "release fresh")
