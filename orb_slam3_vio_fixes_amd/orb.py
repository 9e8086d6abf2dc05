"""Host-side mirror of the reference interface for the ORB hot path.

``ORBextractor`` follows ORB_SLAM3::ORBextractor (reference
include/ORBextractor.h:43-109): same constructor arguments, ``__call__`` ==
``operator()(image, mask, keypoints, descriptors, vLappingArea)`` returning
(keypoints, descriptors, monoIndex), the scale-table getters and
``mvImagePyramid``.  ``ORBmatcher`` follows include/ORBmatcher.h:36-103
(nnratio, checkOri, the Search* entry points, DescriptorDistance).  Every
call goes through the C ABI of liborb_mi355x.so onto the GPU; there is no
CPU path.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi, capi


class ORBextractor:
    HARRIS_SCORE, FAST_SCORE = 0, 1

    def __init__(self, nfeatures: int, scaleFactor: float, nlevels: int, iniThFAST: int, minThFAST: int,
                 device: int = 0, blur_variant: int = 0, fma_sampling: int = 1):
        self._p = abi.params(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, blur_variant, fma_sampling)
        self.nlevels = nlevels
        self.scaleFactor = float(np.float32(scaleFactor))
        self._h = capi.lib().orbx_create(C.byref(self._p), device)
        if not self._h:
            raise RuntimeError("orbx_create failed (bad parameters or no HIP device)")
        L = nlevels
        self._tab = [np.zeros(L, np.float32) for _ in range(4)] + [np.zeros(L, np.int32), np.zeros(16, np.int32)]
        capi.check(capi.lib().orbx_get_tables(self._h, *[abi.ptr(a) for a in self._tab]), "orbx_get_tables")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            capi.lib().orbx_destroy(h)
            self._h = None

    # getters (ORBextractor.h:61-81)
    def GetLevels(self): return self.nlevels
    def GetScaleFactor(self): return self.scaleFactor
    def GetScaleFactors(self): return self._tab[0].copy()
    def GetInverseScaleFactors(self): return self._tab[1].copy()
    def GetScaleSigmaSquares(self): return self._tab[2].copy()
    def GetInverseScaleSigmaSquares(self): return self._tab[3].copy()
    def FeaturesPerLevel(self): return self._tab[4].copy()
    def UMax(self): return self._tab[5].copy()

    def set_pyramid_mode(self, mode: int) -> None:
        """0 auto, 1 row bands (k_pyramid), 2 sliding frame (k_pyr_stream)."""
        capi.check(capi.lib().orbx_set_pyramid_mode(self._h, mode), "orbx_set_pyramid_mode")

    def set_host_pyramid(self, enable: bool) -> None:
        """orbx_set_host_pyramid: later extractions also download their pyramid
        (mvImagePyramid then reads host memory)."""
        capi.check(capi.lib().orbx_set_host_pyramid(self._h, int(enable)), "orbx_set_host_pyramid")

    def pyramid_kernel(self) -> int:
        """Pyramid kernel of the last extraction: 1 k_pyramid, 2 k_pyr_stream."""
        return int(capi.lib().orbx_pyramid_kernel(self._h))

    def max_keypoints(self, w: int, h: int) -> int:
        return capi.check(capi.lib().orbx_max_keypoints(self._h, w, h), "orbx_max_keypoints")

    def __call__(self, image: np.ndarray, mask=None, vLappingArea=(0, 0)):
        """operator() (ORBextractor.cc:1086-1168): returns (keypoints, descriptors, monoIndex);
        -1 for an empty image like the reference."""
        if image is None or image.size == 0:
            return np.zeros(0, abi.KEYPOINT_DTYPE), np.zeros((0, 32), np.uint8), -1
        img = np.ascontiguousarray(image, np.uint8)
        if img.ndim != 2:
            raise ValueError("ORBextractor expects an 8UC1 image")
        h, w = img.shape
        cap = self.max_keypoints(w, h)
        kps = np.zeros(cap, abi.KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n, mono = C.c_int(0), C.c_int(0)
        rc = capi.lib().orbx_extract(self._h, abi.ptr(img), w, h, w, int(vLappingArea[0]), int(vLappingArea[1]),
                                     abi.ptr(kps), abi.ptr(desc), cap, C.byref(n), C.byref(mono))
        capi.check(rc, "orbx_extract")
        return kps[:n.value].copy(), desc[:n.value].copy(), mono.value

    def extract_batch(self, images, laps=None):
        """operator() on several images of one size in one call (orbx_extract_batch):
        a list of (keypoints, descriptors, monoIndex)."""
        # row-strided 8UC1 views are passed as they are (cv::Mat::step)
        imgs = [im if (isinstance(im, np.ndarray) and im.dtype == np.uint8 and im.ndim == 2 and im.strides[1] == 1
                       and im.strides[0] >= im.shape[1]) else np.ascontiguousarray(im, np.uint8) for im in images]
        if not imgs:
            return []
        h, w = imgs[0].shape
        if any(im.ndim != 2 or im.shape != (h, w) for im in imgs):
            raise ValueError("extract_batch expects 8UC1 images of one size")
        nf = len(imgs)
        ptrs = (C.c_void_p * nf)(*[im.ctypes.data for im in imgs])
        steps = np.array([im.strides[0] for im in imgs], np.uintp)
        lap = None if laps is None else np.ascontiguousarray(np.asarray(laps, np.int32).reshape(nf, 2))
        cap = self.max_keypoints(w, h)
        kps = np.zeros((nf, cap), abi.KEYPOINT_DTYPE)
        desc = np.zeros((nf, cap, 32), np.uint8)
        n = np.zeros(nf, np.int32)
        mono = np.zeros(nf, np.int32)
        rc = capi.lib().orbx_extract_batch(self._h, nf, ptrs, abi.ptr(steps), w, h, abi.ptr(lap), abi.ptr(kps), abi.ptr(desc),
                                           cap, abi.ptr(n), abi.ptr(mono))
        capi.check(rc, "orbx_extract_batch")
        return [(kps[f, :n[f]].copy(), desc[f, :n[f]].copy(), int(mono[f])) for f in range(nf)]

    @property
    def mvImagePyramid(self):
        out = []
        for l in range(self.nlevels):
            w, h = C.c_int(0), C.c_int(0)
            capi.check(capi.lib().orbx_get_level(self._h, l, None, 0, C.byref(w), C.byref(h)), "orbx_get_level")
            a = np.zeros((h.value, w.value), np.uint8)
            capi.check(capi.lib().orbx_get_level(self._h, l, abi.ptr(a), w.value, C.byref(w), C.byref(h)),
                       "orbx_get_level")
            out.append(a)
        return out

    def batch_pyramid(self, frame: int):
        """mvImagePyramid of frame `frame` of the last batch call (orbx_get_batch_level)."""
        out = []
        for l in range(self.nlevels):
            w, h = C.c_int(0), C.c_int(0)
            capi.check(capi.lib().orbx_get_batch_level(self._h, frame, l, None, 0, C.byref(w), C.byref(h)),
                       "orbx_get_batch_level")
            a = np.zeros((h.value, w.value), np.uint8)
            capi.check(capi.lib().orbx_get_batch_level(self._h, frame, l, abi.ptr(a), w.value, C.byref(w),
                                                       C.byref(h)), "orbx_get_batch_level")
            out.append(a)
        return out

    def plan_info(self, w: int, h: int) -> dict:
        """orbx_debug_plan_info: the k_pyr_stream / FAST plan for a w x h image."""
        info = np.zeros(8, np.int32)
        capi.check(capi.lib().orbx_debug_plan_info(self._h, w, h, abi.ptr(info), 8), "orbx_debug_plan_info")
        keys = ["stream", "pretest", "K0", "nsteps", "lds_bytes", "entries", "ncells", "bm_ok"]
        return dict(zip(keys, (int(x) for x in info)))

    def debug_pretest(self, frame: int, level: int):
        """k_pyr_stream's fused FAST pre-test bitmap of (frame, level) of the
        last batch call (orbx_debug_pretest) as a bool array (h, w), and the
        window union (y0, y1, x0, x1) inside which it is defined."""
        win = np.zeros(6, np.int32)
        capi.check(capi.lib().orbx_debug_pretest(self._h, frame, level, None, 0, abi.ptr(win)), "orbx_debug_pretest")
        nb, h = int(win[4]), int(win[5])
        raw = np.zeros((h, nb), np.uint8)
        capi.check(capi.lib().orbx_debug_pretest(self._h, frame, level, abi.ptr(raw), nb, None), "orbx_debug_pretest")
        bits = np.unpackbits(raw, axis=1, bitorder="little")
        return bits.astype(bool), tuple(int(x) for x in win[:4])

    def debug_stage(self, stage: int, cap: int = 400000):
        kps = np.zeros(cap, abi.KEYPOINT_DTYPE)
        counts = np.zeros(self.nlevels, np.int32)
        n = capi.check(capi.lib().orbx_debug_stage(self._h, stage, abi.ptr(kps), cap, abi.ptr(counts)),
                       "orbx_debug_stage")
        out, off = [], 0
        for c in counts[:self.nlevels]:
            out.append(kps[off:off + c].copy())
            off += c
        assert off == n
        return out

    def extract_batch_device(self, frames, lapping=(0, 1000), out=None, stream=None):
        """HBM-resident batch path: ``frames`` is a (B, H, W) uint8 CUDA tensor.
        Returns (kps (B, cap) as a raw int32 tensor view, desc (B, cap, 32),
        n (B,), mono (B,))."""
        import torch
        assert frames.is_cuda and frames.dtype == torch.uint8 and frames.dim() == 3
        frames = frames.contiguous()
        B, H, W = frames.shape
        cap = self.max_keypoints(W, H)
        if out is None:
            dev = frames.device
            out = (torch.empty((B, cap, 7), dtype=torch.int32, device=dev),
                   torch.empty((B, cap, 32), dtype=torch.uint8, device=dev),
                   torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, dtype=torch.int32, device=dev))
        kps, desc, n, mono = out
        st = stream.cuda_stream if stream is not None else torch.cuda.current_stream().cuda_stream
        rc = capi.lib().orbx_extract_batch_device(self._h, B, frames.data_ptr(), H * W, W, W, H, int(lapping[0]),
                                                  int(lapping[1]), kps.data_ptr(), desc.data_ptr(), cap,
                                                  n.data_ptr(), mono.data_ptr(), C.c_void_p(st))
        capi.check(rc, "orbx_extract_batch_device")
        return kps, desc, n, mono, cap


def ComputeStereoMatches(ex_left: ORBextractor, ex_right: ORBextractor, mvKeys, mDescriptors, mvKeysRight,
                         mDescriptorsRight, mb: float, mbf: float):
    """Frame::ComputeStereoMatches (Frame.cc:811-981) on the GPU pyramids of the
    last images given to the two extractors: returns (mvuRight, mvDepth)."""
    kl = np.ascontiguousarray(mvKeys, abi.KEYPOINT_DTYPE)
    kr = np.ascontiguousarray(mvKeysRight, abi.KEYPOINT_DTYPE)
    dl = np.ascontiguousarray(mDescriptors, np.uint8).reshape(-1, 32)
    dr = np.ascontiguousarray(mDescriptorsRight, np.uint8).reshape(-1, 32)
    ur = np.full(len(kl), -1.0, np.float32)
    dep = np.full(len(kl), -1.0, np.float32)
    capi.check(capi.lib().orbs_compute_stereo_matches(ex_left._h, ex_right._h, abi.ptr(kl), len(kl), abi.ptr(dl),
                                                      abi.ptr(kr), len(kr), abi.ptr(dr), mb, mbf, abi.ptr(ur),
                                                      abi.ptr(dep)), "orbs_compute_stereo_matches")
    return ur, dep


def compute_stereo_matches_batch_device(ex: ORBextractor, npairs: int, left0: int, right0: int, kps, desc, n,
                                        cap: int, mb: float, mbf: float, stream=None):
    """Batched stereo matching on the outputs of ``ex.extract_batch_device``
    (pairs = frames left0+i / right0+i of that batch).  Returns CUDA tensors
    (uright, depth, sad), each (npairs, cap)."""
    import torch
    dev = kps.device
    ur = torch.empty((npairs, cap), dtype=torch.float32, device=dev)
    dep = torch.empty((npairs, cap), dtype=torch.float32, device=dev)
    sad = torch.empty((npairs, cap), dtype=torch.int32, device=dev)
    st = stream.cuda_stream if stream is not None else torch.cuda.current_stream().cuda_stream
    rc = capi.lib().orbs_compute_stereo_matches_batch_device(ex._h, npairs, left0, right0, kps.data_ptr(),
                                                             desc.data_ptr(), n.data_ptr(), cap, mb, mbf,
                                                             ur.data_ptr(), dep.data_ptr(), sad.data_ptr(),
                                                             C.c_void_p(st))
    capi.check(rc, "orbs_compute_stereo_matches_batch_device")
    return ur, dep, sad


def knn_match2(query: np.ndarray, train: np.ndarray, device: int = 0):
    """BFMatcher(NORM_HAMMING).knnMatch(query, train, 2) on the GPU: (idx, dist), each (nq, 2)."""
    q = np.ascontiguousarray(query, np.uint8).reshape(-1, 32)
    t = np.ascontiguousarray(train, np.uint8).reshape(-1, 32)
    idx = np.zeros((len(q), 2), np.int32)
    dist = np.zeros((len(q), 2), np.int32)
    capi.check(capi.lib().orbs_knn_match2(abi.ptr(q), len(q), abi.ptr(t), len(t), abi.ptr(idx), abi.ptr(dist),
                                          device), "orbs_knn_match2")
    return idx, dist


def fisheye_stereo_candidates_batch_device(npairs: int, left0: int, right0: int, desc, n, mono, cap: int,
                                           ratio: float = 0.7, stream=None):
    """ComputeStereoFishEyeMatches' knnMatch + ratio on device batch outputs:
    (idx (P, cap, 2), dist (P, cap, 2), l2r (P, cap)) CUDA tensors."""
    import torch
    dev = desc.device
    idx = torch.empty((npairs, cap, 2), dtype=torch.int32, device=dev)
    dist = torch.empty((npairs, cap, 2), dtype=torch.int32, device=dev)
    l2r = torch.empty((npairs, cap), dtype=torch.int32, device=dev)
    st = stream.cuda_stream if stream is not None else torch.cuda.current_stream().cuda_stream
    capi.check(capi.lib().orbs_fisheye_stereo_candidates_batch_device(
        npairs, left0, right0, desc.data_ptr(), n.data_ptr(), mono.data_ptr(), cap, ratio, idx.data_ptr(),
        dist.data_ptr(), l2r.data_ptr(), C.c_void_p(st)), "orbs_fisheye_stereo_candidates_batch_device")
    return idx, dist, l2r


class TextVocabulary:
    """TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1338-1424)
    through the library's loader.  ``.struct`` is the orbv_vocab view (valid
    while this object lives); ``.arrays()`` copies it into the dict layout of
    ``synth.vocabulary`` (with ``child_idx``)."""

    def __init__(self, path):
        err = C.c_int32(0)
        self._h = capi.lib().orbv_load_text(str(path).encode(), C.byref(err))
        if not self._h:
            raise ValueError(f"vocabulary loading failure ({err.value}): {path}")
        self.struct = abi.OrbvVocab()
        k, sc, wt, nw = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int32()
        capi.check(capi.lib().orbv_text_vocab_view(self._h, C.byref(self.struct), C.byref(k), C.byref(sc),
                                                   C.byref(wt), C.byref(nw)), "orbv_text_vocab_view")
        self.k, self.L, self.scoring, self.weighting, self.nwords = k.value, self.struct.depth_levels, sc.value, \
            wt.value, nw.value
        self.nnodes = self.struct.nnodes

    def ref(self):
        return C.byref(self.struct)

    def arrays(self) -> dict:
        n = self.nnodes

        def arr(p, ctype, count, dtype):
            if not p or count == 0:
                return np.zeros(count, dtype)
            return np.ctypeslib.as_array(C.cast(p, C.POINTER(ctype)), (count,)).astype(dtype).copy()
        nchild = arr(self.struct.nchild, C.c_int32, n, np.int32)
        first = arr(self.struct.first_child, C.c_int32, n, np.int32)
        total = int((first + nchild).max()) if n else 0
        return dict(nnodes=n, depth_levels=self.L, first_child=first, nchild=nchild,
                    node_desc=arr(self.struct.node_desc, C.c_uint8, n * 32, np.uint8).reshape(n, 32),
                    word_id=arr(self.struct.word_id, C.c_int32, n, np.int32),
                    weight=arr(self.struct.weight, C.c_double, n, np.float64),
                    child_idx=arr(self.struct.child_idx, C.c_int32, total, np.int32))

    def __del__(self):
        if getattr(self, "_h", None):
            capi.lib().orbv_free_text(self._h)
            self._h = None


def transform_bow(voc, desc: np.ndarray, scoring: int = 0, weighting: int = 0, levelsup: int = 4,
                  device: int = 0):
    """transform(features, BowVector, FeatureVector, levelsup): the descent on
    the GPU, then the library's BowVector/FeatureVector assembly.  Returns
    (bow_words, bow_values, fv_nodes, fv_off, fv_idx)."""
    wid, w, nid = transform(voc, desc, levelsup, device)
    n = len(wid)
    bw, bv = np.zeros(n, np.int32), np.zeros(n, np.float64)
    fn, fo, fi = np.zeros(n, np.int32), np.zeros(n + 1, np.int32), np.zeros(n, np.int32)
    nb, nf = C.c_int32(), C.c_int32()
    capi.check(capi.lib().orbv_bow_assemble(scoring, weighting, n, abi.ptr(wid), abi.ptr(w), abi.ptr(nid),
                                            abi.ptr(bw), abi.ptr(bv), C.byref(nb), abi.ptr(fn), abi.ptr(fo),
                                            abi.ptr(fi), C.byref(nf)), "orbv_bow_assemble")
    return bw[:nb.value], bv[:nb.value], fn[:nf.value], fo[:nf.value + 1], fi[:fo[nf.value]]


def score(scoring: int, w1, v1, w2, v2) -> float:
    """GeneralScoring::score of two BowVectors (ScoringObject.cpp)."""
    w1, v1 = np.ascontiguousarray(w1, np.int32), np.ascontiguousarray(v1, np.float64)
    w2, v2 = np.ascontiguousarray(w2, np.int32), np.ascontiguousarray(v2, np.float64)
    return capi.lib().orbv_score(scoring, abi.ptr(w1), abi.ptr(v1), len(w1), abi.ptr(w2), abi.ptr(v2), len(w2))


class KeyFrameDatabase:
    """Device snapshot of KeyFrameDatabase for DetectRelocalizationCandidates
    (KeyFrameDatabase.cc:733-845).  ``db`` is a dict of CSR arrays: bow_off,
    bow_words, bow_vals, inv_off, inv_kf, cov_off, cov_kf, kf_map, nkf, nwords."""

    def __init__(self, db: dict, device: int = 0):
        self._h = capi.lib().orbk_db_create(device)
        if not self._h:
            raise RuntimeError("orbk_db_create failed (no HIP device)")
        self.nkf = int(db["nkf"])
        self._keep = [np.ascontiguousarray(db[k], dt) for k, dt in
                      (("bow_off", np.int32), ("bow_words", np.int32), ("bow_vals", np.float64), ("inv_off", np.int32),
                       ("inv_kf", np.int32), ("cov_off", np.int32), ("cov_kf", np.int32), ("kf_map", np.int32))]
        bo, bw, bv, io, ik, co, ck, km = self._keep
        capi.check(capi.lib().orbk_db_upload(self._h, self.nkf, abi.ptr(bo), abi.ptr(bw), abi.ptr(bv),
                                             int(db["nwords"]), abi.ptr(io), abi.ptr(ik), abi.ptr(co), abi.ptr(ck),
                                             abi.ptr(km)), "orbk_db_upload")

    def DetectRelocalizationCandidates(self, q_words, q_vals, map_id: int, reloc_score: np.ndarray):
        qw = np.ascontiguousarray(q_words, np.int32)
        qv = np.ascontiguousarray(q_vals, np.float64)
        assert reloc_score.dtype == np.float32 and reloc_score.flags["C_CONTIGUOUS"] and len(reloc_score) >= self.nkf
        cand = np.zeros(max(1, self.nkf), np.int32)
        n = capi.lib().orbk_detect_relocalization_candidates(self._h, abi.ptr(qw), abi.ptr(qv), len(qw), map_id,
                                                              abi.ptr(reloc_score), abi.ptr(cand), self.nkf)
        capi.check(min(n, 0), "orbk_detect_relocalization_candidates")
        return cand[:n].copy()

    def __del__(self):
        if getattr(self, "_h", None):
            capi.lib().orbk_db_destroy(self._h)
            self._h = None


def keypoints_from_device(kps_i32) -> np.ndarray:
    """(cap, 7) int32 tensor/array -> structured KEYPOINT_DTYPE array."""
    a = np.ascontiguousarray(kps_i32.cpu().numpy() if hasattr(kps_i32, "cpu") else kps_i32, dtype=np.int32)
    return a.view(abi.KEYPOINT_DTYPE).reshape(a.shape[:-1])


class DeviceFrame:
    """A Frame or KeyFrame resident in HBM (orbm_dframe, include/orb_mi355x.h):
    the Tracking thread's searches then move only their per-call inputs and
    results across PCIe (Tracking.cc:2720-2730, 2886, 3413)."""

    def __init__(self, device: int = 0):
        self._L = capi.lib()
        self._h = self._L.orbm_dframe_create(device)
        if not self._h:
            raise RuntimeError("orbm_dframe_create failed (no device?)")
        self._keep = None

    def upload(self, F: abi.Keep, fv: abi.Keep | None = None) -> "DeviceFrame":
        capi.check(self._L.orbm_dframe_upload(self._h, F.ref(), fv.ref() if fv is not None else None),
                   "orbm_dframe_upload")
        return self

    def from_extractor(self, ex: "ORBextractor", geom: abi.Keep, fv: abi.Keep | None = None) -> "DeviceFrame":
        """The last image `ex` extracted (ORBextractor.__call__), copied device to device."""
        capi.check(self._L.orbm_dframe_from_extractor(self._h, ex._h, geom.ref(), fv.ref() if fv is not None else None),
                   "orbm_dframe_from_extractor")
        return self

    def set_featvec(self, fv: abi.Keep) -> "DeviceFrame":
        capi.check(self._L.orbm_dframe_set_featvec(self._h, fv.ref()), "orbm_dframe_set_featvec")
        return self

    @property
    def n(self) -> int:
        return capi.check(self._L.orbm_dframe_count(self._h), "orbm_dframe_count")

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.orbm_dframe_destroy(self._h)
            self._h = None


class ORBmatcher:
    TH_HIGH, TH_LOW, HISTO_LENGTH = 100, 50, 30

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True):
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)

    @staticmethod
    def DescriptorDistance(a: np.ndarray, b: np.ndarray) -> int:
        a = np.ascontiguousarray(a, np.uint8)
        b = np.ascontiguousarray(b, np.uint8)
        return capi.lib().orbm_descriptor_distance(abi.ptr(a), abi.ptr(b))

    def SearchForInitialization(self, F1: abi.Keep, F2: abi.Keep, vbPrevMatched: np.ndarray, windowSize: int = 10):
        prev = np.ascontiguousarray(vbPrevMatched, np.float32).copy()
        m12 = np.zeros(F1.struct.n, np.int32)
        nm = capi.lib().orbm_search_for_initialization(F1.ref(), F2.ref(), abi.ptr(prev), windowSize,
                                                       self.mfNNratio, int(self.mbCheckOrientation), abi.ptr(m12))
        capi.check(nm, "SearchForInitialization")
        return nm, m12, prev

    def SearchByBoW(self, KF: abi.Keep, KFfv: abi.Keep, kf_valid: np.ndarray, F: abi.Keep, Ffv: abi.Keep):
        kf_valid = np.ascontiguousarray(kf_valid, np.uint8)
        match = np.zeros(F.struct.n, np.int32)
        nm = capi.lib().orbm_search_by_bow(KF.ref(), KFfv.ref(), abi.ptr(kf_valid), F.ref(), Ffv.ref(),
                                           self.mfNNratio, int(self.mbCheckOrientation), abi.ptr(match))
        capi.check(nm, "SearchByBoW")
        return nm, match

    # ---- the same searches on HBM-resident frames (orbm_*_dframe) ----
    def SearchForInitializationDevice(self, F1: DeviceFrame, F2: DeviceFrame, vbPrevMatched: np.ndarray,
                                      windowSize: int = 10):
        prev = np.ascontiguousarray(vbPrevMatched, np.float32).copy()
        m12 = np.zeros(F1.n, np.int32)
        nm = capi.lib().orbm_search_for_initialization_dframe(F1._h, F2._h, abi.ptr(prev), windowSize,
                                                              self.mfNNratio, int(self.mbCheckOrientation),
                                                              abi.ptr(m12))
        capi.check(nm, "SearchForInitialization(dframe)")
        return nm, m12, prev

    def SearchByBoWDevice(self, KF: DeviceFrame, kf_valid: np.ndarray, F: DeviceFrame):
        kf_valid = np.ascontiguousarray(kf_valid, np.uint8)
        match = np.zeros(F.n, np.int32)
        nm = capi.lib().orbm_search_by_bow_dframe(KF._h, abi.ptr(kf_valid), F._h, self.mfNNratio,
                                                  int(self.mbCheckOrientation), abi.ptr(match))
        capi.check(nm, "SearchByBoW(dframe)")
        return nm, match

    def SearchByProjectionDevice(self, F: DeviceFrame, mps: abi.Keep, th: float = 3.0, bFarPoints: bool = False,
                                 thFarPoints: float = 50.0, owner=None, blocked=None):
        n = F.n
        owner = np.full(n, -1, np.int32) if owner is None else np.ascontiguousarray(owner, np.int32).copy()
        blocked = np.zeros(n, np.uint8) if blocked is None else np.ascontiguousarray(blocked, np.uint8)
        nm = capi.lib().orbm_search_by_projection_mps_dframe(F._h, mps.ref(), th, int(bFarPoints), thFarPoints,
                                                             self.mfNNratio, abi.ptr(owner), abi.ptr(blocked))
        capi.check(nm, "SearchByProjection(dframe, MPs)")
        return nm, owner

    def SearchByProjectionLastDevice(self, cur: DeviceFrame, valid, u, v, ur, octave, angle, has_obs, desc,
                                     th: float, mode: int = 0, owner=None, blocked=None):
        n = cur.n
        arrs = [np.ascontiguousarray(valid, np.uint8), np.ascontiguousarray(u, np.float32),
                np.ascontiguousarray(v, np.float32), np.ascontiguousarray(ur, np.float32),
                np.ascontiguousarray(octave, np.int32), np.ascontiguousarray(angle, np.float32),
                np.ascontiguousarray(has_obs, np.uint8), np.ascontiguousarray(desc, np.uint8)]
        owner = np.full(n, -1, np.int32) if owner is None else np.ascontiguousarray(owner, np.int32).copy()
        blocked = np.zeros(n, np.uint8) if blocked is None else np.ascontiguousarray(blocked, np.uint8)
        nm = capi.lib().orbm_search_by_projection_last_dframe(cur._h, len(arrs[0]), *[abi.ptr(a) for a in arrs], th,
                                                              mode, int(self.mbCheckOrientation), abi.ptr(owner),
                                                              abi.ptr(blocked))
        capi.check(nm, "SearchByProjection(dframe, LastFrame)")
        return nm, owner

    def SearchByBoWMany(self, KFs, KFfvs, kf_valids, F: abi.Keep, Ffv: abi.Keep):
        """SearchByBoW(KF_i, F) for several candidate keyframes in one launch
        (orbm_search_by_bow_many; the loop of Tracking.cc:3641-3648):
        (counts[nkf], match[nkf, F.n])."""
        nkf = len(KFs)
        valids = [np.ascontiguousarray(v, np.uint8) for v in kf_valids]
        ks = (C.c_void_p * max(1, nkf))(*[C.addressof(k.struct) for k in KFs])
        fs = (C.c_void_p * max(1, nkf))(*[C.addressof(k.struct) for k in KFfvs])
        vs = (C.c_void_p * max(1, nkf))(*[v.ctypes.data for v in valids])
        match = np.zeros((nkf, F.struct.n), np.int32)
        counts = np.zeros(nkf, np.int32)
        rc = capi.lib().orbm_search_by_bow_many(nkf, ks, fs, vs, F.ref(), Ffv.ref(), self.mfNNratio,
                                                int(self.mbCheckOrientation), abi.ptr(match), abi.ptr(counts))
        capi.check(rc, "SearchByBoWMany")
        return counts, match

    def SearchByProjection(self, F: abi.Keep, mps: abi.Keep, th: float = 3.0, bFarPoints: bool = False,
                           thFarPoints: float = 50.0, owner=None, blocked=None):
        n = F.struct.n
        owner = np.full(n, -1, np.int32) if owner is None else np.ascontiguousarray(owner, np.int32).copy()
        blocked = np.zeros(n, np.uint8) if blocked is None else np.ascontiguousarray(blocked, np.uint8)
        nm = capi.lib().orbm_search_by_projection_mps(F.ref(), mps.ref(), th, int(bFarPoints), thFarPoints,
                                                      self.mfNNratio, abi.ptr(owner), abi.ptr(blocked))
        capi.check(nm, "SearchByProjection(F, MPs)")
        return nm, owner

    def SearchByProjectionLast(self, cur: abi.Keep, valid, u, v, ur, octave, angle, has_obs, desc, th: float,
                               mode: int = 0, owner=None, blocked=None):
        n = cur.struct.n
        arrs = [np.ascontiguousarray(valid, np.uint8), np.ascontiguousarray(u, np.float32),
                np.ascontiguousarray(v, np.float32), np.ascontiguousarray(ur, np.float32),
                np.ascontiguousarray(octave, np.int32), np.ascontiguousarray(angle, np.float32),
                np.ascontiguousarray(has_obs, np.uint8), np.ascontiguousarray(desc, np.uint8)]
        owner = np.full(n, -1, np.int32) if owner is None else np.ascontiguousarray(owner, np.int32).copy()
        blocked = np.zeros(n, np.uint8) if blocked is None else np.ascontiguousarray(blocked, np.uint8)
        nm = capi.lib().orbm_search_by_projection_last(cur.ref(), len(arrs[0]), *[abi.ptr(a) for a in arrs], th,
                                                       mode, int(self.mbCheckOrientation), abi.ptr(owner),
                                                       abi.ptr(blocked))
        capi.check(nm, "SearchByProjection(F, LastFrame)")
        return nm, owner

    @staticmethod
    def Fuse(KF: abi.Keep, inv_level_sigma2, valid, u, v, ur, level, desc, th: float = 3.0, fma: int = 1):
        """Fuse(pKF, vpMapPoints, th) matching (ORBmatcher.cc:1148-1331): (nfused, best_idx, best_dist)."""
        n = len(valid)
        arrs = [np.ascontiguousarray(inv_level_sigma2, np.float32), np.ascontiguousarray(valid, np.uint8),
                np.ascontiguousarray(u, np.float32), np.ascontiguousarray(v, np.float32),
                np.ascontiguousarray(ur, np.float32), np.ascontiguousarray(level, np.int32),
                np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)]
        bi, bd = np.zeros(n, np.int32), np.zeros(n, np.int32)
        nf = capi.lib().orbm_fuse(KF.ref(), *[abi.ptr(a) for a in arrs[:1]], n, *[abi.ptr(a) for a in arrs[1:]],
                                  th, fma, abi.ptr(bi), abi.ptr(bd))
        capi.check(min(nf, 0), "Fuse")
        return nf, bi, bd

    def SearchForTriangulation(self, KF1: abi.Keep, fv1: abi.Keep, has_mp1, KF2: abi.Keep, fv2: abi.Keep, has_mp2,
                               F12, ep, level_sigma2_2, bOnlyStereo: bool = False, bCoarse: bool = False,
                               fma: int = 1):
        """SearchForTriangulation (ORBmatcher.cc:907-1146): (nmatches, matches12)."""
        m1 = np.ascontiguousarray(has_mp1, np.uint8)
        m2 = np.ascontiguousarray(has_mp2, np.uint8)
        F = np.ascontiguousarray(F12, np.float32).reshape(9)
        s2 = np.ascontiguousarray(level_sigma2_2, np.float32)
        out = np.full(len(m1), -1, np.int32)
        nm = capi.lib().orbm_search_for_triangulation(KF1.ref(), fv1.ref(), abi.ptr(m1), KF2.ref(), fv2.ref(),
                                                      abi.ptr(m2), abi.ptr(F), float(ep[0]), float(ep[1]),
                                                      abi.ptr(s2), int(bOnlyStereo), int(bCoarse),
                                                      int(self.mbCheckOrientation), fma, abi.ptr(out))
        capi.check(min(nm, 0), "SearchForTriangulation")
        return nm, out

    def SearchForTriangulationChecked(self, KF1: abi.Keep, fv1: abi.Keep, has_mp1, KF2: abi.Keep, fv2: abi.Keep,
                                      has_mp2, check, bOnlyStereo: bool = False):
        """SearchForTriangulation (ORBmatcher.cc:907-1146) with the per-candidate
        geometry supplied by the caller, check(idx1, idx2) -> bool (the epipole
        test + epipolarConstrain of a KannalaBrandt8 or two-camera keyframe
        pair, :1014-1076): the GPU ranks the candidates, the first one the check
        accepts is the match.  (nmatches, matches12)."""
        m1 = np.ascontiguousarray(has_mp1, np.uint8)
        m2 = np.ascontiguousarray(has_mp2, np.uint8)
        out = np.full(len(m1), -1, np.int32)
        cb = abi.TRI_CHECK(lambda _ctx, i1, i2: int(bool(check(i1, i2))))
        nm = capi.lib().orbm_search_for_triangulation_checked(KF1.ref(), fv1.ref(), abi.ptr(m1), KF2.ref(),
                                                              fv2.ref(), abi.ptr(m2), int(bOnlyStereo),
                                                              int(self.mbCheckOrientation), cb, None, abi.ptr(out))
        capi.check(min(nm, 0), "SearchForTriangulationChecked")
        return nm, out

    # ---- relocalisation / loop closing (ORBmatcher.h:55-63,71-84) ----

    def SearchByBoWKF(self, KF1: abi.Keep, fv1: abi.Keep, valid1, KF2: abi.Keep, fv2: abi.Keep, valid2):
        """SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vpMatches12) (ORBmatcher.cc:765-905):
        (nmatches, matches12) with matches12[i1] = KF2 feature or -1."""
        v1 = np.ascontiguousarray(valid1, np.uint8)
        v2 = np.ascontiguousarray(valid2, np.uint8)
        m12 = np.full(KF1.struct.n, -1, np.int32)
        nm = capi.lib().orbm_search_by_bow_kf(KF1.ref(), fv1.ref(), abi.ptr(v1), KF2.ref(), fv2.ref(), abi.ptr(v2),
                                              self.mfNNratio, int(self.mbCheckOrientation), abi.ptr(m12))
        capi.check(nm, "SearchByBoW(KF1, KF2)")
        return nm, m12

    def SearchByProjectionKF(self, F: abi.Keep, valid, u, v, level, kf_angle, desc, th: float, ORBdist: int,
                             owner=None):
        """SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist) (ORBmatcher.cc:1889-2010):
        (nmatches, owner) -- owner[i2] = keyframe point index for the new matches."""
        q = _queries(valid, u, v, level, desc)
        ang = np.ascontiguousarray(kf_angle, np.float32)
        own = np.full(F.struct.n, -1, np.int32) if owner is None else np.ascontiguousarray(owner, np.int32).copy()
        nm = capi.lib().orbm_search_by_projection_kf(F.ref(), len(q[0]), abi.ptr(q[0]), abi.ptr(q[1]),
                                                     abi.ptr(q[2]), abi.ptr(q[3]), abi.ptr(ang), abi.ptr(q[4]),
                                                     float(th), int(ORBdist), int(self.mbCheckOrientation),
                                                     abi.ptr(own))
        capi.check(nm, "SearchByProjection(F, KF)")
        return nm, own

    @staticmethod
    def SearchByProjectionSim3(KF: abi.Keep, valid, u, v, level, desc, th: float, ratioHamming: float = 1.0,
                               matched=None):
        """SearchByProjection(KeyFrame*, Sim3, vpPoints, vpMatched, th, ratioHamming)
        (ORBmatcher.cc:427-646): (nmatches, matched) -- matched[idx] = point index for the new matches."""
        q = _queries(valid, u, v, level, desc)
        m = np.full(KF.struct.n, -1, np.int32) if matched is None else np.ascontiguousarray(matched, np.int32).copy()
        nm = capi.lib().orbm_search_by_projection_sim3(KF.ref(), len(q[0]), *[abi.ptr(a) for a in q], float(th),
                                                       float(ratioHamming), abi.ptr(m))
        capi.check(nm, "SearchByProjection(KF, Sim3)")
        return nm, m

    @staticmethod
    def SearchBySim3(KF1: abi.Keep, KF2: abi.Keep, q1, q2, th: float):
        """SearchBySim3(pKF1, pKF2, vpMatches12, S12, th) (ORBmatcher.cc:1457-1674); q1 / q2 =
        (valid, u, v, level, desc) of KF1's points projected into KF2 and KF2's into KF1:
        (nFound, matches12) with the new mutual matches."""
        a1, a2 = _queries(*q1), _queries(*q2)
        m12 = np.full(KF1.struct.n, -1, np.int32)
        nf = capi.lib().orbm_search_by_sim3(KF1.ref(), KF2.ref(), *[abi.ptr(a) for a in a1],
                                            *[abi.ptr(a) for a in a2], float(th), abi.ptr(m12))
        capi.check(nf, "SearchBySim3")
        return nf, m12

    @staticmethod
    def FuseSim3(KF: abi.Keep, valid, u, v, level, desc, th: float):
        """Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) matching (ORBmatcher.cc:1340-1455):
        (nfused, best_idx, best_dist)."""
        q = _queries(valid, u, v, level, desc)
        n = len(q[0])
        bi, bd = np.zeros(n, np.int32), np.zeros(n, np.int32)
        nf = capi.lib().orbm_fuse_sim3(KF.ref(), n, *[abi.ptr(a) for a in q], float(th), abi.ptr(bi), abi.ptr(bd))
        capi.check(nf, "Fuse(KF, Sim3)")
        return nf, bi, bd

    # ---- fisheye stereo frames (Frame::Nleft != -1; F = [mvKeys; mvKeysRight]) ----

    def SearchByBoWFisheye(self, KF: abi.Keep, KFfv: abi.Keep, kf_valid, F: abi.Keep, Ffv: abi.Keep, Nleft: int):
        """SearchByBoW(KeyFrame*, Frame&) with F.Nleft != -1 (ORBmatcher.cc:296-386): (nmatches, match)."""
        kf_valid = np.ascontiguousarray(kf_valid, np.uint8)
        match = np.zeros(F.struct.n, np.int32)
        nm = capi.lib().orbm_search_by_bow_fisheye(KF.ref(), KFfv.ref(), abi.ptr(kf_valid), F.ref(), Ffv.ref(),
                                                   int(Nleft), self.mfNNratio, int(self.mbCheckOrientation),
                                                   abi.ptr(match))
        capi.check(nm, "SearchByBoW(KF, F fisheye)")
        return nm, match

    def SearchByProjectionFisheye(self, F: abi.Keep, Nleft: int, l2r, r2l, mps: abi.Keep, mps_r: abi.Keep,
                                  th: float = 3.0, bFarPoints: bool = False, thFarPoints: float = 50.0, owner=None,
                                  blocked=None):
        """SearchByProjection(Frame&, vector<MapPoint*>) with F.Nleft != -1 (ORBmatcher.cc:43-213)."""
        n = F.struct.n
        l2r = np.ascontiguousarray(l2r, np.int32)
        r2l = np.ascontiguousarray(r2l, np.int32)
        owner = np.full(n, -1, np.int32) if owner is None else np.ascontiguousarray(owner, np.int32).copy()
        blocked = np.zeros(n, np.uint8) if blocked is None else np.ascontiguousarray(blocked, np.uint8)
        nm = capi.lib().orbm_search_by_projection_mps_fisheye(F.ref(), int(Nleft), abi.ptr(l2r), abi.ptr(r2l),
                                                              mps.ref(), mps_r.ref(), th, int(bFarPoints),
                                                              thFarPoints, self.mfNNratio, abi.ptr(owner),
                                                              abi.ptr(blocked))
        capi.check(nm, "SearchByProjection(F fisheye, MPs)")
        return nm, owner

    def SearchByProjectionLastFisheye(self, cur: abi.Keep, Nleft: int, valid, u, v, ur, vr, octave, angle, has_obs,
                                      desc, th: float, mode: int = 0, owner=None, blocked=None):
        """SearchByProjection(Frame& Current, const Frame& Last) with Current.Nleft != -1
        (ORBmatcher.cc:1676-1887); ur / vr = projections into the right camera."""
        n = cur.struct.n
        arrs = [np.ascontiguousarray(valid, np.uint8), np.ascontiguousarray(u, np.float32),
                np.ascontiguousarray(v, np.float32), np.ascontiguousarray(ur, np.float32),
                np.ascontiguousarray(vr, np.float32), np.ascontiguousarray(octave, np.int32),
                np.ascontiguousarray(angle, np.float32), np.ascontiguousarray(has_obs, np.uint8),
                np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)]
        owner = np.full(n, -1, np.int32) if owner is None else np.ascontiguousarray(owner, np.int32).copy()
        blocked = np.zeros(n, np.uint8) if blocked is None else np.ascontiguousarray(blocked, np.uint8)
        nm = capi.lib().orbm_search_by_projection_last_fisheye(cur.ref(), int(Nleft), len(arrs[0]),
                                                               *[abi.ptr(x) for x in arrs], th, mode,
                                                               int(self.mbCheckOrientation), abi.ptr(owner),
                                                               abi.ptr(blocked))
        capi.check(nm, "SearchByProjection(F fisheye, LastFrame)")
        return nm, owner


def _queries(valid, u, v, level, desc):
    return (np.ascontiguousarray(valid, np.uint8), np.ascontiguousarray(u, np.float32),
            np.ascontiguousarray(v, np.float32), np.ascontiguousarray(level, np.int32),
            np.ascontiguousarray(desc, np.uint8).reshape(-1, 32))


def compute_distinctive_descriptors(off, desc, device: int = 0) -> np.ndarray:
    """MapPoint::ComputeDistinctiveDescriptors for every point of a CSR batch:
    per point the index of its most distinctive descriptor (-1 if none)."""
    off = np.ascontiguousarray(off, np.int32)
    desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    best = np.zeros(max(len(off) - 1, 0), np.int32)
    capi.check(capi.lib().orbm_compute_distinctive_descriptors(len(best), abi.ptr(off), abi.ptr(desc), abi.ptr(best),
                                                               device), "orbm_compute_distinctive_descriptors")
    return best


def transform_device(voc_dev, desc, levelsup: int = 4, stream=None):
    """transform on a vocabulary resident in HBM (voc_dev: abi.Keep of an
    orbv_vocab holding device pointers, e.g. sharding.vocab_device_struct) for
    a CUDA uint8 tensor of descriptors: (word_id, weight, node_id) tensors."""
    import torch
    assert desc.is_cuda and desc.dtype == torch.uint8 and desc.is_contiguous()
    n = desc.shape[0]
    wid = torch.empty(n, dtype=torch.int32, device=desc.device)
    w = torch.empty(n, dtype=torch.float64, device=desc.device)
    nid = torch.empty(n, dtype=torch.int32, device=desc.device)
    st = (stream or torch.cuda.current_stream(desc.device)).cuda_stream
    capi.check(capi.lib().orbv_transform_device(voc_dev.ref(), n, desc.data_ptr(), levelsup, wid.data_ptr(),
                                                w.data_ptr(), nid.data_ptr(), st), "orbv_transform_device")
    return wid, w, nid


def transform(voc, desc: np.ndarray, levelsup: int = 4, device: int = 0):
    """TemplatedVocabulary::transform per descriptor on the GPU: (word_id, weight, node_id)."""
    desc = np.ascontiguousarray(desc, np.uint8)
    n = len(desc)
    wid = np.zeros(n, np.int32)
    w = np.zeros(n, np.float64)
    nid = np.zeros(n, np.int32)
    capi.check(capi.lib().orbv_transform(voc.ref(), n, abi.ptr(desc), levelsup, abi.ptr(wid), abi.ptr(w),
                                         abi.ptr(nid), device), "orbv_transform")
    return wid, w, nid
