"""ctypes mirror of include/orb_mi355x.h (types only).

Shared by the product bindings (``capi.py``) and by the test-side oracle
wrapper, so both sides marshal identical structs.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

# cv::KeyPoint, 28 bytes (orb_keypoint)
KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KEYPOINT_DTYPE.itemsize == 28

ORB_OK = 0
ORB_ERR_EMPTY = -1
ORB_ERR_CAPACITY = -2
ORB_ERR_PARAM = -3
ORB_ERR_DEVICE = -4
ORB_ERR_UNSUPPORTED = -5


class OrbxParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32), ("blur_variant", C.c_int32),
                ("fma_sampling", C.c_int32), ("reserved", C.c_int32)]


def params(nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th_fast=20, min_th_fast=7,
           blur_variant=0, fma_sampling=1) -> OrbxParams:
    return OrbxParams(nfeatures, scale_factor, nlevels, ini_th_fast, min_th_fast,
                      blur_variant, fma_sampling, 0)


class OrbmFrame(C.Structure):
    _fields_ = [("n", C.c_int32), ("kps", C.c_void_p), ("desc", C.c_void_p),
                ("min_x", C.c_float), ("max_x", C.c_float), ("min_y", C.c_float), ("max_y", C.c_float),
                ("grid_inv_w", C.c_float), ("grid_inv_h", C.c_float), ("u_right", C.c_void_p),
                ("scale_factors", C.c_void_p), ("nlevels", C.c_int32)]


class OrbmFeatVec(C.Structure):
    _fields_ = [("nnodes", C.c_int32), ("node_ids", C.c_void_p), ("offsets", C.c_void_p),
                ("idx", C.c_void_p)]


class OrbmMapPoints(C.Structure):
    _fields_ = [("n", C.c_int32), ("proj_x", C.c_void_p), ("proj_y", C.c_void_p),
                ("proj_xr", C.c_void_p), ("level", C.c_void_p), ("view_cos", C.c_void_p),
                ("track_depth", C.c_void_p), ("in_view", C.c_void_p), ("has_obs", C.c_void_p),
                ("desc", C.c_void_p)]


class OrbvVocab(C.Structure):
    _fields_ = [("nnodes", C.c_int32), ("depth_levels", C.c_int32), ("first_child", C.c_void_p),
                ("nchild", C.c_void_p), ("node_desc", C.c_void_p), ("word_id", C.c_void_p),
                ("weight", C.c_void_p), ("child_idx", C.c_void_p)]


class OrbmMapPointsRight(C.Structure):
    _fields_ = [("in_view", C.c_void_p), ("proj_x", C.c_void_p), ("proj_y", C.c_void_p), ("level", C.c_void_p),
                ("view_cos", C.c_void_p)]


# orbm_tri_check_fn: int (*)(void* ctx, int idx1, int idx2)
TRI_CHECK = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_int)


def ptr(a: np.ndarray | None) -> int | None:
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "arrays crossing the C ABI must be contiguous"
    return a.ctypes.data


class Keep:
    """Holds numpy arrays alive while a ctypes struct points at them."""

    def __init__(self, struct, arrays):
        self.struct = struct
        self.arrays = arrays

    def ref(self):
        return C.byref(self.struct)


def frame_struct(kps: np.ndarray, desc: np.ndarray, width: int, height: int,
                 scale_factors: np.ndarray | None = None, u_right: np.ndarray | None = None,
                 bounds=None) -> Keep:
    """orbm_frame for an undistorted pinhole frame of width x height
    (Frame::ComputeImageBounds with zero distortion: 0..cols, 0..rows;
    mfGridElementWidthInv = 64/(maxX-minX), Frame.cc:249-252)."""
    kps = np.ascontiguousarray(kps, dtype=KEYPOINT_DTYPE)
    desc = np.ascontiguousarray(desc, dtype=np.uint8).reshape(-1, 32)
    if bounds is None:
        min_x, max_x, min_y, max_y = 0.0, float(width), 0.0, float(height)
    else:
        min_x, max_x, min_y, max_y = bounds
    inv_w = np.float32(64) / np.float32(np.float32(max_x) - np.float32(min_x))
    inv_h = np.float32(48) / np.float32(np.float32(max_y) - np.float32(min_y))
    sf = None if scale_factors is None else np.ascontiguousarray(scale_factors, np.float32)
    ur = None if u_right is None else np.ascontiguousarray(u_right, np.float32)
    s = OrbmFrame(len(kps), ptr(kps), ptr(desc), min_x, max_x, min_y, max_y, float(inv_w), float(inv_h),
                  ptr(ur), ptr(sf), 0 if sf is None else len(sf))
    return Keep(s, [kps, desc, sf, ur])


def featvec_struct(node_of_feature: np.ndarray) -> Keep:
    """FeatureVector CSR from a per-feature node id array (-1 = stopped word,
    not added; FeatureVector::addFeature keeps ascending node ids and feature
    indices in insertion order, FeatureVector.cpp:31-45)."""
    nid = np.asarray(node_of_feature, dtype=np.int64)
    feats = np.nonzero(nid >= 0)[0]
    order = np.lexsort((feats, nid[feats]))
    feats = feats[order]
    nodes, starts = np.unique(nid[feats], return_index=True)
    offsets = np.append(starts, len(feats)).astype(np.int32)
    node_ids = nodes.astype(np.uint32)
    idx = feats.astype(np.uint32)
    s = OrbmFeatVec(len(node_ids), ptr(node_ids), ptr(offsets), ptr(idx))
    return Keep(s, [node_ids, offsets, idx])


def vocab_struct(v: dict) -> Keep:
    keys = ("first_child", "nchild", "node_desc", "word_id", "weight")
    arrs = {k: np.ascontiguousarray(v[k]) for k in keys}
    if v.get("child_idx") is not None:
        arrs["child_idx"] = np.ascontiguousarray(v["child_idx"], np.int32)
    s = OrbvVocab(int(v["nnodes"]), int(v["depth_levels"]), ptr(arrs["first_child"]), ptr(arrs["nchild"]),
                  ptr(arrs["node_desc"]), ptr(arrs["word_id"]), ptr(arrs["weight"]), ptr(arrs.get("child_idx")))
    return Keep(s, list(arrs.values()))


def mappoints_struct(proj_x, proj_y, proj_xr, level, view_cos, track_depth, in_view, has_obs, desc) -> Keep:
    a = [np.ascontiguousarray(proj_x, np.float32), np.ascontiguousarray(proj_y, np.float32),
         np.ascontiguousarray(proj_xr, np.float32), np.ascontiguousarray(level, np.int32),
         np.ascontiguousarray(view_cos, np.float32), np.ascontiguousarray(track_depth, np.float32),
         np.ascontiguousarray(in_view, np.uint8), np.ascontiguousarray(has_obs, np.uint8),
         np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)]
    s = OrbmMapPoints(len(a[0]), *[ptr(x) for x in a])
    return Keep(s, a)


def mappoints_right_struct(in_view, proj_x, proj_y, level, view_cos) -> Keep:
    """orbm_mappoints_right: MapPoint mbTrackInViewR (&& !isBad), mTrackProjXR/YR, mnTrackScaleLevelR,
    mTrackViewCosR."""
    a = [np.ascontiguousarray(in_view, np.uint8), np.ascontiguousarray(proj_x, np.float32),
         np.ascontiguousarray(proj_y, np.float32), np.ascontiguousarray(level, np.int32),
         np.ascontiguousarray(view_cos, np.float32)]
    return Keep(OrbmMapPointsRight(*[ptr(x) for x in a]), a)
