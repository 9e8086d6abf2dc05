"""HBM-resident keyframe map for map-wide SearchByBoW (orbm_search_by_bow_batch_device).

Mirrors what relocalization does per candidate keyframe (reference
src/Tracking.cc:3641-3648: one ORBmatcher(0.75, true).SearchByBoW(KF_i, F)
per candidate) for a whole (shard of a) keyframe map at once.  Keyframes are
concatenated: features (orb_keypoint, 32-B descriptor, MapPoint validity) and
their FeatureVector as CSR (DBoW2 FeatureVector.h:24-25).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi, capi


class OrbmKfMapDevice(C.Structure):
    _fields_ = [("nkf", C.c_int32), ("kps", C.c_void_p), ("desc", C.c_void_p), ("valid", C.c_void_p),
                ("kp_off", C.c_void_p), ("fv_node", C.c_void_p), ("fv_off", C.c_void_p), ("fv_idx", C.c_void_p),
                ("fv_node_off", C.c_void_p), ("fv_idx_off", C.c_void_p),
                ("n_nodes_total", C.c_int64), ("n_fv_total", C.c_int64), ("fv_desc", C.c_void_p),
                ("fv_angle", C.c_void_p)]


def featvec_csr(node_of_feature: np.ndarray):
    """(node_ids, offsets, idx) of a FeatureVector built by addFeature in
    feature order (nodes ascending, feature indices ascending per node)."""
    nid = np.asarray(node_of_feature, dtype=np.int64)
    feats = np.nonzero(nid >= 0)[0]
    feats = feats[np.argsort(nid[feats], kind="stable")]    # by node, feature index ascending within
    sn = nid[feats]
    starts = np.flatnonzero(np.r_[True, sn[1:] != sn[:-1]]) if len(sn) else np.zeros(0, np.int64)
    return sn[starts].astype(np.uint32), np.append(starts, len(feats)).astype(np.int32), feats.astype(np.uint32)


def pack(keyframes) -> dict:
    """The keyframes concatenated in the orbm_kf_map_device layout, as host
    arrays: kps (u8 view of orb_keypoint rows), desc, valid, kp_off, fv_node,
    fv_off, fv_idx, fv_node_off, fv_idx_off (include/orb_mi355x.h).
    keyframes: iterable of (kps KEYPOINT_DTYPE[n], desc u8[n,32], valid u8[n], node_of_feature i[n])."""
    kps, desc, valid, nodes, offs, idxs = [], [], [], [], [], []
    kp_off, node_off, idx_off = [0], [0], []
    nidx = 0
    for k, d, v, nid in keyframes:
        n_ids, o, ix = featvec_csr(nid)
        kps.append(np.ascontiguousarray(k, abi.KEYPOINT_DTYPE).view(np.uint8).reshape(-1))
        desc.append(np.ascontiguousarray(d, np.uint8).reshape(-1))
        valid.append(np.ascontiguousarray(v, np.uint8))
        nodes.append(n_ids)
        offs.append(o)
        idx_off.append(nidx)
        nidx += len(ix)
        idxs.append(ix)
        kp_off.append(kp_off[-1] + len(k))
        node_off.append(node_off[-1] + len(n_ids))
    cat = lambda a, dt: np.ascontiguousarray(np.concatenate(a) if a else np.zeros(0, dt), dt)
    return dict(kps=cat(kps, np.uint8), desc=cat(desc, np.uint8), valid=cat(valid, np.uint8),
                kp_off=np.array(kp_off, np.int64), fv_node=cat(nodes, np.uint32), fv_off=cat(offs, np.int32),
                fv_idx=cat(idxs, np.uint32), fv_node_off=np.array(node_off, np.int64),
                fv_idx_off=np.array(idx_off, np.int64))


def keyframe_view(arrays: dict, i: int):
    """Keyframe i of a packed map as (kps, desc, valid, (node_ids, offsets, idx))."""
    a0, a1 = int(arrays["kp_off"][i]), int(arrays["kp_off"][i + 1])
    n0, n1 = int(arrays["fv_node_off"][i]), int(arrays["fv_node_off"][i + 1])
    i0 = int(arrays["fv_idx_off"][i])
    offs = arrays["fv_off"][n0 + i:n1 + i + 1]
    kps = arrays["kps"][a0 * 28:a1 * 28].view(abi.KEYPOINT_DTYPE)
    return (kps, arrays["desc"][a0 * 32:a1 * 32].reshape(-1, 32), arrays["valid"][a0:a1],
            (arrays["fv_node"][n0:n1], offs, arrays["fv_idx"][i0:i0 + (int(offs[-1]) if len(offs) else 0)]))


class DeviceKeyframeMap:
    def __init__(self, keyframes=None, device="cuda", fv_desc=True, arrays=None, fv_angle=True):
        """keyframes: iterable of (kps KEYPOINT_DTYPE[n], desc u8[n,32], valid u8[n], node_of_feature i[n]),
        or arrays: the same already packed (pack(), synth.keyframe_map()).
        fv_desc / fv_angle: also keep the descriptors / keypoint angles in
        FeatureVector order (map->fv_desc, map->fv_angle)."""
        import torch
        a = arrays if arrays is not None else pack(keyframes)
        self.nkf = len(a["kp_off"]) - 1
        if self.nkf > 0 and int(np.diff(np.asarray(a["kp_off"], np.int64)).max()) >= 1 << 26:
            raise ValueError("a keyframe holds fewer than 2^26 features (orbm_search_by_bow_batch_device)")
        self.t = {name: torch.from_numpy(np.ascontiguousarray(a[name])).to(device)
                  for name in ("kps", "desc", "valid", "kp_off", "fv_node", "fv_off", "fv_idx", "fv_node_off",
                               "fv_idx_off")}
        p = lambda name: self.t[name].data_ptr()
        self.struct = OrbmKfMapDevice(self.nkf, p("kps"), p("desc"), p("valid"), p("kp_off"), p("fv_node"),
                                      p("fv_off"), p("fv_idx"), p("fv_node_off"), p("fv_idx_off"),
                                      int(a["fv_node_off"][-1]), int(len(a["fv_idx"])), None, None)
        self.ready = None
        # the descriptors in FeatureVector order (orbm_kf_map_fv_desc), once per map
        nfv = self.struct.n_fv_total
        self.t["fv_desc"] = torch.empty(max(1, nfv) * 32, dtype=torch.uint8, device=device)
        self.t["fv_angle"] = torch.empty(max(1, nfv), dtype=torch.float32, device=device)
        if (fv_desc or fv_angle) and self.nkf > 0 and torch.device(device).type == "cuda":
            cur = torch.cuda.current_stream(self.t["fv_desc"].device)
            if fv_desc:
                rc = capi.lib().orbm_kf_map_fv_desc(C.byref(self.struct), C.c_void_p(self.t["fv_desc"].data_ptr()),
                                                    C.c_void_p(cur.cuda_stream))
                capi.check(rc, "orbm_kf_map_fv_desc")
                self.struct.fv_desc = self.t["fv_desc"].data_ptr()
            if fv_angle:
                rc = capi.lib().orbm_kf_map_fv_angle(C.byref(self.struct), C.c_void_p(self.t["fv_angle"].data_ptr()),
                                                     C.c_void_p(cur.cuda_stream))
                capi.check(rc, "orbm_kf_map_fv_angle")
                self.struct.fv_angle = self.t["fv_angle"].data_ptr()
            # a search on another stream waits for them (search_prepared)
            self.ready = torch.cuda.Event()
            self.ready.record(cur)

    def prepare_frame(self, kps, desc, node_of_feature):
        """The query frame resident in HBM (keypoints, descriptors, FeatureVector
        CSR) plus its output buffers, for search_prepared."""
        import torch
        dev = self.t["kps"].device
        kps = np.ascontiguousarray(kps, abi.KEYPOINT_DTYPE)
        n = len(kps)
        n_ids, offs, idx = featvec_csr(node_of_feature)
        ft = dict(kps=torch.from_numpy(kps.view(np.uint8).copy()).to(dev),
                  desc=torch.from_numpy(np.ascontiguousarray(desc, np.uint8)).to(dev),
                  node=torch.from_numpy(n_ids.astype(np.int64)).to(dev).to(torch.int32),
                  off=torch.from_numpy(offs).to(dev), idx=torch.from_numpy(idx.astype(np.int64)).to(dev).to(torch.int32),
                  match=torch.empty((self.nkf, n), dtype=torch.int32, device=dev),
                  nm=torch.empty(self.nkf, dtype=torch.int32, device=dev))
        ft["frame"] = abi.OrbmFrame(n, ft["kps"].data_ptr(), ft["desc"].data_ptr(), 0, 0, 0, 0, 0, 0, None, None, 0)
        ft["featvec"] = abi.OrbmFeatVec(len(n_ids), ft["node"].data_ptr(), ft["off"].data_ptr(), ft["idx"].data_ptr())
        return ft

    def search_prepared(self, ft, nnratio=0.75, check_ori=True, stream=None):
        """SearchByBoW(KF_i, F) for every keyframe against a prepared frame:
        (match [nkf, N] int32 KF-feature index or -1, nmatches [nkf]), the
        frame's device output tensors (overwritten by the next call)."""
        import torch
        dev = self.t["kps"].device
        strm = stream or torch.cuda.current_stream(dev)
        if self.ready is not None:
            strm.wait_event(self.ready)
        st = strm.cuda_stream
        rc = capi.lib().orbm_search_by_bow_batch_device(C.byref(self.struct), C.byref(ft["frame"]),
                                                        C.byref(ft["featvec"]), nnratio, int(check_ori),
                                                        ft["match"].data_ptr(), ft["nm"].data_ptr(), C.c_void_p(st))
        capi.check(rc, "orbm_search_by_bow_batch_device")
        return ft["match"], ft["nm"]

    def search_by_bow(self, kps, desc, node_of_feature, nnratio=0.75, check_ori=True, stream=None):
        """SearchByBoW(KF_i, F) for every keyframe: returns (match [nkf, N] int32
        KF-feature index or -1, nmatches [nkf]) as device tensors."""
        ft = self.prepare_frame(kps, desc, node_of_feature)
        self._keep = ft
        return self.search_prepared(ft, nnratio, check_ori, stream)
