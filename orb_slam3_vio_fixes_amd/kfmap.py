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
                ("n_nodes_total", C.c_int64), ("n_fv_total", C.c_int64), ("fv_desc", C.c_void_p)]


def featvec_csr(node_of_feature: np.ndarray):
    """(node_ids, offsets, idx) of a FeatureVector built by addFeature in
    feature order (nodes ascending, feature indices ascending per node)."""
    nid = np.asarray(node_of_feature, dtype=np.int64)
    feats = np.nonzero(nid >= 0)[0]
    order = np.lexsort((feats, nid[feats]))
    feats = feats[order]
    nodes, starts = np.unique(nid[feats], return_index=True)
    return nodes.astype(np.uint32), np.append(starts, len(feats)).astype(np.int32), feats.astype(np.uint32)


class DeviceKeyframeMap:
    def __init__(self, keyframes, device="cuda", fv_desc=True):
        """keyframes: iterable of (kps KEYPOINT_DTYPE[n], desc u8[n,32], valid u8[n], node_of_feature i[n]).
        fv_desc: also keep the descriptors in FeatureVector order (map->fv_desc)."""
        import torch
        kps, desc, valid, nodes, offs, idxs = [], [], [], [], [], []
        kp_off, node_off, idx_off = [0], [0], []
        for k, d, v, nid in keyframes:
            n_ids, o, ix = featvec_csr(nid)
            kps.append(np.ascontiguousarray(k, abi.KEYPOINT_DTYPE).view(np.uint8).reshape(-1))
            desc.append(np.ascontiguousarray(d, np.uint8).reshape(-1))
            valid.append(np.ascontiguousarray(v, np.uint8))
            nodes.append(n_ids)
            offs.append(o)
            idx_off.append(sum(len(x) for x in idxs))
            idxs.append(ix)
            kp_off.append(kp_off[-1] + len(k))
            node_off.append(node_off[-1] + len(n_ids))
        self.nkf = len(kp_off) - 1
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(np.concatenate(a) if a else np.zeros(0, dt), dt)).to(device)
        self.t = dict(kps=t(kps, np.uint8), desc=t(desc, np.uint8), valid=t(valid, np.uint8),
                      kp_off=t([np.array(kp_off, np.int64)], np.int64), fv_node=t(nodes, np.uint32),
                      fv_off=t(offs, np.int32), fv_idx=t(idxs, np.uint32),
                      fv_node_off=t([np.array(node_off, np.int64)], np.int64),
                      fv_idx_off=t([np.array(idx_off, np.int64)], np.int64))
        p = lambda name: self.t[name].data_ptr()
        self.struct = OrbmKfMapDevice(self.nkf, p("kps"), p("desc"), p("valid"), p("kp_off"), p("fv_node"),
                                      p("fv_off"), p("fv_idx"), p("fv_node_off"), p("fv_idx_off"),
                                      node_off[-1], sum(len(x) for x in idxs), None)
        # the descriptors in FeatureVector order (orbm_kf_map_fv_desc), once per map
        nfv = self.struct.n_fv_total
        self.t["fv_desc"] = torch.empty(max(1, nfv) * 32, dtype=torch.uint8, device=device)
        if fv_desc and self.nkf > 0 and torch.device(device).type == "cuda":
            st = torch.cuda.current_stream(self.t["fv_desc"].device).cuda_stream
            rc = capi.lib().orbm_kf_map_fv_desc(C.byref(self.struct), C.c_void_p(self.t["fv_desc"].data_ptr()),
                                                C.c_void_p(st))
            capi.check(rc, "orbm_kf_map_fv_desc")
            self.struct.fv_desc = self.t["fv_desc"].data_ptr()

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
        st = (stream or torch.cuda.current_stream(dev)).cuda_stream
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
