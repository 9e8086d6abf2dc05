"""ctypes bindings of liborb_mi355x.so (the product C ABI, include/orb_mi355x.h).

There is no CPU fallback: if the library is missing or no device is visible,
every entry point raises.  The shared object is built in-tree by build.py.
"""
from __future__ import annotations

import contextlib
import ctypes as C
from pathlib import Path

from . import abi

LIB_PATH = Path(__file__).resolve().parent / "liborb_mi355x.so"

EXPORTS = [
    "orbx_create", "orbx_destroy", "orbx_get_tables", "orbx_max_keypoints", "orbx_extract", "orbx_extract_batch",
    "orbx_get_level", "orbx_get_batch_level", "orbx_debug_math", "orbx_debug_sort", "orbx_set_host_pyramid",
    "orbx_extract_batch_device", "orbx_debug_stage", "orbm_descriptor_distance", "orbm_search_for_initialization",
    "orbm_search_for_initialization_batch_device", "orbm_search_by_bow", "orbm_search_by_projection_mps",
    "orbm_search_by_projection_last", "orbv_transform", "orbx_set_profiling", "orbx_get_profile", "orbm_search_by_bow_batch_device", "orbm_search_by_bow_many", "orbm_kf_map_fv_desc", "orbm_kf_map_fv_angle",
    "orbx_set_streams", "orbs_compute_stereo_matches", "orbs_compute_stereo_matches_batch_device",
    "orbs_knn_match2", "orbs_fisheye_stereo_candidates_batch_device",
    "orbv_load_text", "orbv_text_vocab_view", "orbv_free_text", "orbv_bow_assemble", "orbv_score",
    "orbk_db_create", "orbk_db_destroy", "orbk_db_upload", "orbk_detect_relocalization_candidates",
    "orbm_fuse", "orbm_search_for_triangulation", "orbm_search_for_triangulation_checked", "orbm_compute_distinctive_descriptors",
    "orbm_search_by_bow_kf", "orbm_search_by_projection_kf", "orbm_search_by_projection_sim3",
    "orbm_search_by_sim3", "orbm_fuse_sim3", "orbm_search_by_bow_fisheye", "orbm_search_by_projection_mps_fisheye",
    "orbm_search_by_projection_last_fisheye", "orbx_set_pyramid_mode", "orbx_pyramid_kernel", "orbv_transform_device",
    "orbx_set_stage_event", "orb_debug_set_option", "orb_debug_get_option",
    "orbm_release_scratch", "orbm_debug_proj_stats", "orbx_debug_pretest", "orbx_debug_plan_info",
    "orbm_dframe_create", "orbm_dframe_destroy", "orbm_dframe_upload", "orbm_dframe_from_extractor",
    "orbm_dframe_set_featvec", "orbm_dframe_count", "orbm_search_by_bow_dframe",
    "orbm_search_by_projection_last_dframe", "orbm_search_by_projection_mps_dframe",
    "orbm_search_for_initialization_dframe",
]

# orb_debug_set_option keys (include/orb_mi355x.h): alternative kernel forms
(ORB_OPT_PROJ_FORM, ORB_OPT_BOW_FORM, ORB_OPT_BOWK_BIG, ORB_OPT_PYR_CNT_END, ORB_OPT_PYR_PRETEST, ORB_OPT_SFI_FORM,
 ORB_OPT_HOST_OUT, ORB_OPT_UPLOAD, ORB_OPT_FAST_CAND_CAP, ORB_OPT_BOW_TRACE, ORB_OPT_QT_FORM) = 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10

_lib = None


def load(path: Path | str = LIB_PATH):
    """dlopen + prototypes, no device call (usable without a GPU)."""
    L = C.CDLL(str(path))
    vp, i32, f32, sz = C.c_void_p, C.c_int, C.c_float, C.c_size_t
    L.orbx_create.restype = vp
    L.orbx_create.argtypes = [vp, i32]
    L.orbx_destroy.argtypes = [vp]
    L.orbx_get_tables.argtypes = [vp] * 7
    L.orbx_max_keypoints.argtypes = [vp, i32, i32]
    L.orbx_extract.argtypes = [vp, vp, i32, i32, sz, i32, i32, vp, vp, i32, vp, vp]
    L.orbx_extract_batch.argtypes = [vp, i32, vp, vp, i32, i32, vp, vp, vp, i32, vp, vp]
    L.orbx_get_level.argtypes = [vp, i32, vp, sz, vp, vp]
    L.orbx_get_batch_level.argtypes = [vp, i32, i32, vp, sz, vp, vp]
    L.orbx_debug_math.argtypes = [i32, i32, C.c_longlong, C.c_longlong, i32, i32, vp]
    L.orbx_debug_sort.argtypes = [i32, i32, vp, vp, vp, vp, vp]
    L.orbx_set_host_pyramid.argtypes = [vp, i32]
    L.orbx_extract_batch_device.argtypes = [vp, i32, vp, sz, sz, i32, i32, i32, i32, vp, vp, i32, vp, vp, vp]
    L.orbx_debug_stage.argtypes = [vp, i32, vp, i32, vp]
    L.orbm_descriptor_distance.argtypes = [vp, vp]
    L.orbm_search_for_initialization.argtypes = [vp, vp, vp, i32, f32, i32, vp]
    L.orbm_search_for_initialization_batch_device.argtypes = [i32, vp, vp, vp, i32, f32, f32, f32, f32, f32, f32,
                                                              i32, f32, i32, vp, vp, vp]
    L.orbm_search_by_bow.argtypes = [vp, vp, vp, vp, vp, f32, i32, vp]
    L.orbm_search_by_projection_mps.argtypes = [vp, vp, f32, i32, f32, f32, vp, vp]
    L.orbm_search_by_projection_last.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, f32, i32, i32, vp, vp]
    L.orbv_transform.argtypes = [vp, i32, vp, i32, vp, vp, vp, i32]
    L.orbx_set_profiling.argtypes = [vp, i32]
    L.orbx_get_profile.argtypes = [vp, vp, i32]
    L.orbm_search_by_bow_batch_device.argtypes = [vp, vp, vp, f32, i32, vp, vp, vp]
    L.orbm_kf_map_fv_desc.argtypes = [vp, vp, vp]
    L.orbm_kf_map_fv_angle.argtypes = [vp, vp, vp]
    L.orbm_search_by_bow_many.argtypes = [i32, vp, vp, vp, vp, vp, f32, i32, vp, vp]
    L.orbx_set_streams.argtypes = [vp, i32]
    L.orbx_set_pyramid_mode.argtypes = [vp, i32]
    L.orbx_pyramid_kernel.argtypes = [vp]
    L.orbv_transform_device.argtypes = [vp, i32, vp, i32, vp, vp, vp, vp]
    L.orbx_set_stage_event.argtypes = [vp, i32, vp]
    L.orb_debug_set_option.argtypes = [i32, i32]
    L.orb_debug_get_option.argtypes = [i32]
    L.orbm_release_scratch.argtypes = [vp, i32]
    L.orbm_debug_proj_stats.argtypes = [vp]
    L.orbx_debug_pretest.argtypes = [vp, i32, i32, vp, sz, vp]
    L.orbx_debug_plan_info.argtypes = [vp, i32, i32, vp, i32]
    L.orbm_compute_distinctive_descriptors.argtypes = [i32, vp, vp, vp, i32]
    L.orbm_fuse.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp, vp, f32, i32, vp, vp]
    L.orbm_search_for_triangulation.argtypes = [vp, vp, vp, vp, vp, vp, vp, f32, f32, vp, i32, i32, i32, i32, vp]
    L.orbm_search_for_triangulation_checked.argtypes = [vp, vp, vp, vp, vp, vp, i32, i32, abi.TRI_CHECK, vp, vp]
    L.orbm_search_by_bow_kf.argtypes = [vp, vp, vp, vp, vp, vp, f32, i32, vp]
    L.orbm_search_by_projection_kf.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp, f32, i32, i32, vp]
    L.orbm_search_by_projection_sim3.argtypes = [vp, i32, vp, vp, vp, vp, vp, f32, f32, vp]
    L.orbm_search_by_sim3.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, f32, vp]
    L.orbm_fuse_sim3.argtypes = [vp, i32, vp, vp, vp, vp, vp, f32, vp, vp]
    L.orbm_search_by_bow_fisheye.argtypes = [vp, vp, vp, vp, vp, i32, f32, i32, vp]
    L.orbm_search_by_projection_mps_fisheye.argtypes = [vp, i32, vp, vp, vp, vp, f32, i32, f32, f32, vp, vp]
    L.orbm_search_by_projection_last_fisheye.argtypes = [vp, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, f32, i32,
                                                         i32, vp, vp]
    L.orbm_dframe_create.restype = vp
    L.orbm_dframe_create.argtypes = [i32]
    L.orbm_dframe_destroy.argtypes = [vp]
    L.orbm_dframe_upload.argtypes = [vp, vp, vp]
    L.orbm_dframe_from_extractor.argtypes = [vp, vp, vp, vp]
    L.orbm_dframe_set_featvec.argtypes = [vp, vp]
    L.orbm_dframe_count.argtypes = [vp]
    L.orbm_search_by_bow_dframe.argtypes = [vp, vp, vp, f32, i32, vp]
    L.orbm_search_by_projection_last_dframe.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, f32, i32, i32, vp,
                                                        vp]
    L.orbm_search_by_projection_mps_dframe.argtypes = [vp, vp, f32, i32, f32, f32, vp, vp]
    L.orbm_search_for_initialization_dframe.argtypes = [vp, vp, vp, i32, f32, i32, vp]
    L.orbk_db_create.restype = vp
    L.orbk_db_create.argtypes = [i32]
    L.orbk_db_destroy.argtypes = [vp]
    L.orbk_db_upload.argtypes = [vp, i32, vp, vp, vp, i32, vp, vp, vp, vp, vp]
    L.orbk_detect_relocalization_candidates.argtypes = [vp, vp, vp, i32, i32, vp, vp, i32]
    L.orbv_load_text.restype = vp
    L.orbv_load_text.argtypes = [C.c_char_p, vp]
    L.orbv_text_vocab_view.argtypes = [vp, vp, vp, vp, vp, vp]
    L.orbv_free_text.argtypes = [vp]
    L.orbv_bow_assemble.argtypes = [i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.orbv_score.restype = C.c_double
    L.orbv_score.argtypes = [i32, vp, vp, i32, vp, vp, i32]
    L.orbs_knn_match2.argtypes = [vp, i32, vp, i32, vp, vp, i32]
    L.orbs_fisheye_stereo_candidates_batch_device.argtypes = [i32, i32, i32, vp, vp, vp, i32, C.c_double, vp, vp,
                                                              vp, vp]
    L.orbs_compute_stereo_matches.argtypes = [vp, vp, vp, i32, vp, vp, i32, vp, f32, f32, vp, vp]
    L.orbs_compute_stereo_matches_batch_device.argtypes = [vp, i32, i32, i32, vp, vp, vp, i32, f32, f32, vp, vp, vp,
                                                           vp]
    return L


def lib():
    """The loaded product library; raises if it is absent (no fallback)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        _lib = load()
    return _lib


def check(rc: int, what: str) -> int:
    if rc < 0:
        names = {abi.ORB_ERR_EMPTY: "empty image", abi.ORB_ERR_CAPACITY: "capacity", abi.ORB_ERR_PARAM: "bad parameter",
                 abi.ORB_ERR_DEVICE: "HIP device error", abi.ORB_ERR_UNSUPPORTED: "unsupported configuration"}
        raise RuntimeError(f"{what} failed: {names.get(rc, rc)}")
    return rc


@contextlib.contextmanager
def debug_option(option: int, value: int):
    """Selects an alternative kernel form (orb_debug_set_option, a test hook)
    for the duration of the block, then restores the previous value."""
    L = lib()
    old = L.orb_debug_get_option(option)
    check(L.orb_debug_set_option(option, value), "orb_debug_set_option")
    try:
        yield
    finally:
        L.orb_debug_set_option(option, old)
