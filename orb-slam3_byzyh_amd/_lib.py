"""ctypes binding of liborbgpu.so (the C ABI declared in include/orbgpu.h).

The product path is the HIP library: if it is missing or cannot be loaded this module raises --
there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import pathlib

import numpy as np

PKG_DIR = pathlib.Path(__file__).resolve().parent
LIB_PATH = PKG_DIR / "lib" / "liborbgpu.so"

ORB_OK = 0
ORB_ERR_EMPTY = -1
ORB_ERR_ARG = -2
ORB_ERR_CAPACITY = -3
ORB_ERR_DEVICE = -4
ORB_ERR_ABORTED = -5
ORB_ERR_INTERNAL = -6

# cv::KeyPoint layout (28 bytes)
KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KEYPOINT_DTYPE.itemsize == 28


# orb_pose_edge_t (56 bytes) / orb_pose_frame_t (88 bytes, 8-byte aligned) of include/orbgpu.h
POSE_EDGE_DTYPE = np.dtype([("xw", "<f8", 3), ("obs", "<f8", 3), ("inv_sigma2", "<f4"), ("stereo", "<i4")])
POSE_CAMERA_DTYPE = np.dtype([("fx", "<f4"), ("fy", "<f4"), ("cx", "<f4"), ("cy", "<f4"), ("bf", "<f4")])
POSE_FRAME_DTYPE = np.dtype({"names": ["pose", "cam", "edge_begin", "n_edges"],
                             "formats": [("<f8", 7), POSE_CAMERA_DTYPE, "<i4", "<i4"],
                             "offsets": [0, 56, 76, 80], "itemsize": 88})
assert POSE_EDGE_DTYPE.itemsize == 56


class VocabularyView(ctypes.Structure):  # orb_vocabulary_view_t
    _fields_ = [("k", ctypes.c_int32), ("L", ctypes.c_int32), ("weighting", ctypes.c_int32),
                ("scoring", ctypes.c_int32), ("n_nodes", ctypes.c_int32), ("child_begin", ctypes.c_void_p),
                ("child_idx", ctypes.c_void_p), ("desc", ctypes.c_void_p), ("word_id", ctypes.c_void_p),
                ("weight", ctypes.c_void_p)]


def vocabulary_view(voc: dict) -> tuple:
    """(VocabularyView, keep-alive arrays) for a vocabulary dict (k, L, weighting, scoring,
    child_begin, child_idx, desc [n,32], word_id, weight)."""
    arrs = {"child_begin": np.ascontiguousarray(voc["child_begin"], np.int32),
            "child_idx": np.ascontiguousarray(voc["child_idx"], np.int32),
            "desc": np.ascontiguousarray(voc["desc"], np.uint8), "word_id": np.ascontiguousarray(voc["word_id"], np.int32),
            "weight": np.ascontiguousarray(voc["weight"], np.float64)}
    v = VocabularyView(int(voc["k"]), int(voc["L"]), int(voc.get("weighting", 0)), int(voc.get("scoring", 0)),
                       len(arrs["word_id"]), arrs["child_begin"].ctypes.data, arrs["child_idx"].ctypes.data,
                       arrs["desc"].ctypes.data, arrs["word_id"].ctypes.data, arrs["weight"].ctypes.data)
    return v, arrs


class OrbGpuError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str = ""):
        super().__init__(f"{where} failed with status {code}: {msg}")
        self.code = code


class OrbParams(ctypes.Structure):
    _fields_ = [("nfeatures", ctypes.c_int32), ("scale_factor", ctypes.c_float), ("nlevels", ctypes.c_int32),
                ("ini_th_fast", ctypes.c_int32), ("min_th_fast", ctypes.c_int32)]


_vp, _i, _f, _sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
_ip = ctypes.POINTER(ctypes.c_int)
_fp = ctypes.POINTER(ctypes.c_float)

# (name, restype, argtypes) for every symbol include/orbgpu.h declares
PROTOTYPES = {
    "orb_device_count": (_i, []),
    "orb_last_error": (ctypes.c_char_p, []),
    "orb_extractor_create": (_i, [ctypes.POINTER(OrbParams), _i, _i, _i, ctypes.POINTER(_vp)]),
    "orb_extractor_destroy": (_i, [_vp]),
    "orb_extractor_scales": (_i, [_vp, _fp, _fp, _fp, _fp, _ip]),
    "orb_extract": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp, _vp, _i, _ip]),
    "orb_extract_batch_device": (_i, [_vp, _vp, _i, _i, _i, _i, _sz, _i, _i, _vp, _vp, _i, _vp, _vp]),
    "orb_extractor_set_overlap": (_i, [_vp, _i]),
    "orb_extractor_level": (_i, [_vp, _i, _i, ctypes.POINTER(_vp), _ip, _ip, _ip]),
    "orb_extractor_level_download": (_i, [_vp, _i, _i, _vp]),
    "orb_timers_enable": (_i, [_i]),
    "orb_timers_enabled": (_i, []),
    "orb_timers_reset": (_i, []),
    "orb_timer_add": (_i, [ctypes.c_char_p, ctypes.c_double]),
    "orb_timer_stats": (_i, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                             ctypes.POINTER(ctypes.c_longlong)]),
    "orb_timers_write": (_i, [ctypes.c_char_p]),
    "orb_descriptor_distance": (_i, [_vp, _vp]),
    "orb_hamming_knn2_device": (_i, [_vp, _i, _vp, _i, _vp, _vp, _vp, _vp]),
    "orb_hamming_knn2_frames_device": (_i, [_vp, _vp, _i, _i, _vp, _i, _vp, _vp, _vp, _vp]),
    "orb_matcher_create": (_i, [_f, _i, ctypes.POINTER(_vp)]),
    "orb_matcher_destroy": (_i, [_vp]),
    "orb_compute_distinctive_descriptors": (_i, [_vp, _vp, _vp, _i, _vp, _vp]),
    "orb_compute_distinctive_descriptors_device": (_i, [_vp, _vp, _i, _vp, _vp, _vp]),
    "orb_kf_pair_geometry": (_i, [_vp, _vp, _f, _f, _f, _f, _vp]),
    "orb_search_for_triangulation": (_i, [_vp, _vp, _vp, _vp, _i, _i, _i, _vp, _vp]),
    "orb_search_for_triangulation_device": (_i, [_vp, _vp, _i, _vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp]),
    "orb_search_by_projection_frame": (_i, [_vp, _vp, _vp, _f, _i, _vp, _vp]),
    "orb_search_by_projection_local": (_i, [_vp, _vp, _vp, _vp, _f, _i, _f, _vp, _vp]),
    "orb_compute_stereo_matches": (_i, [_vp, _vp, _vp, _i, _vp, _vp, _i, _vp, _f, _f, _vp, _vp]),
    "orb_compute_stereo_matches_batch_device": (_i, [_vp, _vp, _i, _vp, _vp, _vp, _i, _vp, _vp, _vp, _i, _f, _f, _vp,
                                                     _vp, _vp, _vp]),
    "orb_pose_optimization": (_i, [_i, _vp, _i, _vp, _vp, _vp, _vp]),
    "orb_pose_optimization_device": (_i, [_i, _vp, _i, _vp, _vp, _vp, _vp, _vp]),
    "orb_is_in_frustum": (_i, [_vp, _i, _vp, _vp, _vp, _vp, _f, _vp, _vp, _vp, _vp, _vp]),
    "orb_is_in_frustum_device": (_i, [_vp, _i, _vp, _vp, _vp, _vp, _f, _vp, _vp, _vp, _vp, _vp, _vp]),
    "orb_vocabulary_create": (_i, [_vp, ctypes.POINTER(_vp)]),
    "orb_vocabulary_destroy": (_i, [_vp]),
    "orb_bow_transform": (_i, [_vp, _vp, _i, _i, _vp, _vp, _ip, _vp, _vp, _vp, _ip]),
    "orb_bow_transform_batch_device": (_i, [_vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "orb_bow_transform_frames_device": (_i, [_vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "orb_undistort_keypoints_device": (_i, [_vp, _vp, _i, _i, _vp, _vp, _i, _vp, _vp]),
    "orb_search_by_projection_frame_device": (_i, [_vp, _vp, _vp, _f, _i, _vp, _vp, _vp]),
    "orb_search_by_projection_local_device": (_i, [_vp, _vp, _vp, _vp, _f, _i, _f, _vp, _vp, _vp]),
    "orb_is_in_frustum_pose_device": (_i, [_vp, _vp, _i, _vp, _vp, _vp, _vp, _f, _vp, _vp, _vp, _vp, _vp, _vp]),
    "orb_tracking_pose_edges_device": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "orb_tracking_discard_outliers_device": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _vp, _vp]),
    "orb_tracking_local_seen_device": (_i, [_vp, _i, _i, _vp, _i, _vp, _vp]),
    "orb_tracking_chain_scratch_bytes": (_sz, [_i, _i, _i]),
    "orb_tracking_chain_batch_scratch_bytes": (_sz, [_i, _i, _i, _i]),
    "orb_tracking_chain_batch_release": (_i, [_vp]),
    "orb_tracking_chain_batch_device": (_i, [_vp, _vp, _i, _vp, _vp, _vp, _vp]),
    "orb_tracking_chain_device": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                        _vp]),
    "orb_ba_create": (_i, [ctypes.POINTER(_vp)]),
    "orb_ba_destroy": (_i, [_vp]),
    "orb_ba_optimize": (_i, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "orb_ba_dist_unique_id": (_i, [_vp]),
    "orb_ba_dist_init_rccl": (_i, [_vp, _vp, _i, _i]),
    "orb_ba_dist_init_host": (_i, [_vp, _vp, _vp, _i, _i]),
}

# parity / debugging hooks exported by the library (not part of the public header)
DEBUG_PROTOTYPES = {
    "orb_debug_level_candidates": (_i, [_vp, _i, _i, _vp, _i, _vp, _i]),
    "orb_debug_level_selected": (_i, [_vp, _i, _i, _vp, _i]),
    "orb_debug_level_blurred": (_i, [_vp, _i, _i, _vp]),
    "orb_debug_status": (_i, [_vp]),
    "orb_extractor_profile": (_i, [_vp, _i]),
    "orb_debug_qt_stamps": (_i, [_vp, _vp, _i]),
    "orb_debug_node_sort": (_i, [_vp, _vp, _i, _i, _vp]),
    "orb_extractor_stage_ms": (_i, [_vp, _fp, _ip, ctypes.POINTER(ctypes.c_longlong)]),
    "orb_extractor_pyramid_launch_ms": (_i, [_vp, _fp, _ip]),
    "orb_extractor_launch_durations": (_i, [_vp, _i, _fp, _i, _ip]),
    "orb_debug_ba_chol_timeout": (_i, [_i, _i]),
    "orb_debug_pose_trace": (_i, [_vp, _i]),
    "orb_debug_pose_extra": (_i, [_i]),
    "orb_debug_ba_chol_timeout_status": (_i, [_ip]),
}

STAGES = ("pyramid", "fast", "quadtree", "place", "describe")

_LIB = None


def header_symbols() -> list[str]:
    """Function names declared in include/orbgpu.h (parsed, so the ABI test follows the header)."""
    import re
    hdr = (PKG_DIR.parent / "include" / "orbgpu.h").read_text()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(orb_[a-z0-9_]+)\s*\(", hdr)))


def load(path: os.PathLike | str | None = None) -> ctypes.CDLL:
    """Load liborbgpu.so and declare its prototypes.  Raises if the library was not built."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = pathlib.Path(path) if path else LIB_PATH
    # One HIP runtime per process: torch wheels bundle their own libamdhip64/libhsa-runtime64 (same
    # sonames as /opt/rocm's).  Importing torch first makes liborbgpu.so bind to that already-loaded
    # copy instead of pulling in a second ROCr instance, which would fail to open the device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not p.exists():
        raise FileNotFoundError(f"{p} not found: build it with `make` (or __graft_entry__.build())")
    lib = ctypes.CDLL(str(p))
    for name, (res, args) in {**PROTOTYPES, **DEBUG_PROTOTYPES}.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _LIB = lib
    return lib


def last_error() -> str:
    return load().orb_last_error().decode(errors="replace")


def check(code: int, where: str) -> int:
    if code < 0:
        raise OrbGpuError(code, where, last_error())
    return code


def device_count() -> int:
    return load().orb_device_count()


def require_device() -> None:
    if device_count() <= 0:
        raise OrbGpuError(ORB_ERR_DEVICE, "liborbgpu", "no HIP device visible (the HIP path has no CPU fallback)")
