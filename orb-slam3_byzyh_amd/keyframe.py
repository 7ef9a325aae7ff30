"""Flat keyframe view for the matcher ABI (orb_kf_view_t in include/orbgpu.h).

Holds the KeyFrame fields ORBmatcher::SearchForTriangulation reads (reference
src/ORBmatcher.cc:1046-1324): mvKeysUn, mDescriptors, mvuRight, the map-point slots (as flags),
mFeatVec (DBoW2::FeatureVector, a std::map node id -> feature indices) as CSR arrays, the pose
Tcw and the pinhole intrinsics, mvScaleFactors and mvLevelSigma2.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import KEYPOINT_DTYPE


class KfView(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("kps_un", ctypes.c_void_p), ("desc", ctypes.c_void_p),
                ("u_right", ctypes.c_void_p), ("has_mappoint", ctypes.c_void_p), ("n_nodes", ctypes.c_int32),
                ("fv_node", ctypes.c_void_p), ("fv_offset", ctypes.c_void_p), ("fv_index", ctypes.c_void_p),
                ("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float),
                ("nlevels", ctypes.c_int32), ("scale_factors", ctypes.c_void_p), ("level_sigma2", ctypes.c_void_p)]


class PairGeom(ctypes.Structure):
    _fields_ = [("R12", ctypes.c_float * 9), ("t12", ctypes.c_float * 3), ("ep", ctypes.c_float * 2)]


def _ptr(a):
    return None if a is None else a.ctypes.data


class KeyFrame:
    """Keyframe data for the matcher.  feat_vec: dict node_id -> list of feature indices."""

    def __init__(self, keys_un, descriptors, Tcw, camera, scale_factors, level_sigma2, u_right=None,
                 has_mappoint=None, feat_vec=None):
        self.mvKeysUn = np.ascontiguousarray(keys_un, dtype=KEYPOINT_DTYPE)
        self.N = len(self.mvKeysUn)
        self.mDescriptors = np.ascontiguousarray(descriptors, dtype=np.uint8).reshape(self.N, 32)
        self.Tcw = np.ascontiguousarray(Tcw, dtype=np.float32).reshape(3, 4)
        self.fx, self.fy, self.cx, self.cy = (float(np.float32(v)) for v in camera)
        self.mvScaleFactors = np.ascontiguousarray(scale_factors, dtype=np.float32)
        self.mvLevelSigma2 = np.ascontiguousarray(level_sigma2, dtype=np.float32)
        self.mvuRight = None if u_right is None else np.ascontiguousarray(u_right, dtype=np.float32)
        self.has_mappoint = None if has_mappoint is None else np.ascontiguousarray(has_mappoint, dtype=np.uint8)
        feat_vec = feat_vec or {}
        nodes = sorted(feat_vec)
        self.fv_node = np.asarray(nodes, dtype=np.uint32)
        self.fv_offset = np.zeros(len(nodes) + 1, np.int32)
        idx = []
        for i, k in enumerate(nodes):
            idx.extend(feat_vec[k])
            self.fv_offset[i + 1] = len(idx)
        self.fv_index = np.asarray(idx, dtype=np.int32)
        self._view = None

    @property
    def mFeatVec(self) -> dict:
        return {int(k): self.fv_index[self.fv_offset[i]:self.fv_offset[i + 1]].tolist()
                for i, k in enumerate(self.fv_node)}

    def view(self) -> KfView:
        if self._view is None:
            self._view = KfView(self.N, _ptr(self.mvKeysUn), _ptr(self.mDescriptors), _ptr(self.mvuRight),
                                _ptr(self.has_mappoint), len(self.fv_node), _ptr(self.fv_node), _ptr(self.fv_offset),
                                _ptr(self.fv_index), self.fx, self.fy, self.cx, self.cy, len(self.mvScaleFactors),
                                _ptr(self.mvScaleFactors), _ptr(self.mvLevelSigma2))
        return self._view


class KfDeviceView(ctypes.Structure):  # orb_kf_device_t
    _fields_ = [("kps", ctypes.c_void_p), ("desc", ctypes.c_void_p), ("n", ctypes.c_void_p), ("u_right", ctypes.c_void_p),
                ("has_mappoint", ctypes.c_void_p), ("fv_node", ctypes.c_void_p), ("fv_begin", ctypes.c_void_p),
                ("fv_feat", ctypes.c_void_p), ("n_nodes", ctypes.c_void_p), ("cap", ctypes.c_int32),
                ("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float),
                ("nlevels", ctypes.c_int32), ("scale_factors", ctypes.c_void_p), ("level_sigma2", ctypes.c_void_p)]


class DeviceKeyFrame:
    """A keyframe whose features never left the GPU: frame `f` of the outputs of
    ORBextractor.extract_batch_device (kps, desc, counts), compute_stereo_matches_batch_device (u_right,
    optional) and ORBVocabulary.transform_frames_device (bow), plus the pose and intrinsics the pair
    geometry needs.  has_mappoint: optional [B, cap] uint8 CUDA tensor."""

    def __init__(self, extracted, bow, f: int, Tcw, camera, scale_factors, level_sigma2, u_right=None,
                 has_mappoint=None):
        kps, desc, counts = extracted
        self._keep = (kps, desc, counts, bow, u_right, has_mappoint)
        self.cap = int(kps.shape[1])
        self.f = int(f)
        self.Tcw = np.ascontiguousarray(Tcw, dtype=np.float32).reshape(3, 4)
        self.fx, self.fy, self.cx, self.cy = (float(np.float32(v)) for v in camera)
        self.mvScaleFactors = np.ascontiguousarray(scale_factors, dtype=np.float32)
        self.mvLevelSigma2 = np.ascontiguousarray(level_sigma2, dtype=np.float32)
        cap, f = self.cap, self.f
        fv_node, fv_begin, fv_feat, bcounts = bow[2], bow[3], bow[4], bow[5]
        self._view = KfDeviceView(kps.data_ptr() + 28 * cap * f, desc.data_ptr() + 32 * cap * f,
                                  counts.data_ptr() + 8 * f, None if u_right is None else u_right.data_ptr() + 4 * cap * f,
                                  None if has_mappoint is None else has_mappoint.data_ptr() + cap * f,
                                  fv_node.data_ptr() + 4 * cap * f, fv_begin.data_ptr() + 4 * (cap + 1) * f,
                                  fv_feat.data_ptr() + 4 * cap * f, bcounts.data_ptr() + 8 * f + 4, cap, self.fx,
                                  self.fy, self.cx, self.cy, len(self.mvScaleFactors), self.mvScaleFactors.ctypes.data,
                                  self.mvLevelSigma2.ctypes.data)

    def view(self) -> KfDeviceView:
        return self._view


class FrameView(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("kps_un", ctypes.c_void_p), ("desc", ctypes.c_void_p),
                ("u_right", ctypes.c_void_p), ("min_x", ctypes.c_float), ("max_x", ctypes.c_float),
                ("min_y", ctypes.c_float), ("max_y", ctypes.c_float), ("grid_inv_w", ctypes.c_float),
                ("grid_inv_h", ctypes.c_float), ("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float),
                ("cy", ctypes.c_float), ("bf", ctypes.c_float), ("b", ctypes.c_float), ("nlevels", ctypes.c_int32),
                ("scale_factors", ctypes.c_void_p), ("Tcw", ctypes.c_float * 12)]


class LastPoints(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("valid", ctypes.c_void_p), ("observed", ctypes.c_void_p),
                ("xyz", ctypes.c_void_p), ("desc", ctypes.c_void_p), ("kps_un", ctypes.c_void_p),
                ("Tcw", ctypes.c_float * 12)]


FRAME_GRID_COLS, FRAME_GRID_ROWS = 64, 48  # include/Frame.h:44-45


class Frame:
    """The Frame fields SearchByProjection reads (src/Frame.cc; pinhole, no second camera)."""

    def __init__(self, keys_un, descriptors, Tcw, camera, scale_factors, width, height, bf=0.0, u_right=None,
                 map_points=None):
        self.mvKeysUn = np.ascontiguousarray(keys_un, dtype=KEYPOINT_DTYPE)
        self.N = len(self.mvKeysUn)
        self.mDescriptors = np.ascontiguousarray(descriptors, dtype=np.uint8).reshape(self.N, 32)
        self.Tcw = np.ascontiguousarray(Tcw, dtype=np.float32).reshape(3, 4)
        self.fx, self.fy, self.cx, self.cy = (float(np.float32(v)) for v in camera)
        self.mvScaleFactors = np.ascontiguousarray(scale_factors, dtype=np.float32)
        self.mbf = float(np.float32(bf))
        self.mb = float(np.float32(np.float32(bf) / np.float32(self.fx))) if bf else 0.0
        self.mvuRight = None if u_right is None else np.ascontiguousarray(u_right, dtype=np.float32)
        # undistorted image bounds (no distortion: the image rectangle, Frame::ComputeImageBounds)
        self.mnMinX, self.mnMaxX, self.mnMinY, self.mnMaxY = 0.0, float(width), 0.0, float(height)
        self.mfGridElementWidthInv = float(np.float32(FRAME_GRID_COLS) / np.float32(self.mnMaxX - self.mnMinX))
        self.mfGridElementHeightInv = float(np.float32(FRAME_GRID_ROWS) / np.float32(self.mnMaxY - self.mnMinY))
        # tracked map points, for use as a LastFrame: dict with valid, observed, xyz, desc arrays
        self.map_points = map_points

    def view(self) -> FrameView:
        v = FrameView(self.N, _ptr(self.mvKeysUn), _ptr(self.mDescriptors), _ptr(self.mvuRight), self.mnMinX,
                      self.mnMaxX, self.mnMinY, self.mnMaxY, self.mfGridElementWidthInv, self.mfGridElementHeightInv,
                      self.fx, self.fy, self.cx, self.cy, self.mbf, self.mb, len(self.mvScaleFactors),
                      _ptr(self.mvScaleFactors))
        v.Tcw[:] = [float(x) for x in self.Tcw.reshape(-1)]
        self._keep = v
        return v

    def last_points(self) -> LastPoints:
        mp = self.map_points
        self._mp_arrays = {k: np.ascontiguousarray(mp[k], dtype=dt) for k, dt in
                           (("valid", np.uint8), ("observed", np.uint8), ("xyz", np.float32), ("desc", np.uint8))}
        a = self._mp_arrays
        v = LastPoints(self.N, _ptr(a["valid"]), _ptr(a["observed"]), _ptr(a["xyz"]), _ptr(a["desc"]),
                       _ptr(self.mvKeysUn))
        v.Tcw[:] = [float(x) for x in self.Tcw.reshape(-1)]
        self._keep_last = v
        return v


class LocalPointsView(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("track_in_view", ctypes.c_void_p), ("is_bad", ctypes.c_void_p),
                ("observed", ctypes.c_void_p), ("track_proj", ctypes.c_void_p), ("track_view_cos", ctypes.c_void_p),
                ("track_depth", ctypes.c_void_p), ("track_level", ctypes.c_void_p), ("desc", ctypes.c_void_p)]


class LocalMapPoints:
    """Local map points with the tracking fields Frame::isInFrustum sets (src/Frame.cc:667-773)."""

    _fields = (("track_in_view", np.uint8), ("is_bad", np.uint8), ("observed", np.uint8), ("track_proj", np.float32),
               ("track_view_cos", np.float32), ("track_depth", np.float32), ("track_level", np.int32),
               ("desc", np.uint8))

    def __init__(self, **arrays):
        for k, dt in self._fields:
            setattr(self, k, np.ascontiguousarray(arrays[k], dtype=dt))
        self.n = len(self.track_in_view)

    def view(self) -> LocalPointsView:
        self._v = LocalPointsView(self.n, *[_ptr(getattr(self, k)) for k, _ in self._fields])
        return self._v


class FrustumFrame(ctypes.Structure):  # orb_frustum_frame_t
    _fields_ = [("Tcw", ctypes.c_float * 12), ("Ow", ctypes.c_float * 3), ("fx", ctypes.c_float), ("fy", ctypes.c_float),
                ("cx", ctypes.c_float), ("cy", ctypes.c_float), ("bf", ctypes.c_float), ("min_x", ctypes.c_float),
                ("max_x", ctypes.c_float), ("min_y", ctypes.c_float), ("max_y", ctypes.c_float),
                ("log_scale_factor", ctypes.c_float), ("n_levels", ctypes.c_int32)]


_LIBM = None


def logf(x: float) -> np.float32:
    """glibc's logf: the float overload the reference's unqualified log(float) resolves to
    (`using namespace std` from Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:36)."""
    global _LIBM
    if _LIBM is None:
        _LIBM = ctypes.CDLL("libm.so.6")
        _LIBM.logf.restype = ctypes.c_float
        _LIBM.logf.argtypes = [ctypes.c_float]
    return np.float32(_LIBM.logf(float(np.float32(x))))


def frustum_frame(Tcw, Ow, camera, bf, bounds, scale_factor: float = 1.2, n_levels: int = 8) -> FrustumFrame:
    """orb_frustum_frame_t of a Frame: Tcw 3x4 (mRcw | mtcw), Ow = mOw, camera (fx, fy, cx, cy), mbf,
    bounds (mnMinX, mnMaxX, mnMinY, mnMaxY); mfLogScaleFactor = logf(mfScaleFactor) (src/Frame.cc:121)."""
    T = np.asarray(Tcw, np.float32).reshape(12)
    lsf = logf(scale_factor)
    return FrustumFrame((ctypes.c_float * 12)(*T), (ctypes.c_float * 3)(*np.asarray(Ow, np.float32)), *[float(c) for c in camera],
                        float(bf), *[float(b) for b in bounds], float(lsf), int(n_levels))


def is_in_frustum(frame: FrustumFrame, pos, normal, min_dist, max_dist, viewing_cos_limit: float = 0.5) -> dict:
    """Frame::isInFrustum (src/Frame.cc:667-773) for n map points on the GPU.  Returns the tracking
    fields LocalMapPoints takes: track_in_view, track_proj (n x 3), track_depth, track_level,
    track_view_cos (fields of rejected points as documented in include/orbgpu.h)."""
    from . import _lib
    from ._lib import check
    P = np.ascontiguousarray(pos, np.float32).reshape(-1, 3)
    n = len(P)
    Nn = np.ascontiguousarray(normal, np.float32).reshape(-1, 3)
    mn = np.ascontiguousarray(min_dist, np.float32)
    mx = np.ascontiguousarray(max_dist, np.float32)
    out = dict(track_in_view=np.zeros(max(n, 1), np.uint8), track_proj=np.zeros((max(n, 1), 3), np.float32),
               track_depth=np.zeros(max(n, 1), np.float32), track_level=np.zeros(max(n, 1), np.int32),
               track_view_cos=np.zeros(max(n, 1), np.float32))
    check(_lib.load().orb_is_in_frustum(ctypes.byref(frame), n, _ptr(P), _ptr(Nn), _ptr(mn), _ptr(mx),
                                        float(viewing_cos_limit), _ptr(out["track_in_view"]), _ptr(out["track_proj"]),
                                        _ptr(out["track_depth"]), _ptr(out["track_level"]), _ptr(out["track_view_cos"])),
          "orb_is_in_frustum")
    return {k: v[:n] for k, v in out.items()}
