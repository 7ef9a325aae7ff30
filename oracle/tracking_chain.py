"""ORACLE (test infrastructure only; imported by tests/ and bench.py's cpu_baseline leg): one frame of
Tracking::TrackWithMotionModel -> TrackLocalMap composed from the oracle's restated stages, in the
reference's order (src/Tracking.cc):

    :4149  SearchByProjection(mCurrentFrame, mLastFrame, th, bMono)       oracle_search_by_projection_frame
    :4153-4158  nmatches < 20: cleared, SearchByProjection(..., 2 th, ...) again
    :4161-4168  nmatches < 20: TrackWithMotionModel returns false (status FAIL_SEARCH: nothing more runs)
    :4175  Optimizer::PoseOptimization(&mCurrentFrame)                     oracle_pose_optimization
           (graph: src/Optimizer.cc:93-180, an edge per keypoint holding a map point, in keypoint order)
    :4176-4203  outliers lose their map point (and are marked seen); nmatchesMap      numpy
    :4216  return nmatchesMap >= 10 (else status FAIL_MAP: the local-map stages do not run)
    :4745-4766  SearchLocalPoints skips the points the frame holds or discarded     numpy
    :4770-4790  Frame::isInFrustum(pMP, 0.5) at the optimised pose         oracle_is_in_frustum
           (the pose as Frame::SetPose keeps it: oracle_pose7_to_frame)
    :4825  SearchByProjection(mCurrentFrame, mvpLocalMapPoints, th, ...)  oracle_search_by_projection_local
    :4262  Optimizer::PoseOptimization(&mCurrentFrame)                     oracle_pose_optimization
           (starting from the float round trip of the first result: oracle_pose7_float_roundtrip)

The frames are the product's plain-data Frame / LocalMapPoints views (keyframe.py), which only hold
arrays; every computation here is the oracle's.  The local map is a table whose row j is the last
frame's keypoint last_row[j] (-1: a point the last frame does not hold).

A frame that fails (status bits 2 / 4, the device chain's ORB_TRACK_*) reports what the device chain
documents for the stages the reference does not run (include/orbgpu.h, orb_tracking_chain_params_t):
empty graphs, pose1 = the motion model's pose (FAIL_SEARCH), pose2 = pose1 as Frame::SetPose keeps it,
no local-map matches; the frustum fields are still those at pose1.
"""
from __future__ import annotations

import numpy as np

from . import oracle

POSE_EDGE_DTYPE = np.dtype([("xw", "<f8", 3), ("obs", "<f8", 3), ("inv_sigma2", "<f4"), ("stereo", "<i4")])
_CAM = np.dtype([("fx", "<f4"), ("fy", "<f4"), ("cx", "<f4"), ("cy", "<f4"), ("bf", "<f4")])
POSE_FRAME_DTYPE = np.dtype({"names": ["pose", "cam", "edge_begin", "n_edges"],
                             "formats": [("<f8", 7), _CAM, "<i4", "<i4"], "offsets": [0, 56, 76, 80], "itemsize": 88})


def pose_graph(F, pose7, level_sigma2, m_a, xyz_a, m_b=None, xyz_b=None):
    """PoseOptimization's graph for frame F (src/Optimizer.cc:93-180): an edge per keypoint whose map
    point is m_b[i] (a row of xyz_b) or else m_a[i] (a row of xyz_a), in keypoint order; stereo when
    mvuRight[i] >= 0; information 1 / mvLevelSigma2[octave] (src/Frame.cc:124).  Returns (frame record,
    edges, keypoint of each edge)."""
    use_b = (m_b >= 0) if m_b is not None else np.zeros(F.N, bool)
    use_a = ~use_b & (m_a >= 0)
    kp = np.flatnonzero(use_a | use_b)
    e = np.zeros(len(kp), POSE_EDGE_DTYPE)
    xa = np.asarray(xyz_a, np.float32).reshape(-1, 3)
    xw = xa[np.maximum(m_a, 0)[kp]]
    if m_b is not None:
        xb = np.asarray(xyz_b, np.float32).reshape(-1, 3)
        xw = np.where(use_b[kp, None], xb[np.maximum(m_b, 0)[kp]], xw)
    e["xw"] = xw.astype(np.float64)
    k = F.mvKeysUn[kp]
    ur = F.mvuRight[kp] if F.mvuRight is not None else np.full(len(kp), -1, np.float32)
    st = ur >= 0
    e["obs"][:, 0], e["obs"][:, 1] = k["x"], k["y"]
    e["obs"][:, 2] = np.where(st, ur, 0).astype(np.float64)
    e["stereo"] = st
    inv = (np.float32(1.0) / np.asarray(level_sigma2, np.float32)).astype(np.float32)
    e["inv_sigma2"] = inv[np.clip(k["octave"], 0, len(inv) - 1)]
    fr = np.zeros(1, POSE_FRAME_DTYPE)
    fr["pose"] = pose7
    fr["cam"] = (F.fx, F.fy, F.cx, F.cy, F.mbf)
    fr["n_edges"] = len(kp)
    return fr, e, kp


def track(pkg, C, L, local: dict, pose7_pred, level_sigma2, th_motion: float, th_local: float, mono: bool = False,
          far: bool = False, th_far: float = 20.0, pose1=None, scale_factor: float = 1.2, gate: bool = True):
    """The chain for current frame C (pkg.Frame at the predicted pose), last frame L (pkg.Frame with
    map_points) and the local map `local` (dict: pos, normal, min_dist, max_dist, desc, observed,
    is_bad, last_row).  pose1: when given, the stages after the first PoseOptimization start from it
    (stage-by-stage checking against a device chain).  gate: TrackWithMotionModel's retry and failure
    decisions (False: every stage runs).  Returns a dict of every stage's outputs and `status`."""
    n1, m1 = oracle.search_by_projection_frame(C, L, th_motion, mono, True)
    status = 0
    if gate and n1 < 20:  # src/Tracking.cc:4153-4158
        status |= 1
        n1, m1 = oracle.search_by_projection_frame(C, L, 2 * th_motion, mono, True)
    if gate and n1 < 20:  # :4161-4168
        status |= 2
    fail_search = bool(status & 2)
    fr1, e1, kp1 = pose_graph(C, pose7_pred, level_sigma2, np.full_like(m1, -1) if fail_search else m1,
                              L.map_points["xyz"])
    P1, O1, I1 = oracle.pose_optimization(fr1, e1)  # (no edges: the start pose, 0 inliers)
    p1 = P1[0] if pose1 is None else np.asarray(pose1, np.float64)
    m1d = m1.copy()
    m1d[kp1[O1]] = -1
    kept = (m1d >= 0) & (not fail_search)
    obs_l = np.asarray(L.map_points["observed"], np.uint8)
    n_map = int(obs_l[m1d[kept]].astype(bool).sum())
    if gate and not fail_search and n_map < 10:  # :4216
        status |= 4
    alive = not (status & 6)
    held1 = m1d >= 0  # (a frame that failed the search keeps its matches: the discard had no graph)
    taken = np.zeros(C.N, np.uint8)
    taken[held1] = obs_l[m1d[held1]] != 0
    Tcw1, Ow1 = oracle.pose7_to_frame(p1)
    ff = pkg.frustum_frame(Tcw1, Ow1, (C.fx, C.fy, C.cx, C.cy), C.mbf, (C.mnMinX, C.mnMaxX, C.mnMinY, C.mnMaxY),
                           scale_factor, len(C.mvScaleFactors))
    tf = oracle.is_in_frustum(ff, local["pos"], local["normal"], local["min_dist"], local["max_dist"], 0.5)
    # mnLastFrameSeen: every point the first search assigned, the discarded outliers included
    # (src/Tracking.cc:4195, 4258)
    held = np.zeros(max(L.N, 1), bool)
    held[m1[m1 >= 0]] = True
    lr = np.asarray(local["last_row"], np.int32)
    seen = (lr >= 0) & held[np.clip(lr, 0, len(held) - 1)]
    in_view = tf["track_in_view"].copy()
    in_view[seen] = 0
    Pm = pkg.LocalMapPoints(track_in_view=in_view, is_bad=local["is_bad"], observed=local["observed"],
                            track_proj=tf["track_proj"], track_view_cos=tf["track_view_cos"],
                            track_depth=tf["track_depth"], track_level=tf["track_level"], desc=local["desc"])
    if alive:
        n2, m2 = oracle.search_by_projection_local(C, Pm, th_local, far, th_far, 0.8, taken)
    else:
        n2, m2 = 0, np.full(C.N, -1, np.int32)
    none = np.full(C.N, -1, np.int32)
    fr2, e2, kp2 = pose_graph(C, oracle.pose7_float_roundtrip(p1), level_sigma2, m1d if alive else none,
                              L.map_points["xyz"], m2, local["pos"])
    P2, O2, I2 = oracle.pose_optimization(fr2, e2)
    return dict(n1=n1, m1_raw=m1, m1=m1d, e1=e1, kp1=kp1, pose1=P1[0], O1=O1, I1=int(I1[0]), n_kept=int(kept.sum()),
                n_map=n_map if not fail_search else 0, taken=taken, in_view=in_view, tf=tf, n2=n2, m2=m2, e2=e2,
                kp2=kp2, pose2=P2[0], O2=O2, I2=int(I2[0]), status=status)
