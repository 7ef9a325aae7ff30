"""The device-resident tracking chain: one frame of Tracking::TrackWithMotionModel -> TrackLocalMap
(reference src/Tracking.cc:4112-4217, 4234-4300, 4742-4825) with every stage on the GPU and no host
round trip between them:

    SearchByProjection(CurrentFrame, LastFrame, th)         orb_search_by_projection_frame_device
    Optimizer::PoseOptimization                             orb_tracking_pose_edges_device +
                                                            orb_pose_optimization_device
    Frame::isInFrustum of the local map at the new pose     orb_is_in_frustum_pose_device +
        (points the first search assigned are skipped)      orb_tracking_local_seen_device
    discard the outliers (nmatchesMap, SearchLocalPoints'   orb_tracking_discard_outliers_device
        skip set)
    SearchByProjection(Frame, local map points, th)         orb_search_by_projection_local_device
    Optimizer::PoseOptimization                             (edges from both searches) + pose kernel

isInFrustum and the seen marks run before the discard here: they read the first pose and the first
search's assignments, which the discard does not change (the reference marks its discarded outliers
seen too, src/Tracking.cc:4195), so the order gives the reference's result.

TrackWithMotionModel's decisions run on the device too (gate=True, src/Tracking.cc:4149-4217): fewer
than 20 matches -> the search again with 2 th; still fewer -> the frame fails (no PoseOptimization,
no local-map stages); nmatchesMap < 10 after the first PoseOptimization -> it fails as well.  The
result's `status` holds the ORB_TRACK_* bits (RETRIED 1, FAIL_SEARCH 2, FAIL_MAP 4); a failed frame is
the caller's to hand to TrackReferenceKeyFrame, as Tracking::Track does.

The current frame is frame `f` of device arrays (ORBextractor.extract_batch_device, optionally
undistort_keypoints_device, compute_stereo_matches_batch_device).  The last frame's tracked map points
are a table indexed by its keypoints (Frame::mvpMapPoints with MapPoint::GetWorldPos / GetDescriptor /
Observations); the local map (Tracking::mvpLocalMapPoints, as UpdateLocalMap leaves it) is a second
table with the fields isInFrustum reads.  What the chain does not cover (the caller's): the motion
model's pose prediction (mVelocity * mLastFrame.GetPose()), UpdateLocalMap's keyframe / point
selection, the MapPoint counters (IncreaseVisible / IncreaseFound) and the IMU / relocalisation paths.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import POSE_EDGE_DTYPE, POSE_FRAME_DTYPE, check
from .keyframe import FRAME_GRID_COLS, FRAME_GRID_ROWS, FrustumFrame, logf
from .matcher import ORBmatcher


class FrameDeviceView(ctypes.Structure):  # orb_frame_device_t
    _fields_ = [("kps_un", ctypes.c_void_p), ("desc", ctypes.c_void_p), ("n", ctypes.c_void_p),
                ("u_right", ctypes.c_void_p), ("cap", ctypes.c_int32), ("min_x", ctypes.c_float),
                ("max_x", ctypes.c_float), ("min_y", ctypes.c_float), ("max_y", ctypes.c_float),
                ("grid_inv_w", ctypes.c_float), ("grid_inv_h", ctypes.c_float), ("fx", ctypes.c_float),
                ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float), ("bf", ctypes.c_float),
                ("b", ctypes.c_float), ("nlevels", ctypes.c_int32), ("scale_factors", ctypes.c_void_p),
                ("Tcw", ctypes.c_float * 12)]


class LastPointsDeviceView(ctypes.Structure):  # orb_last_points_device_t
    _fields_ = [("n", ctypes.c_void_p), ("cap", ctypes.c_int32), ("valid", ctypes.c_void_p),
                ("observed", ctypes.c_void_p), ("xyz", ctypes.c_void_p), ("desc", ctypes.c_void_p),
                ("kps_un", ctypes.c_void_p), ("Tcw", ctypes.c_float * 12)]


class LocalPointsDeviceView(ctypes.Structure):  # orb_local_points_device_t
    _fields_ = [("n", ctypes.c_int32), ("track_in_view", ctypes.c_void_p), ("is_bad", ctypes.c_void_p),
                ("observed", ctypes.c_void_p), ("track_proj", ctypes.c_void_p), ("track_view_cos", ctypes.c_void_p),
                ("track_depth", ctypes.c_void_p), ("track_level", ctypes.c_void_p), ("desc", ctypes.c_void_p)]


class TrackingChainParams(ctypes.Structure):  # orb_tracking_chain_params_t
    _fields_ = [("th_motion", ctypes.c_float), ("mono", ctypes.c_int32), ("th_local", ctypes.c_float),
                ("far_points", ctypes.c_int32), ("th_far_points", ctypes.c_float),
                ("viewing_cos_limit", ctypes.c_float), ("motion_gate", ctypes.c_int32)]


class TrackingChainBuffers(ctypes.Structure):  # orb_tracking_chain_buffers_t
    _fields_ = [(k, ctypes.c_void_p) for k in ("m1", "m2", "n_match", "frames", "edges1", "edges2", "edge_kp1",
                                               "edge_kp2", "outlier1", "outlier2", "poses", "inliers", "n_out",
                                               "taken", "scratch", "status")]

ORB_TRACK_RETRIED, ORB_TRACK_FAIL_SEARCH, ORB_TRACK_FAIL_MAP = 1, 2, 4


def _alloc_scratch(need: int, have, device):
    """A uint8 device buffer of at least `need` bytes, grown geometrically (1.5x) past `have`'s size so a
    slowly growing workload reallocates O(log) times.  The size is the SearchByProjection candidate lists'
    (orb_tracking_chain_*scratch_bytes: cap x points x 8 B per frame)."""
    import torch
    size = max(need, int(1.5 * have.numel())) if have.numel() else need
    try:
        return torch.empty(size, dtype=torch.uint8, device=device)
    except torch.cuda.OutOfMemoryError as e:
        raise MemoryError(f"tracking chain scratch of {size} bytes (cap x max(last-frame cap, local points) x 8 B "
                          f"per frame) does not fit in device memory: lower cap or the local map size") from e


def _stream_handle(stream, device):
    import torch
    st = stream if stream is not None else torch.cuda.current_stream(device)
    return ctypes.c_void_p(st.cuda_stream)


class DeviceFrame:
    """A Frame whose features live on the GPU: frame `f` of kps_un [B, cap, 7] (cv::KeyPoint rows,
    mvKeysUn), desc [B, cap, 32], counts [B, 2] (N at counts[f, 0]) and optionally u_right [B, cap]
    (mvuRight).  Host fields: the pose Tcw (3 x 4), camera (fx, fy, cx, cy), mvScaleFactors,
    mvLevelSigma2, mbf and the undistorted image bounds (mnMinX, mnMaxX, mnMinY, mnMaxY; default the
    image rectangle, Frame::ComputeImageBounds without distortion, src/Frame.cc:1053-1100)."""

    def __init__(self, kps_un, desc, counts, f: int, Tcw, camera, scale_factors, level_sigma2, width: int,
                 height: int, bf: float = 0.0, u_right=None, bounds=None):
        self._keep = (kps_un, desc, counts, u_right)
        self.device = kps_un.device
        self.cap = int(kps_un.shape[1])
        self.f = int(f)
        self.fx, self.fy, self.cx, self.cy = (float(np.float32(v)) for v in camera)
        self.mvScaleFactors = np.ascontiguousarray(scale_factors, np.float32)
        self.mvLevelSigma2 = np.ascontiguousarray(level_sigma2, np.float32)
        self.mvInvLevelSigma2 = (np.float32(1.0) / self.mvLevelSigma2).astype(np.float32)  # src/Frame.cc:124
        self._inv_sigma2_ptr = self.mvInvLevelSigma2.ctypes.data  # (a batch record per call reads it)
        self.mbf = float(np.float32(bf))
        self.mb = float(np.float32(np.float32(bf) / np.float32(self.fx))) if bf else 0.0
        b = (0.0, float(width), 0.0, float(height)) if bounds is None else tuple(float(v) for v in bounds)
        self.mnMinX, self.mnMaxX, self.mnMinY, self.mnMaxY = b
        gw = float(np.float32(FRAME_GRID_COLS) / np.float32(self.mnMaxX - self.mnMinX))
        gh = float(np.float32(FRAME_GRID_ROWS) / np.float32(self.mnMaxY - self.mnMinY))
        cap, f = self.cap, self.f
        self._view = FrameDeviceView(kps_un.data_ptr() + 28 * cap * f, desc.data_ptr() + 32 * cap * f,
                                     counts.data_ptr() + 8 * f,
                                     None if u_right is None else u_right.data_ptr() + 4 * cap * f, cap, self.mnMinX,
                                     self.mnMaxX, self.mnMinY, self.mnMaxY, gw, gh, self.fx, self.fy, self.cx, self.cy,
                                     self.mbf, self.mb, len(self.mvScaleFactors), self.mvScaleFactors.ctypes.data)
        self.set_pose(Tcw)

    def set_pose(self, Tcw) -> None:
        self.Tcw = np.ascontiguousarray(Tcw, np.float32).reshape(3, 4)
        self._view.Tcw[:] = [float(x) for x in self.Tcw.reshape(-1)]
        self._ff = None
        self._pose_version = getattr(self, "_pose_version", 0) + 1  # (DeviceLastPoints copies it on change)

    def view(self) -> FrameDeviceView:
        return self._view

    def frustum_frame(self, scale_factor: float = 1.2) -> FrustumFrame:
        """orb_frustum_frame_t of this frame (pose fields unused by orb_is_in_frustum_pose_device)."""
        key = float(scale_factor)
        if getattr(self, "_ff", None) is not None and self._ff[0] == key:
            return self._ff[1]
        T = self.Tcw.reshape(12)
        ff = FrustumFrame((ctypes.c_float * 12)(*T), (ctypes.c_float * 3)(0, 0, 0), self.fx, self.fy, self.cx,
                          self.cy, self.mbf, self.mnMinX, self.mnMaxX, self.mnMinY, self.mnMaxY,
                          float(logf(scale_factor)), len(self.mvScaleFactors))
        self._ff = (key, ff)
        return ff


class DeviceLastPoints:
    """The last frame's tracked map points, device arrays indexed like its keypoints: valid
    (mvpMapPoints[i] && !mvbOutlier[i]), observed (Observations() > 0), xyz (GetWorldPos, cap x 3
    float32), desc (GetDescriptor, cap x 32).  `frame` is the last frame (its keypoints, N and pose)."""

    def __init__(self, frame: DeviceFrame, valid, observed, xyz, desc):
        self.frame = frame
        self._keep = (valid, observed, xyz, desc)
        self.xyz = xyz
        self.observed = observed
        self.cap = frame.cap
        fv = frame.view()
        self._view = LastPointsDeviceView(fv.n, frame.cap, valid.data_ptr(), observed.data_ptr(), xyz.data_ptr(),
                                          desc.data_ptr(), fv.kps_un)
        self._view.Tcw[:] = list(fv.Tcw)
        self._pose_version = frame._pose_version

    def view(self) -> LastPointsDeviceView:
        if self._pose_version != self.frame._pose_version:  # the last frame's pose changed since
            self._view.Tcw[:] = list(self.frame.view().Tcw)
            self._pose_version = self.frame._pose_version
        return self._view


class DeviceLocalMap:
    """Tracking::mvpLocalMapPoints as device arrays: pos / normal (n x 3, GetWorldPos / GetNormal),
    min_dist / max_dist (mfMinDistance, mfMaxDistance), desc (n x 32), observed, is_bad and last_row
    (the last frame's keypoint holding the point, -1: none; the mnLastFrameSeen skip).  Owns the
    tracking fields isInFrustum writes (track_in_view, track_proj, track_depth, track_level,
    track_view_cos)."""

    def __init__(self, pos, normal, min_dist, max_dist, desc, observed, is_bad, last_row=None):
        import torch
        self.n = int(pos.shape[0])
        self.device = pos.device
        self.pos, self.normal, self.min_dist, self.max_dist = pos, normal, min_dist, max_dist
        self.desc, self.observed, self.is_bad, self.last_row = desc, observed, is_bad, last_row
        m = max(self.n, 1)
        dev = self.device
        self.track_in_view = torch.zeros(m, dtype=torch.uint8, device=dev)
        self.track_proj = torch.zeros((m, 3), dtype=torch.float32, device=dev)
        self.track_depth = torch.zeros(m, dtype=torch.float32, device=dev)
        self.track_level = torch.zeros(m, dtype=torch.int32, device=dev)
        self.track_view_cos = torch.zeros(m, dtype=torch.float32, device=dev)
        self._view = LocalPointsDeviceView(self.n, self.track_in_view.data_ptr(), is_bad.data_ptr(),
                                           observed.data_ptr(), self.track_proj.data_ptr(),
                                           self.track_view_cos.data_ptr(), self.track_depth.data_ptr(),
                                           self.track_level.data_ptr(), desc.data_ptr())

    @classmethod
    def from_host(cls, device, **arrays):
        import torch
        dt = dict(pos=np.float32, normal=np.float32, min_dist=np.float32, max_dist=np.float32, desc=np.uint8,
                  observed=np.uint8, is_bad=np.uint8, last_row=np.int32)
        t = {k: torch.from_numpy(np.ascontiguousarray(arrays[k], dt[k])).to(device) for k in dt if k in arrays}
        return cls(**t)

    def view(self) -> LocalPointsDeviceView:
        return self._view

    def chain_pointers(self) -> tuple:
        """(view address, pos, normal, min_dist, max_dist, last_row or 0) for a tracking-chain frame record
        (the arrays are fixed at construction)."""
        cp = getattr(self, "_chain_ptrs", None)
        if cp is None:
            lr = self.last_row
            cp = self._chain_ptrs = (ctypes.addressof(self._view), self.pos.data_ptr(), self.normal.data_ptr(),
                                     self.min_dist.data_ptr(), self.max_dist.data_ptr(),
                                     0 if lr is None else lr.data_ptr())
        return cp


class TrackResult:
    """Device outputs of one TrackingChain.track call (valid once the stream reaches them)."""

    def __init__(self, chain, stream):
        self.chain, self.stream = chain, stream

    def sync(self) -> dict:
        """Wait for the stream and return host copies: n1 (SearchByProjection(LastFrame) matches), m1 /
        m2 (per keypoint: the last-frame row / local map point assigned, m1 after the discard), pose1 /
        pose2 (SE3Quat vectors), edges1 / edges2 (the PoseOptimization graphs), edge_kp1 / edge_kp2,
        outlier1 / outlier2 (per edge), inliers (the PoseOptimization returns), n_kept (nmatches after
        the discard), n_map (nmatchesMap), n2 (SearchByProjection(local) matches), status (ORB_TRACK_*
        bits: the 2 th retry ran / the frame failed after the search / after PoseOptimization)."""
        c = self.chain
        self.stream.synchronize()
        fr = c.frames.cpu().numpy().view(POSE_FRAME_DTYPE).reshape(2)
        ne = [int(fr[0]["n_edges"]), int(fr[1]["n_edges"])]
        out = dict(frames=fr, n1=int(c.n_match[0]), n2=int(c.n_match[1]), m1=c.m1.cpu().numpy(),
                   m2=c.m2.cpu().numpy(), pose1=c.poses[0].cpu().numpy(), pose2=c.poses[1].cpu().numpy(),
                   inliers=c.inliers.cpu().numpy(), n_kept=int(c.n_out[0]), n_map=int(c.n_out[1]),
                   status=int(c.status[0]))
        for k in (0, 1):
            out[f"edges{k + 1}"] = c.edges[k][:ne[k]].cpu().numpy().view(POSE_EDGE_DTYPE).reshape(-1)
            out[f"edge_kp{k + 1}"] = c.edge_kp[k][:ne[k]].cpu().numpy()
            out[f"outlier{k + 1}"] = c.outlier[k][:ne[k]].cpu().numpy().astype(bool)
        return out


class TrackingChain:
    """Buffers and launch sequence for TrackWithMotionModel -> TrackLocalMap on frames of up to `cap`
    keypoints (one chain object per concurrently tracked frame).  th_motion: 7 for stereo, 15
    otherwise (src/Tracking.cc:4141-4146); th_local: SearchLocalPoints' th (1 for stereo / mono
    without IMU, 3 for RGB-D, src/Tracking.cc:4801-4823); mono: bMono of the last-frame search; gate:
    TrackWithMotionModel's retry / failure decisions on the device (False: every stage always runs)."""

    def __init__(self, cap: int, device=None, th_motion: float = 7, th_local: float = 1, mono: bool = False,
                 far_points: bool = False, th_far_points: float = 20.0, viewing_cos_limit: float = 0.5,
                 scale_factor: float = 1.2, gate: bool = True):
        import torch
        self.device = torch.device(device if device is not None else "cuda")
        self.cap = int(cap)
        self.th_motion, self.th_local, self.mono = float(th_motion), float(th_local), bool(mono)
        self.far_points, self.th_far_points = bool(far_points), float(th_far_points)
        self.viewing_cos_limit, self.scale_factor = float(viewing_cos_limit), float(scale_factor)
        self.m_motion = ORBmatcher(0.9, True)   # TrackWithMotionModel's ORBmatcher(0.9, true)
        self.m_local = ORBmatcher(0.8, True)    # SearchLocalPoints' ORBmatcher(0.8)
        d, c = self.device, self.cap
        self.m1 = torch.empty(c, dtype=torch.int32, device=d)
        self.m2 = torch.empty(c, dtype=torch.int32, device=d)
        self.n_match = torch.zeros(2, dtype=torch.int32, device=d)
        self.frames = torch.zeros(2 * POSE_FRAME_DTYPE.itemsize, dtype=torch.uint8, device=d)
        self.edges = [torch.empty((c, POSE_EDGE_DTYPE.itemsize), dtype=torch.uint8, device=d) for _ in range(2)]
        self.edge_kp = [torch.empty(c, dtype=torch.int32, device=d) for _ in range(2)]
        self.outlier = [torch.empty(c, dtype=torch.uint8, device=d) for _ in range(2)]
        self.poses = torch.zeros((2, 7), dtype=torch.float64, device=d)
        self.inliers = torch.zeros(2, dtype=torch.int32, device=d)
        self.n_out = torch.zeros(2, dtype=torch.int32, device=d)
        self.taken = torch.empty(c, dtype=torch.uint8, device=d)
        self.status = torch.zeros(1, dtype=torch.int32, device=d)
        self._h_motion, self._h_local = self.m_motion._handle(), self.m_local._handle()
        self._params = TrackingChainParams(self.th_motion, int(self.mono), self.th_local, int(self.far_points),
                                           self.th_far_points, self.viewing_cos_limit, int(bool(gate)))
        fsz = POSE_FRAME_DTYPE.itemsize
        self._bufs = TrackingChainBuffers(
            self.m1.data_ptr(), self.m2.data_ptr(), self.n_match.data_ptr(), self.frames.data_ptr(),
            self.edges[0].data_ptr(), self.edges[1].data_ptr(), self.edge_kp[0].data_ptr(),
            self.edge_kp[1].data_ptr(), self.outlier[0].data_ptr(), self.outlier[1].data_ptr(),
            self.poses.data_ptr(), self.inliers.data_ptr(), self.n_out.data_ptr(), self.taken.data_ptr(), None,
            self.status.data_ptr())
        assert self.frames.numel() == 2 * fsz
        self._scratch = torch.empty(0, dtype=torch.uint8, device=d)
        self._scratch_key = None
        self._scratch_streams = {}  # the streams that used the current scratch (its retirement waits for them)

    def track(self, cur: DeviceFrame, last: DeviceLastPoints, local: DeviceLocalMap, pose7, stream=None) -> TrackResult:
        """Enqueue the chain for `cur` on `stream` (default: torch's current stream).  pose7: the motion
        model's prediction as the SE3Quat vector PoseOptimization starts from (tx ty tz qx qy qz qw of
        the frame's float pose); cur's Tcw must be the same pose.  TrackWithMotionModel's 2 th retry and
        failure are decided on the device (the result's status)."""
        import torch
        if cur.cap > self.cap:
            raise ValueError(f"frame capacity {cur.cap} exceeds the chain's {self.cap}")
        lib = _lib.load()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        p0 = np.ascontiguousarray(pose7, np.float64).reshape(7)
        lr = local.last_row
        key = (cur.cap, last.cap, local.n)
        if key != self._scratch_key:  # one scratch for every stage of the call, grown as the sizes need
            need = int(lib.orb_tracking_chain_scratch_bytes(*key))
            if need > self._scratch.numel():
                old = self._scratch
                self._scratch = _alloc_scratch(need, old, self.device)
                # the old scratch goes back to torch's allocator once every stream that used it has
                # passed this point (record_stream), not while an earlier call's stages still read it
                for s_ in self._scratch_streams.values():
                    old.record_stream(s_)
                self._scratch_streams = {}
                self._bufs.scratch = self._scratch.data_ptr()
            self._scratch_key = key
        self._scratch_streams[st.cuda_stream] = st
        check(lib.orb_tracking_chain_device(self._h_motion, self._h_local, ctypes.byref(cur.view()),
                                            ctypes.byref(last.view()), ctypes.byref(local.view()),
                                            local.pos.data_ptr(), local.normal.data_ptr(), local.min_dist.data_ptr(),
                                            local.max_dist.data_ptr(), None if lr is None else lr.data_ptr(),
                                            ctypes.byref(cur.frustum_frame(self.scale_factor)),
                                            cur.mvInvLevelSigma2.ctypes.data, p0.ctypes.data,
                                            ctypes.byref(self._params), ctypes.byref(self._bufs),
                                            ctypes.c_void_p(st.cuda_stream)),
              "orb_tracking_chain_device")
        return TrackResult(self, st)


class TrackingChainFrame(ctypes.Structure):  # orb_tracking_chain_frame_t
    _fields_ = [("frame", ctypes.c_void_p), ("last", ctypes.c_void_p), ("local", ctypes.c_void_p),
                ("pos", ctypes.c_void_p), ("normal", ctypes.c_void_p), ("min_dist", ctypes.c_void_p),
                ("max_dist", ctypes.c_void_p), ("last_row", ctypes.c_void_p), ("frustum", ctypes.c_void_p),
                ("inv_level_sigma2", ctypes.c_void_p), ("pose7", ctypes.c_double * 7)]


# The same record as a numpy dtype: track() fills a whole batch's records column-wise (the per-frame
# ctypes constructions were half of a 512-frame call's host time)
_CHAIN_FRAME_DTYPE = np.dtype([("p", "<u8", (10,)), ("pose7", "<f8", (7,))])
assert _CHAIN_FRAME_DTYPE.itemsize == ctypes.sizeof(TrackingChainFrame)


class TrackingChainBatchBuffers(ctypes.Structure):  # orb_tracking_chain_batch_buffers_t
    _fields_ = TrackingChainBuffers._fields_


class BatchTrackResult:
    """Device outputs of one TrackingChainBatch.track call: sync() returns one TrackResult-style dict
    per frame."""

    def __init__(self, chain, stream, nb):
        self.chain, self.stream, self.nb = chain, stream, nb

    def sync(self) -> list:
        c, B = self.chain, self.nb
        self.stream.synchronize()
        # the per-graph arrays are laid out 2 x (frames of the call)
        fr = c.frames.cpu().numpy().view(POSE_FRAME_DTYPE)[:2 * B].reshape(2, B)
        m1, m2 = c.m1.cpu().numpy(), c.m2.cpu().numpy()
        nm, no, stat = c.n_match.cpu().numpy(), c.n_out.cpu().numpy(), c.status.cpu().numpy()
        poses = c.poses.cpu().numpy().reshape(-1)[:14 * B].reshape(2, B, 7)
        inl = c.inliers.cpu().numpy().reshape(-1)[:2 * B].reshape(2, B)
        edges = [c.edges[k].cpu().numpy() for k in (0, 1)]
        ekp = [c.edge_kp[k].cpu().numpy() for k in (0, 1)]
        outl = [c.outlier[k].cpu().numpy() for k in (0, 1)]
        out = []
        for b in range(B):
            d = dict(frames=fr[:, b].copy(), n1=int(nm[b, 0]), n2=int(nm[b, 1]), m1=m1[b], m2=m2[b], pose1=poses[0, b],
                     pose2=poses[1, b], inliers=inl[:, b].copy(), n_kept=int(no[b, 0]), n_map=int(no[b, 1]),
                     status=int(stat[b]))
            for k in (0, 1):
                ne = int(fr[k, b]["n_edges"])
                d[f"edges{k + 1}"] = edges[k][b, :ne].view(POSE_EDGE_DTYPE).reshape(-1)
                d[f"edge_kp{k + 1}"] = ekp[k][b, :ne]
                d[f"outlier{k + 1}"] = outl[k][b, :ne].astype(bool)
            out.append(d)
        return out


class TrackingChainBatch:
    """TrackWithMotionModel -> TrackLocalMap for up to B frames in one call
    (orb_tracking_chain_batch_device): every stage is one launch over the batch, frame b's results are
    the single chain's.  All frames of a call share `cap`; per frame its own last frame, local map and
    motion-model pose.  Parameters as TrackingChain."""

    def __init__(self, cap: int, B: int, device=None, th_motion: float = 7, th_local: float = 1, mono: bool = False,
                 far_points: bool = False, th_far_points: float = 20.0, viewing_cos_limit: float = 0.5,
                 scale_factor: float = 1.2, gate: bool = True):
        import torch
        self.device = torch.device(device if device is not None else "cuda")
        self.cap, self.B = int(cap), int(B)
        self.th_motion, self.th_local, self.mono = float(th_motion), float(th_local), bool(mono)
        self.scale_factor = float(scale_factor)
        self.m_motion = ORBmatcher(0.9, True)
        self.m_local = ORBmatcher(0.8, True)
        d, c, B = self.device, self.cap, self.B
        self.m1 = torch.empty((B, c), dtype=torch.int32, device=d)
        self.m2 = torch.empty((B, c), dtype=torch.int32, device=d)
        self.n_match = torch.zeros((B, 2), dtype=torch.int32, device=d)
        self.frames = torch.zeros(2 * B * POSE_FRAME_DTYPE.itemsize, dtype=torch.uint8, device=d)
        self.edges = [torch.empty((B, c, POSE_EDGE_DTYPE.itemsize), dtype=torch.uint8, device=d) for _ in range(2)]
        self.edge_kp = [torch.empty((B, c), dtype=torch.int32, device=d) for _ in range(2)]
        self.outlier = [torch.empty((B, c), dtype=torch.uint8, device=d) for _ in range(2)]
        self.poses = torch.zeros((2, B, 7), dtype=torch.float64, device=d)
        self.inliers = torch.zeros((2, B), dtype=torch.int32, device=d)
        self.n_out = torch.zeros((B, 2), dtype=torch.int32, device=d)
        self.taken = torch.empty((B, c), dtype=torch.uint8, device=d)
        self.status = torch.zeros(B, dtype=torch.int32, device=d)
        self._scratch = torch.empty(0, dtype=torch.uint8, device=d)
        self._h_motion, self._h_local = self.m_motion._handle(), self.m_local._handle()
        self._params = TrackingChainParams(self.th_motion, int(self.mono), self.th_local, int(far_points),
                                           float(th_far_points), float(viewing_cos_limit), int(bool(gate)))
        self._bufs = TrackingChainBatchBuffers(
            self.m1.data_ptr(), self.m2.data_ptr(), self.n_match.data_ptr(), self.frames.data_ptr(),
            self.edges[0].data_ptr(), self.edges[1].data_ptr(), self.edge_kp[0].data_ptr(),
            self.edge_kp[1].data_ptr(), self.outlier[0].data_ptr(), self.outlier[1].data_ptr(),
            self.poses.data_ptr(), self.inliers.data_ptr(), self.n_out.data_ptr(), self.taken.data_ptr(), None,
            self.status.data_ptr())

    def _records(self, items):
        """The batch's orb_tracking_chain_frame_t records (a numpy buffer of _CHAIN_FRAME_DTYPE), the
        objects they point into, and the largest last-frame capacity and local map."""
        nb = len(items)
        rows, poses, keep = [], [], []
        last_cap = n_local = 0
        sf = self.scale_factor
        seen_maps = set()
        for cur, last, local, pose7 in items:
            if cur.cap != self.cap:
                raise ValueError(f"frame capacity {cur.cap} differs from the batch's {self.cap}")
            # isInFrustum writes the local map's tracking fields: one map in two slots of a call would race
            if id(local) in seen_maps:
                raise ValueError("a DeviceLocalMap appears in two slots of one batch call (each slot needs its own)")
            seen_maps.add(id(local))
            ff = cur.frustum_frame(sf)
            lv = last.view()  # (refreshes the last frame's pose in its view)
            mp = local.chain_pointers()
            keep.append(ff)
            rows.append((ctypes.addressof(cur.view()), ctypes.addressof(lv), mp[0], mp[1], mp[2], mp[3], mp[4], mp[5],
                         ctypes.addressof(ff), cur._inv_sigma2_ptr))
            poses.append(pose7)
            if last.cap > last_cap:
                last_cap = last.cap
            if local.n > n_local:
                n_local = local.n
        arr = np.empty(nb, _CHAIN_FRAME_DTYPE)
        arr["p"] = np.array(rows, dtype=np.uint64)
        arr["pose7"] = np.asarray(poses, dtype=np.float64).reshape(nb, 7)
        return arr, keep, last_cap, n_local

    def track(self, items, stream=None) -> BatchTrackResult:
        """items: up to B tuples (cur DeviceFrame, DeviceLastPoints, DeviceLocalMap, pose7), each slot
        with its own DeviceLocalMap."""
        import torch
        nb = len(items)
        if not 0 < nb <= self.B:
            raise ValueError(f"{nb} frames for a batch of {self.B}")
        lib = _lib.load()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        arr, keep, last_cap, n_local = self._records(items)  # keep: what the records point into, alive over the call
        need = int(lib.orb_tracking_chain_batch_scratch_bytes(self.B, self.cap, last_cap, n_local))
        if need > self._scratch.numel():
            if self._scratch.numel():  # waits for the last call on the old scratch, then frees its staging
                lib.orb_tracking_chain_batch_release(ctypes.c_void_p(self._scratch.data_ptr()))
            self._scratch = _alloc_scratch(need, self._scratch, self.device)  # (the old one is free: released)
            self._bufs.scratch = self._scratch.data_ptr()
        check(lib.orb_tracking_chain_batch_device(self._h_motion, self._h_local, nb, arr.ctypes.data,
                                                  ctypes.byref(self._params), ctypes.byref(self._bufs),
                                                  ctypes.c_void_p(st.cuda_stream)),
              "orb_tracking_chain_batch_device")
        return BatchTrackResult(self, st, nb)

    def release(self) -> None:
        """Free the library's pinned staging for this batch's scratch; waits until the last call's every
        kernel has finished, so the scratch and the output tensors may be dropped afterwards."""
        if self._scratch.numel():
            _lib.load().orb_tracking_chain_batch_release(ctypes.c_void_p(self._scratch.data_ptr()))

    def __del__(self):
        try:
            self.release()
        except Exception:  # interpreter shutdown: the library may be gone
            pass

