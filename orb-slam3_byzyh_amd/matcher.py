"""ORBmatcher with the reference's interface (include/ORBmatcher.h), HIP-backed."""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import check
from .keyframe import DeviceKeyFrame, Frame, KeyFrame, KfDeviceView, KfView, LocalMapPoints, PairGeom

TH_HIGH = 100  # src/ORBmatcher.cc:36
TH_LOW = 50    # src/ORBmatcher.cc:37
HISTO_LENGTH = 30  # src/ORBmatcher.cc:38


class ORBmatcher:
    TH_HIGH = TH_HIGH
    TH_LOW = TH_LOW
    HISTO_LENGTH = HISTO_LENGTH

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True):
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)
        self._h = None

    def _handle(self):
        if self._h is None:
            lib = _lib.load()
            h = ctypes.c_void_p()
            check(lib.orb_matcher_create(self.mfNNratio, int(self.mbCheckOrientation), ctypes.byref(h)),
                  "orb_matcher_create")
            self._h = h
        return self._h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _lib.load().orb_matcher_destroy(h)
            except Exception:
                pass
            self._h = None

    @staticmethod
    def pair_geometry(pKF1: KeyFrame, pKF2: KeyFrame) -> PairGeom:
        """R12, t12 of T12 = T1w * Tw2 and the epipole of KF1's centre in KF2 (src/ORBmatcher.cc:1063-1090)."""
        g = PairGeom()
        check(_lib.load().orb_kf_pair_geometry(pKF1.Tcw.ctypes.data, pKF2.Tcw.ctypes.data, pKF2.fx, pKF2.fy,
                                               pKF2.cx, pKF2.cy, ctypes.byref(g)), "orb_kf_pair_geometry")
        return g

    def SearchForTriangulation(self, pKF1: KeyFrame, pKF2: KeyFrame, bOnlyStereo: bool, bCoarse: bool = False):
        """src/ORBmatcher.cc:1046-1324.  Returns (nmatches, vMatchedPairs as a list of (idx1, idx2))."""
        (n, m12), = self.SearchForTriangulationMany(pKF1, [pKF2], bOnlyStereo, bCoarse)
        pairs = [(int(i), int(m12[i])) for i in np.flatnonzero(m12 >= 0)]
        return n, pairs

    def SearchForTriangulationMany(self, pKF1: KeyFrame, neighbours, bOnlyStereo: bool, bCoarse: bool = False,
                                   geoms=None):
        """SearchForTriangulation of pKF1 against every keyframe in `neighbours` in one device launch
        (the loop of LocalMapping::CreateNewMapPoints).  Returns [(nmatches, vMatches12 int32[N1])]."""
        neighbours = list(neighbours)
        p = len(neighbours)
        if p == 0:
            return []
        views = (KfView * p)(*[k.view() for k in neighbours])
        if geoms is None:
            geoms = [self.pair_geometry(pKF1, k) for k in neighbours]
        garr = (PairGeom * p)(*geoms)
        m12 = np.full((p, max(pKF1.N, 1)), -1, np.int32)
        cnt = np.zeros(p, np.int32)
        check(_lib.load().orb_search_for_triangulation(self._handle(), ctypes.byref(pKF1.view()), views, garr, p,
                                                       int(bOnlyStereo), int(bCoarse), m12.ctypes.data,
                                                       cnt.ctypes.data), "orb_search_for_triangulation")
        return [(int(cnt[i]), m12[i, :pKF1.N]) for i in range(p)]

    def SearchForTriangulationDevice(self, pKF1: DeviceKeyFrame, neighbours, bOnlyStereo: bool, bCoarse: bool = False,
                                     stream=None, out=None):
        """SearchForTriangulation of a device-resident keyframe against device-resident neighbours
        (orb_search_for_triangulation_device): no host hop for features, stereo depths or FeatureVectors.
        Returns (matches12 [P, cap1] int32, counts [P] int32) CUDA tensors, asynchronous on `stream`."""
        return self.SearchForTriangulationDeviceBatch([(pKF1, list(neighbours))], bOnlyStereo, bCoarse, stream, out)

    def SearchForTriangulationDeviceBatch(self, groups, bOnlyStereo: bool, bCoarse: bool = False, stream=None, out=None,
                                          prepared=None):
        """Several new keyframes, each with its neighbours, in one launch: groups = [(kf1, [kf2, ...]), ...].
        Returns (matches12 [P, C] int32, counts [P] int32), pairs in group order, C = max cap of the kf1s.
        `prepared` (from prepare_device_batch) reuses the ctypes arrays of an identical earlier call."""
        import torch
        if prepared is None:
            prepared = self.prepare_device_batch(groups)
        kf1v, n1, kf2v, k1, geoms, n_pairs, C, dev = prepared
        if out is None:
            out = (torch.empty((max(n_pairs, 1), C), dtype=torch.int32, device=dev),
                   torch.empty(max(n_pairs, 1), dtype=torch.int32, device=dev))
        if n_pairs == 0:
            return out
        st = stream if stream is not None else torch.cuda.current_stream(dev)
        check(_lib.load().orb_search_for_triangulation_device(self._handle(), kf1v, n1, kf2v, k1, geoms, n_pairs,
                                                              int(bOnlyStereo), int(bCoarse), out[0].data_ptr(),
                                                              out[1].data_ptr(), ctypes.c_void_p(st.cuda_stream)),
              "orb_search_for_triangulation_device")
        return out

    def prepare_device_batch(self, groups):
        """The ctypes arguments of SearchForTriangulationDeviceBatch for `groups` (views, pair table, geometry)."""
        groups = [(k1, list(nb)) for k1, nb in groups]
        n1 = len(groups)
        kf1v = (KfDeviceView * max(n1, 1))(*[g[0].view() for g in groups])
        pairs = [(i, k2) for i, (_, nb) in enumerate(groups) for k2 in nb]
        n_pairs = len(pairs)
        kf2v = (KfDeviceView * max(n_pairs, 1))(*[k2.view() for _, k2 in pairs])
        k1 = (ctypes.c_int32 * max(n_pairs, 1))(*[i for i, _ in pairs])
        geoms = (PairGeom * max(n_pairs, 1))(*[self.pair_geometry(groups[i][0], k2) for i, k2 in pairs])
        C = max(g[0].cap for g in groups)
        return kf1v, n1, kf2v, k1, geoms, n_pairs, C, groups[0][0]._keep[0].device

    @staticmethod
    def DescriptorDistance(a, b) -> int:
        """Hamming distance of two 32-byte descriptors (src/ORBmatcher.cc:2384-2404)."""
        a = np.ascontiguousarray(a, dtype=np.uint8).reshape(32)
        b = np.ascontiguousarray(b, dtype=np.uint8).reshape(32)
        return check(_lib.load().orb_descriptor_distance(a.ctypes.data, b.ctypes.data), "orb_descriptor_distance")

    @staticmethod
    def knn2_device(query, train, stream=None):
        """Best/second-best Hamming match of every query row among train rows (torch uint8 [n, 32] on GPU)."""
        import torch
        q = query.contiguous()
        t = train.contiguous()
        n = q.shape[0]
        idx = torch.empty(n, dtype=torch.int32, device=q.device)
        d1 = torch.empty(n, dtype=torch.int32, device=q.device)
        d2 = torch.empty(n, dtype=torch.int32, device=q.device)
        st = stream if stream is not None else torch.cuda.current_stream(q.device)
        check(_lib.load().orb_hamming_knn2_device(q.data_ptr(), n, t.data_ptr(), t.shape[0], idx.data_ptr(),
                                                  d1.data_ptr(), d2.data_ptr(), ctypes.c_void_p(st.cuda_stream)),
              "orb_hamming_knn2_device")
        return idx, d1, d2

    @staticmethod
    def knn2_frames_device(desc, counts, pairs, stream=None, out=None):
        """Cross-frame knn2 over a batch of device feature blocks (orb_hamming_knn2_frames_device):
        desc uint8 [F, cap, 32], counts int32 [F, >= 1] (column 0 = descriptors per frame), pairs int32
        [P, 2] (query frame, train frame) on the device.  Returns (idx, best, second), int32 [P, cap]."""
        import torch
        d = desc.contiguous()
        c = counts.contiguous()
        pr = pairs.to(device=d.device, dtype=torch.int32).contiguous()
        n_pairs, cap = pr.shape[0], d.shape[1]
        if out is None:
            out = tuple(torch.empty((n_pairs, cap), dtype=torch.int32, device=d.device) for _ in range(3))
        st = stream if stream is not None else torch.cuda.current_stream(d.device)
        check(_lib.load().orb_hamming_knn2_frames_device(d.data_ptr(), c.data_ptr(), c.shape[1], cap, pr.data_ptr(),
                                                         n_pairs, out[0].data_ptr(), out[1].data_ptr(),
                                                         out[2].data_ptr(), ctypes.c_void_p(st.cuda_stream)),
              "orb_hamming_knn2_frames_device")
        return out

    def ComputeDistinctiveDescriptors(self, desc, offsets):
        """MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:438-529) for a batch of map points:
        point p's observation descriptors are rows offsets[p]..offsets[p+1] of desc (uint8 [n, 32]).
        Returns (best int32[P], mDescriptor uint8[P, 32]); best -1 / a zero row for a point without
        descriptors (the reference leaves its mDescriptor unchanged)."""
        desc = np.ascontiguousarray(desc, dtype=np.uint8).reshape(-1, 32)
        offsets = np.ascontiguousarray(offsets, dtype=np.int32)
        n = len(offsets) - 1
        best = np.full(max(n, 1), -1, np.int32)
        out = np.zeros((max(n, 1), 32), np.uint8)
        check(_lib.load().orb_compute_distinctive_descriptors(self._handle(), desc.ctypes.data, offsets.ctypes.data, n,
                                                              best.ctypes.data, out.ctypes.data),
              "orb_compute_distinctive_descriptors")
        return best[:n], out[:n]

    @staticmethod
    def compute_distinctive_descriptors_device(desc, offsets, out=None, stream=None):
        """The same on device tensors (desc uint8 [n, 32], offsets int32 [P + 1]); async on `stream`.
        Returns (best int32 [P], out uint8 [P, 32])."""
        import torch
        d = desc.contiguous()
        o = offsets.contiguous()
        n = o.shape[0] - 1
        best = torch.empty(max(n, 1), dtype=torch.int32, device=d.device)
        if out is None:
            out = torch.zeros((max(n, 1), 32), dtype=torch.uint8, device=d.device)
        st = stream if stream is not None else torch.cuda.current_stream(d.device)
        check(_lib.load().orb_compute_distinctive_descriptors_device(d.data_ptr(), o.data_ptr(), n, best.data_ptr(),
                                                                     out.data_ptr(), ctypes.c_void_p(st.cuda_stream)),
              "orb_compute_distinctive_descriptors_device")
        return best[:n], out[:n]

    def SearchByProjectionFrame(self, CurrentFrame: Frame, LastFrame: Frame, th: float, bMono: bool):
        """SearchByProjection(Frame &CurrentFrame, const Frame &LastFrame, th, bMono)
        (src/ORBmatcher.cc:1951-2185).  Returns (nmatches, match) with match[i2] = the LastFrame index
        whose map point CurrentFrame.mvpMapPoints[i2] receives (-1: none)."""
        m = np.full(max(CurrentFrame.N, 1), -1, np.int32)
        n = ctypes.c_int32()
        check(_lib.load().orb_search_by_projection_frame(self._handle(), ctypes.byref(CurrentFrame.view()),
                                                         ctypes.byref(LastFrame.last_points()), float(th),
                                                         int(bMono), m.ctypes.data, ctypes.byref(n)),
              "orb_search_by_projection_frame")
        return n.value, m[:CurrentFrame.N]

    def SearchByProjection(self, F: Frame, vpMapPoints: LocalMapPoints, th: float = 3, bFarPoints: bool = False,
                           thFarPoints: float = 50.0, frame_taken=None):
        """SearchByProjection(Frame &F, const vector<MapPoint*> &vpMapPoints, th, bFarPoints, thFarPoints)
        (src/ORBmatcher.cc:46-240).  frame_taken[i]: keypoint i already holds a map point with
        observations.  Returns (nmatches, match) with match[i] = index of the map point assigned."""
        m = np.full(max(F.N, 1), -1, np.int32)
        n = ctypes.c_int32()
        tk = None if frame_taken is None else np.ascontiguousarray(frame_taken, dtype=np.uint8)
        check(_lib.load().orb_search_by_projection_local(self._handle(), ctypes.byref(F.view()),
                                                         None if tk is None else tk.ctypes.data,
                                                         ctypes.byref(vpMapPoints.view()), float(th), int(bFarPoints),
                                                         float(thFarPoints), m.ctypes.data, ctypes.byref(n)),
              "orb_search_by_projection_local")
        return n.value, m[:F.N]
