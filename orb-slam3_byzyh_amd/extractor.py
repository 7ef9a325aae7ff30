"""ORBextractor with the reference's interface, running on the MI355X HIP path.

Mirrors ORB_SLAM3::ORBextractor (reference include/ORBextractor.h:46-109, src/ORBextractor.cc):
construction from (nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST), the call operator with
(image, mask, vLappingArea) that returns the keypoints, their 32-byte descriptors and monoIndex,
the scale getters and the public image pyramid.  Python has no output parameters, so
``__call__`` returns ``(keypoints, descriptors, mono_index)``; an empty image returns
``([], None, -1)`` like the reference's ``return -1`` (src/ORBextractor.cc:1561-1562).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import KEYPOINT_DTYPE, OrbParams, check


class ORBextractor:
    HARRIS_SCORE = 0
    FAST_SCORE = 1

    def __init__(self, nfeatures: int, scaleFactor: float, nlevels: int, iniThFAST: int, minThFAST: int,
                 max_width: int = 1280, max_height: int = 720, max_batch: int = 1):
        lib = _lib.load()
        _lib.require_device()
        self._lib = lib
        self.nfeatures = int(nfeatures)
        self.scaleFactor = float(np.float32(scaleFactor))  # float argument stored in a double member
        self.nlevels = int(nlevels)
        self.iniThFAST = int(iniThFAST)
        self.minThFAST = int(minThFAST)
        self.max_width, self.max_height, self.max_batch = int(max_width), int(max_height), int(max_batch)
        self._params = OrbParams(self.nfeatures, self.scaleFactor, self.nlevels, self.iniThFAST, self.minThFAST)
        h = ctypes.c_void_p()
        check(lib.orb_extractor_create(ctypes.byref(self._params), self.max_width, self.max_height,
                                       self.max_batch, ctypes.byref(h)), "orb_extractor_create")
        self._h = h
        n = self.nlevels
        bufs = [(ctypes.c_float * n)() for _ in range(4)]
        per = (ctypes.c_int32 * n)()
        check(lib.orb_extractor_scales(h, *bufs, per), "orb_extractor_scales")
        self.mvScaleFactor = [float(v) for v in bufs[0]]
        self.mvInvScaleFactor = [float(v) for v in bufs[1]]
        self.mvLevelSigma2 = [float(v) for v in bufs[2]]
        self.mvInvLevelSigma2 = [float(v) for v in bufs[3]]
        self.mnFeaturesPerLevel = [int(v) for v in per]
        self._last_frames = 0

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                self._lib.orb_extractor_destroy(h)
            except Exception:
                pass
            self._h = None

    # ---- getters, include/ORBextractor.h:61-81
    def GetLevels(self) -> int:
        return self.nlevels

    def GetScaleFactor(self) -> float:
        return self.scaleFactor

    def GetScaleFactors(self) -> list[float]:
        return list(self.mvScaleFactor)

    def GetInverseScaleFactors(self) -> list[float]:
        return list(self.mvInvScaleFactor)

    def GetScaleSigmaSquares(self) -> list[float]:
        return list(self.mvLevelSigma2)

    def GetInverseScaleSigmaSquares(self) -> list[float]:
        return list(self.mvInvLevelSigma2)

    # ---- ORBextractor::operator(), src/ORBextractor.cc:1557-1682
    def __call__(self, image, mask=None, vLappingArea=(0, 0)):
        """Extract ORB keypoints + descriptors from one 8-bit gray image (mask ignored, as upstream)."""
        del mask
        if image is None or getattr(image, "size", 0) == 0:
            return np.zeros(0, KEYPOINT_DTYPE), None, -1
        img = np.ascontiguousarray(image)
        if img.dtype != np.uint8 or img.ndim != 2:
            raise ValueError("ORBextractor expects a single-channel 8-bit image (CV_8UC1)")
        h, w = img.shape
        cap = 2 * self.nfeatures + 64 * self.nlevels
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = ctypes.c_int()
        rc = self._lib.orb_extract(self._h, img.ctypes.data, w, h, w, int(vLappingArea[0]), int(vLappingArea[1]),
                                   kps.ctypes.data, desc.ctypes.data, cap, ctypes.byref(n))
        if rc == _lib.ORB_ERR_CAPACITY:  # retry once with the reported size
            cap = n.value
            kps = np.zeros(cap, KEYPOINT_DTYPE)
            desc = np.zeros((cap, 32), np.uint8)
            rc = self._lib.orb_extract(self._h, img.ctypes.data, w, h, w, int(vLappingArea[0]),
                                       int(vLappingArea[1]), kps.ctypes.data, desc.ctypes.data, cap, ctypes.byref(n))
        check(rc, "orb_extract")
        self._last_frames = 1
        k = n.value
        return kps[:k].copy(), (desc[:k].copy() if k > 0 else None), rc

    # ---- batched device-resident form (throughput path)
    def extract_batch_device(self, images, vLappingArea=(0, 0), cap: int | None = None, out=None, stream=None):
        """images: torch.uint8 tensor [B, H, W] on the GPU.  Returns (kps int8-view tensor, desc, counts).

        kps is a [B, cap, 7] float32/int32-punned tensor in cv::KeyPoint layout, desc [B, cap, 32] uint8,
        counts [B, 2] int32 = (number of keypoints, monoIndex).  Asynchronous on `stream`
        (default: torch's current stream).
        """
        import torch
        if images.dtype != torch.uint8 or images.dim() != 3 or not images.is_cuda:
            raise ValueError("images must be a CUDA uint8 tensor [B, H, W]")
        images = images.contiguous()
        b, h, w = images.shape
        cap = cap or (self.nfeatures + 16 * self.nlevels)
        if out is None:
            kps = torch.empty((b, cap, 7), dtype=torch.float32, device=images.device)
            desc = torch.empty((b, cap, 32), dtype=torch.uint8, device=images.device)
            counts = torch.empty((b, 2), dtype=torch.int32, device=images.device)
        else:
            kps, desc, counts = out
        st = stream if stream is not None else torch.cuda.current_stream(images.device)
        check(self._lib.orb_extract_batch_device(
            self._h, images.data_ptr(), b, w, h, w, h * w, int(vLappingArea[0]), int(vLappingArea[1]),
            kps.data_ptr(), desc.data_ptr(), cap, counts.data_ptr(), ctypes.c_void_p(st.cuda_stream)),
            "orb_extract_batch_device")
        self._last_frames = b
        return kps, desc, counts

    def set_overlap(self, on: bool) -> None:
        """Batch scheduling on the device path (orb_extractor_set_overlap): True (default) runs the
        early levels on the handle's side streams (one batch alone finishes sooner); False runs each
        batch as one chain on the caller's stream (more throughput with several handles in flight)."""
        check(self._lib.orb_extractor_set_overlap(self._h, 1 if on else 0), "orb_extractor_set_overlap")

    # ---- per-stage timing (HIP events on the launch stream)
    def profile(self, enable: bool | str = True) -> None:
        """Record HIP events at stage boundaries: True = every stage, "pyramid" = only around the
        pyramid stage (2 events per call, for timed regions), "pyramid_launches" = around every
        pyramid level launch (kernel durations), False = off."""
        mode = 2 if enable == "pyramid" else 3 if enable == "pyramid_launches" else (1 if enable else 0)
        check(self._lib.orb_extractor_profile(self._h, mode), "orb_extractor_profile")

    def stage_ms(self):
        """Summed ms per stage since profile(True), the number of launches and frames recorded."""
        ms = (ctypes.c_float * len(_lib.STAGES))()
        n = ctypes.c_int()
        fr = ctypes.c_longlong()
        check(self._lib.orb_extractor_stage_ms(self._h, ms, ctypes.byref(n), ctypes.byref(fr)), "orb_extractor_stage_ms")
        return dict(zip(_lib.STAGES, (float(v) for v in ms))), n.value, fr.value

    def pyramid_launch_ms(self):
        """profile("pyramid_launches"): summed ms of the recorded k_pyramid_level launches (an event
        pair around each launch) and their number."""
        ms = ctypes.c_float()
        n = ctypes.c_int()
        check(self._lib.orb_extractor_pyramid_launch_ms(self._h, ctypes.byref(ms), ctypes.byref(n)),
              "orb_extractor_pyramid_launch_ms")
        return float(ms.value), n.value

    LAUNCH_KERNELS = ("k_pyramid_level", "k_fast_cells", "k_quadtree_kp", "k_describe")

    def launch_durations(self, kernel: str):
        """profile("pyramid_launches"): every recorded launch of one stage kernel, in launch order, in
        ms (each from the dispatch's own event pair)."""
        k = self.LAUNCH_KERNELS.index(kernel)
        n = ctypes.c_int()
        check(self._lib.orb_extractor_launch_durations(self._h, k, None, 0, ctypes.byref(n)),
              "orb_extractor_launch_durations")
        buf = (ctypes.c_float * max(1, n.value))()
        check(self._lib.orb_extractor_launch_durations(self._h, k, buf, n.value, ctypes.byref(n)),
              "orb_extractor_launch_durations")
        return [float(buf[i]) for i in range(n.value)]

    # ---- public pyramid, include/ORBextractor.h:83
    def level_padded(self, level: int, frame: int = 0) -> np.ndarray:
        """Padded plane ((h+38) x (w+38)) of level `level` of frame `frame` of the last call.  Only the
        view and its 3-px REFLECT_101 border ([16:-16, 16:-16]) are written by the extractor."""
        w, h, pitch = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(self._lib.orb_extractor_level(self._h, frame, level, None, ctypes.byref(w), ctypes.byref(h),
                                            ctypes.byref(pitch)), "orb_extractor_level")
        out = np.zeros((h.value + 38, w.value + 38), np.uint8)
        check(self._lib.orb_extractor_level_download(self._h, frame, level, out.ctypes.data),
              "orb_extractor_level_download")
        return out

    @property
    def mvImagePyramid(self) -> list[np.ndarray]:
        """Level images of the last extracted frame (views into padded planes, border readable)."""
        out = []
        for l in range(self.nlevels):
            p = self.level_padded(l)
            out.append(p[19:-19, 19:-19])
        return out


def keypoints_to_structured(kps_tensor, count: int) -> np.ndarray:
    """Convert one frame's [cap, 7] float32 keypoint rows from extract_batch_device to KEYPOINT_DTYPE."""
    arr = kps_tensor[:count].contiguous().cpu().numpy()
    return arr.view(KEYPOINT_DTYPE).reshape(-1)


def undistort_keypoints_device(extracted, K, dist, out=None, stream=None):
    """Frame::UndistortKeyPoints (src/Frame.cc:1003-1051) on ORBextractor.extract_batch_device's outputs:
    returns mvKeysUn as a [B, cap, 7] tensor (keypoints past each frame's count are not written).
    K = (fx, fy, cx, cy); dist = mDistCoef, 4 or 5 floats (k1, k2, p1, p2[, k3])."""
    import torch
    kps, _, counts = extracted
    b, cap = kps.shape[0], kps.shape[1]
    out = torch.empty_like(kps) if out is None else out
    Kf = np.ascontiguousarray(K, np.float32)
    d = np.ascontiguousarray(dist, np.float32)
    st = stream if stream is not None else torch.cuda.current_stream(kps.device)
    check(_lib.load().orb_undistort_keypoints_device(kps.data_ptr(), counts.data_ptr(), b, cap, Kf.ctypes.data,
                                                     d.ctypes.data, len(d), out.data_ptr(),
                                                     ctypes.c_void_p(st.cuda_stream)),
          "orb_undistort_keypoints_device")
    return out
