"""Frame::ComputeStereoMatches on the MI355X HIP path (reference src/Frame.cc:1102-1358).

The reference method reads the Frame's left/right keypoints and descriptors, the two extractors'
``mvImagePyramid`` and the rig's ``mbf`` / ``mb``, and fills ``mvuRight`` / ``mvDepth`` (-1 = no
stereo match).  Here the pyramids are the device pyramids the two ``ORBextractor`` handles built in
their last call, so the match runs where the images already are.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import KEYPOINT_DTYPE, check


def compute_stereo_matches(left, right, keys_left, desc_left, keys_right, desc_right, mbf: float, mb: float):
    """Single stereo frame (after ``left(imL)`` / ``right(imR)``): returns (mvuRight, mvDepth, kept)."""
    lib = _lib.load()
    kl = np.ascontiguousarray(keys_left, KEYPOINT_DTYPE)
    kr = np.ascontiguousarray(keys_right, KEYPOINT_DTYPE)
    dl = np.ascontiguousarray(desc_left if desc_left is not None else np.zeros((0, 32), np.uint8), np.uint8)
    dr = np.ascontiguousarray(desc_right if desc_right is not None else np.zeros((0, 32), np.uint8), np.uint8)
    ur = np.full(len(kl), -1.0, np.float32)
    dp = np.full(len(kl), -1.0, np.float32)
    kept = check(lib.orb_compute_stereo_matches(left._h, right._h, kl.ctypes.data, len(kl), dl.ctypes.data,
                                                kr.ctypes.data, len(kr), dr.ctypes.data, float(mbf), float(mb),
                                                ur.ctypes.data, dp.ctypes.data), "orb_compute_stereo_matches")
    return ur, dp, kept


def compute_stereo_matches_batch_device(left, right, out_left, out_right, mbf: float, mb: float, stream=None, out=None):
    """Batch form on the outputs of ``extract_batch_device`` of both extractors (frames 0..B-1).

    Returns (u_right [B, cap_l] float32, depth [B, cap_l] float32, kept [B] int32) CUDA tensors;
    asynchronous on `stream` (default: torch's current stream)."""
    import torch
    kps_l, desc_l, counts_l = out_left
    kps_r, desc_r, counts_r = out_right
    b, cap_l = kps_l.shape[0], kps_l.shape[1]
    cap_r = kps_r.shape[1]
    if out is None:
        out = (torch.empty((b, cap_l), dtype=torch.float32, device=kps_l.device),
               torch.empty((b, cap_l), dtype=torch.float32, device=kps_l.device),
               torch.empty((b,), dtype=torch.int32, device=kps_l.device))
    u, d, kept = out
    st = stream if stream is not None else torch.cuda.current_stream(kps_l.device)
    check(_lib.load().orb_compute_stereo_matches_batch_device(
        left._h, right._h, b, kps_l.data_ptr(), counts_l.data_ptr(), desc_l.data_ptr(), cap_l, kps_r.data_ptr(),
        counts_r.data_ptr(), desc_r.data_ptr(), cap_r, float(mbf), float(mb), u.data_ptr(), d.data_ptr(),
        kept.data_ptr(), ctypes.c_void_p(st.cuda_stream)), "orb_compute_stereo_matches_batch_device")
    return u, d, kept
