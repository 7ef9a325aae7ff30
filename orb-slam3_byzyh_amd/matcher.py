"""ORBmatcher with the reference's interface (include/ORBmatcher.h), HIP-backed."""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import check

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
