"""ORBVocabulary (DBoW2 TemplatedVocabulary<FORB::TDescriptor, FORB>) transform on the MI355X.

Mirrors what ORB-SLAM3 uses of the vocabulary on the BoW path: ``transform(descriptors, levelsup)``
giving the BowVector (``{WordId: WordValue}``) and the FeatureVector (``{NodeId: [feature indices]}``)
that KeyFrame::ComputeBoW / Frame::ComputeBoW store (src/KeyFrame.cc:109, src/Frame.cc:1010) and that
SearchForTriangulation / SearchByBoW walk.  The vocabulary is given as flat arrays (node children
CSR, node descriptors, leaf word ids and weights), e.g. from ``synth.dbow_vocabulary``; ORBvoc.txt is
not shipped with the reference.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import check


class ORBVocabulary:
    def __init__(self, voc: dict):
        lib = _lib.load()
        _lib.require_device()
        self._lib = lib
        self.k, self.L = int(voc["k"]), int(voc["L"])
        view, self._keep = _lib.vocabulary_view(voc)
        h = ctypes.c_void_p()
        check(lib.orb_vocabulary_create(ctypes.byref(view), ctypes.byref(h)), "orb_vocabulary_create")
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                self._lib.orb_vocabulary_destroy(h)
            except Exception:
                pass
            self._h = None

    def transform(self, descriptors, levelsup: int = 4):
        """TemplatedVocabulary::transform(features, BowVector&, FeatureVector&, levelsup).
        Returns (bow: dict word -> value, feat_vec: dict node -> list of feature indices)."""
        d = np.ascontiguousarray(descriptors if descriptors is not None else np.zeros((0, 32), np.uint8), np.uint8)
        d = d.reshape(-1, 32)
        n = len(d)
        m = max(n, 1)
        bw, bv = np.zeros(m, np.int32), np.zeros(m, np.float64)
        fn, fb, ff = np.zeros(m, np.int32), np.zeros(m + 1, np.int32), np.zeros(m, np.int32)
        nw, nn = ctypes.c_int32(), ctypes.c_int32()
        check(self._lib.orb_bow_transform(self._h, d.ctypes.data, n, int(levelsup), bw.ctypes.data, bv.ctypes.data,
                                          ctypes.byref(nw), fn.ctypes.data, fb.ctypes.data, ff.ctypes.data,
                                          ctypes.byref(nn)), "orb_bow_transform")
        bow = {int(bw[i]): float(bv[i]) for i in range(nw.value)}
        fv = {int(fn[j]): [int(x) for x in ff[fb[j]:fb[j + 1]]] for j in range(nn.value)}
        return bow, fv

    def transform_batch_device(self, desc, frame_begin, levelsup: int = 4, stream=None):
        """Device batch: desc [n_total, 32] uint8 and frame_begin [n_frames + 1] int32 CUDA tensors.
        Returns the output tensors (bow_word, bow_value, fv_node, fv_begin, fv_feat, counts)."""
        import torch
        n_total, nf = desc.shape[0], frame_begin.shape[0] - 1
        dev = desc.device
        m = max(n_total, 1)
        out = (torch.empty(m, dtype=torch.int32, device=dev), torch.empty(m, dtype=torch.float64, device=dev),
               torch.empty(m, dtype=torch.int32, device=dev), torch.empty(m + nf, dtype=torch.int32, device=dev),
               torch.empty(m, dtype=torch.int32, device=dev), torch.empty(2 * max(nf, 1), dtype=torch.int32, device=dev))
        st = stream if stream is not None else torch.cuda.current_stream(dev)
        check(self._lib.orb_bow_transform_batch_device(self._h, desc.data_ptr(), frame_begin.data_ptr(), nf, n_total,
                                                       int(levelsup), *[t.data_ptr() for t in out],
                                                       ctypes.c_void_p(st.cuda_stream)), "orb_bow_transform_batch_device")
        return out

    def transform_frames_device(self, desc, counts, levelsup: int = 4, stream=None, out=None):
        """Device batch on the extractor's layout: desc [B, cap, 32] uint8 and counts [B, 2] int32 CUDA
        tensors as ORBextractor.extract_batch_device returns them (no compaction, no host hop).
        Returns (bow_word [B, cap], bow_value [B, cap], fv_node [B, cap], fv_begin [B, cap + 1],
        fv_feat [B, cap], counts [B, 2] = (n_words, n_nodes))."""
        import torch
        b, cap = desc.shape[0], desc.shape[1]
        dev = desc.device
        if out is None:
            out = (torch.empty((b, cap), dtype=torch.int32, device=dev),
                   torch.empty((b, cap), dtype=torch.float64, device=dev),
                   torch.empty((b, cap), dtype=torch.int32, device=dev),
                   torch.empty((b, cap + 1), dtype=torch.int32, device=dev),
                   torch.empty((b, cap), dtype=torch.int32, device=dev), torch.empty((b, 2), dtype=torch.int32, device=dev))
        st = stream if stream is not None else torch.cuda.current_stream(dev)
        check(self._lib.orb_bow_transform_frames_device(self._h, desc.data_ptr(), counts.data_ptr(), b, cap, int(levelsup),
                                                        *[t.data_ptr() for t in out], ctypes.c_void_p(st.cuda_stream)),
              "orb_bow_transform_frames_device")
        return out
