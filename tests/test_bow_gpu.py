"""GPU parity of the DBoW2 transform (orb_bow_transform*, HIP) against the CPU oracle: BowVector
(word ids and double values) and FeatureVector bit-exact, single frame and device batch."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k,L,levelsup,weighting,scoring", [(10, 4, 2, 0, 0), (10, 3, 4, 0, 0), (6, 5, 3, 1, 1),
                                                            (8, 4, 1, 2, 0), (10, 4, 2, 3, 5), (5, 4, 2, 0, 5)])
def test_bow_transform_parity(pkg, oracle, synth, k, L, levelsup, weighting, scoring):
    voc = synth.dbow_vocabulary(k, L, seed=k * 10 + L, weighting=weighting, scoring=scoring, stop_frac=0.05)
    v = pkg.ORBVocabulary(voc)
    for n, seed in [(1000, 1), (1, 2), (4097, 3), (8192, 4)]:
        d = synth.bow_descriptors(voc, n, seed=seed)
        assert v.transform(d, levelsup) == oracle.bow_transform(voc, d, levelsup), (n, seed)


def test_bow_transform_batch_device_and_edges(pkg, oracle, synth):
    import torch
    voc = synth.dbow_vocabulary(10, 4, seed=11)
    v = pkg.ORBVocabulary(voc)
    sizes = [1000, 0, 1, 37, 1200, 5000]
    descs = [synth.bow_descriptors(voc, n, seed=100 + i) for i, n in enumerate(sizes)]
    fb = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    allv = np.concatenate(descs) if sum(sizes) else np.zeros((0, 32), np.uint8)
    bw, bv, fn, fbeg, ff, cnt = v.transform_batch_device(torch.from_numpy(allv).cuda(), torch.from_numpy(fb).cuda(), 4)
    torch.cuda.synchronize()
    bw, bv, fn, fbeg, ff, cnt = (t.cpu().numpy() for t in (bw, bv, fn, fbeg, ff, cnt))
    for f, d in enumerate(descs):
        rbow, rfv = oracle.bow_transform(voc, d, 4)
        b0 = fb[f]
        nw, nn = int(cnt[2 * f]), int(cnt[2 * f + 1])
        assert {int(bw[b0 + i]): float(bv[b0 + i]) for i in range(nw)} == rbow, f
        beg = fbeg[b0 + f:b0 + f + nn + 1]
        assert {int(fn[b0 + j]): [int(x) for x in ff[b0 + beg[j]:b0 + beg[j + 1]]] for j in range(nn)} == rfv, f
    # empty input and a frame above the 8192-feature limit
    assert v.transform(np.zeros((0, 32), np.uint8)) == ({}, {})
    with pytest.raises(pkg.OrbGpuError):
        v.transform(synth.bow_descriptors(voc, 8193, seed=9))
