"""GPU parity of ORBmatcher::SearchForTriangulation (k_tri_match / k_tri_finish) against the oracle.

Bar: bit-exact vMatches12 and match counts for every flag combination of the reference
(bOnlyStereo, bCoarse, mbCheckOrientation), batched over several neighbour keyframes, and the
reference's edge cases (no shared nodes, empty keyframes, all features already mapped).
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FLAGS = [(0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 0, 1), (1, 1, 1)]


@pytest.fixture(scope="module")
def scene(pkg, synth):
    return [pkg.KeyFrame(**k) for k in synth.keyframe_scene(n_kf=6, n_points=1500, seed=201)]


@pytest.mark.parametrize("only_stereo,coarse,check_ori", FLAGS)
def test_search_for_triangulation_parity(pkg, oracle, scene, only_stereo, coarse, check_ori):
    k1, nbrs = scene[0], scene[1:]
    matcher = pkg.ORBmatcher(0.6, bool(check_ori))
    got = matcher.SearchForTriangulationMany(k1, nbrs, only_stereo, coarse)
    total = 0
    for k2, (n, m) in zip(nbrs, got):
        g = matcher.pair_geometry(k1, k2)
        rn, rm = oracle.search_for_triangulation(k1, k2, g, only_stereo, coarse, check_ori)
        assert n == rn, f"count {n} vs oracle {rn}"
        assert np.array_equal(m, rm), f"{int((m != rm).sum())} differing matches"
        total += n
    assert total > 0


def test_single_pair_api(pkg, oracle, scene):
    k1, k2 = scene[0], scene[1]
    matcher = pkg.ORBmatcher(0.6, False)
    n, pairs = matcher.SearchForTriangulation(k1, k2, False, False)
    rn, rm = oracle.search_for_triangulation(k1, k2, matcher.pair_geometry(k1, k2), False, False, False)
    assert n == rn == len(pairs)
    assert pairs == [(int(i), int(rm[i])) for i in np.flatnonzero(rm >= 0)]
    assert all(a < b for (a, _), (b, _) in zip(pairs, pairs[1:]))  # increasing idx1, as vMatchedPairs


def _variant(pkg, k, **over):
    d = dict(keys_un=k.mvKeysUn, descriptors=k.mDescriptors, Tcw=k.Tcw, camera=(k.fx, k.fy, k.cx, k.cy),
             scale_factors=k.mvScaleFactors, level_sigma2=k.mvLevelSigma2, u_right=k.mvuRight,
             has_mappoint=k.has_mappoint, feat_vec=k.mFeatVec)
    d.update(over)
    return pkg.KeyFrame(**d)


def test_edge_cases(pkg, oracle, scene):
    k1, k2 = scene[0], scene[1]
    matcher = pkg.ORBmatcher(0.6, True)
    # no shared node ids
    shifted = _variant(pkg, k2, feat_vec={node + 1000: idx for node, idx in k2.mFeatVec.items()})
    # every KF1 feature already has a MapPoint
    mapped = _variant(pkg, k1, has_mappoint=np.ones(k1.N, np.uint8))
    # monocular keyframes (no mvuRight): the epipole test applies to all pairs
    mono1, mono2 = _variant(pkg, k1, u_right=None), _variant(pkg, k2, u_right=None)
    # empty neighbour
    empty = _variant(pkg, k2, keys_un=k2.mvKeysUn[:0], descriptors=k2.mDescriptors[:0], u_right=None,
                     has_mappoint=None, feat_vec={})
    for a, b, exp_zero in [(k1, shifted, True), (mapped, k2, True), (mono1, mono2, False), (k1, empty, True)]:
        (n, m), = matcher.SearchForTriangulationMany(a, [b], False, False)
        rn, rm = oracle.search_for_triangulation(a, b, matcher.pair_geometry(a, b), False, False, True)
        assert n == rn and np.array_equal(m, rm)
        assert (n == 0) == exp_zero


def test_invalid_views_rejected(pkg, scene):
    k1, k2 = scene[0], scene[1]
    matcher = pkg.ORBmatcher(0.6, False)
    fv = k1.mFeatVec
    first = next(iter(fv))
    dup = dict(fv)
    dup[first] = list(fv[first]) + [fv[first][0]]  # a feature listed twice in KF1's FeatureVector
    with pytest.raises(pkg.OrbGpuError):
        matcher.SearchForTriangulationMany(_variant(pkg, k1, feat_vec=dup), [k2], False, False)
    bad = k2.mvKeysUn.copy()
    bad["octave"][0] = 12  # beyond nlevels
    with pytest.raises(pkg.OrbGpuError):
        matcher.SearchForTriangulationMany(k1, [_variant(pkg, k2, keys_un=bad)], False, False)


def test_distinctive_large_points_grid_stride(pkg, oracle):
    """The large-point kernel walks the points with a bounded grid (512 blocks): points of more than 64
    rows past index 512 and 1024 are still found, on both entries; a point of 65536 rows is rejected
    by the host entry (its u16 histogram's range)."""
    import torch
    rng = np.random.default_rng(77)
    sizes = list(rng.integers(0, 30, 1200))
    for p, n in ((3, 90), (600, 150), (1030, 70), (1199, 65)):
        sizes[p] = n
    desc = rng.integers(0, 256, (int(sum(sizes)), 32), dtype=np.uint8)
    offsets = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    ref = oracle.compute_distinctive_descriptors(desc, offsets)
    m = pkg.ORBmatcher(0.6, False)
    best, out = m.ComputeDistinctiveDescriptors(desc, offsets)
    assert np.array_equal(best, ref)
    dbest, dout = pkg.ORBmatcher.compute_distinctive_descriptors_device(torch.from_numpy(desc).cuda(),
                                                                       torch.from_numpy(offsets).cuda())
    assert np.array_equal(dbest.cpu().numpy(), ref)
    big = np.array([0, 65536], np.int32)
    bd = np.zeros((65536, 32), np.uint8)
    b = np.zeros(1, np.int32)
    o = np.zeros((1, 32), np.uint8)
    rc = pkg._lib.load().orb_compute_distinctive_descriptors(m._handle(), bd.ctypes.data, big.ctypes.data, 1,
                                                             b.ctypes.data, o.ctypes.data)
    assert rc == pkg._lib.ORB_ERR_ARG


@pytest.mark.parametrize("seed", [1, 2])
def test_compute_distinctive_descriptors_parity(pkg, oracle, seed):
    """MapPoint::ComputeDistinctiveDescriptors batched: best row and mDescriptor equal the oracle for
    point sizes 0..300 (lanes looping over rows beyond 64), duplicates (ties) and random rows."""
    import torch
    rng = np.random.default_rng(seed)
    sizes = [0, 1, 2, 3, 4, 7, 16, 63, 64, 65, 128, 300, 0, 5] + list(rng.integers(1, 40, 200))
    rows = []
    for n in sizes:
        base = rng.integers(0, 256, 32, dtype=np.uint8)
        blk = np.repeat(base[None], n, 0)
        flip = rng.random((n, 32)) < rng.uniform(0.02, 0.3)
        blk ^= (flip * rng.integers(1, 256, (n, 32))).astype(np.uint8)
        if n > 4:
            blk[n // 2] = blk[1]  # an exact duplicate
        rows.append(blk)
    desc = np.concatenate(rows)
    offsets = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    ref = oracle.compute_distinctive_descriptors(desc, offsets)
    m = pkg.ORBmatcher(0.6, False)
    best, out = m.ComputeDistinctiveDescriptors(desc, offsets)
    assert np.array_equal(best, ref)
    for p, b in enumerate(ref):
        exp = desc[offsets[p] + b] if b >= 0 else np.zeros(32, np.uint8)
        assert np.array_equal(out[p], exp), p
    dbest, dout = pkg.ORBmatcher.compute_distinctive_descriptors_device(torch.from_numpy(desc).cuda(),
                                                                       torch.from_numpy(offsets).cuda())
    assert np.array_equal(dbest.cpu().numpy(), ref)
    assert np.array_equal(dout.cpu().numpy()[ref >= 0], out[ref >= 0])
