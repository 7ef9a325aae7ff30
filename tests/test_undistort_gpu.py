"""Frame::UndistortKeyPoints on the GPU (orb_undistort_keypoints_device, src/Frame.cc:1003-1051) against
the oracle's restatement of cv::undistortPoints, on the extractor's device layout, and the monocular
device chain that reads it: extraction -> UndistortKeyPoints -> BoW -> SearchForTriangulation, with the
EuRoC monocular distortion (Examples/Monocular/EuRoC.yaml:28-31), against the same chain on the oracle.
Parity with a real OpenCV build is unpinned (no OpenCV here); GPU vs oracle is bit-exact."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EUROC_K = (458.654, 457.296, 367.215, 248.375)
EUROC_D = (-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05)


@pytest.fixture(scope="module")
def mono(pkg, synth, oracle):
    import torch
    L, _, Tcw, _ = synth.stereo_sequence(5, seed=77)
    ex = pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=752, max_height=480, max_batch=8)
    out = ex.extract_batch_device(torch.from_numpy(L).cuda(), (0, 0))
    kun = pkg.undistort_keypoints_device(out, EUROC_K, EUROC_D)
    torch.cuda.synchronize()
    ref = []
    for f in range(len(L)):
        k, d, _ = oracle.OracleExtractor(1000, 1.2, 8, 20, 7)(L[f], (0, 0))
        ref.append((k, d, oracle.undistort_keypoints(k, EUROC_K, EUROC_D)))
    return dict(L=L, Tcw=Tcw, out=out, kun=kun, ref=ref)


def test_undistort_device_vs_oracle(pkg, mono):
    counts = mono["out"][2].cpu().numpy()
    for f, (k, _, ku) in enumerate(mono["ref"]):
        n = int(counts[f, 0])
        assert n == len(k) > 500
        got = pkg.keypoints_to_structured(mono["kun"][f], n)
        assert np.array_equal(got.view(np.uint8), ku.view(np.uint8)), f
        moved = np.hypot(got["x"] - k["x"], got["y"] - k["y"])
        assert moved.max() > 1.0  # EuRoC's k1 = -0.283 moves the corners by pixels


def test_undistort_device_in_place_zero_k1_and_flagged_frames(pkg, synth, oracle):
    import torch
    L, _, _, _ = synth.stereo_sequence(2, seed=78)
    ex = pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=752, max_height=480, max_batch=4)
    out = ex.extract_batch_device(torch.from_numpy(L).cuda(), (0, 0))
    raw = out[0].clone()
    # k1 == 0: a copy of mvKeys
    z = pkg.undistort_keypoints_device(out, EUROC_K, (0.0,) + EUROC_D[1:])
    torch.cuda.synchronize()
    n = out[2].cpu().numpy()
    for f in range(2):
        assert torch.equal(z[f, :n[f, 0]].view(torch.int32), raw[f, :n[f, 0]].view(torch.int32))
    # in place (d_kps_un == d_kps) equals the out-of-place result
    sep = pkg.undistort_keypoints_device(out, EUROC_K, EUROC_D)
    pkg.undistort_keypoints_device(out, EUROC_K, EUROC_D, out=out[0])
    torch.cuda.synchronize()
    for f in range(2):
        assert torch.equal(out[0][f, :n[f, 0]].view(torch.int32), sep[f, :n[f, 0]].view(torch.int32))
    # a frame over the capacity is not read or written
    small = ex.extract_batch_device(torch.from_numpy(L).cuda(), (0, 0), cap=100)
    marker = torch.full_like(small[0], -7.0)
    pkg.undistort_keypoints_device(small, EUROC_K, EUROC_D, out=marker)
    torch.cuda.synchronize()
    assert (small[2].cpu().numpy()[:, 1] == pkg._lib.ORB_ERR_CAPACITY).all()
    assert (marker == -7.0).all()


@pytest.mark.parametrize("check_ori", [0, 1])
def test_mono_chain_on_undistorted_keypoints(pkg, synth, oracle, mono, check_ori):
    """The monocular CreateNewMapPoints chain on mvKeysUn: SearchForTriangulation of the newest keyframe
    against its predecessors, device-resident (undistorted keypoints, BoW), against the oracle chain."""
    import torch
    voc = synth.dbow_vocabulary(10, 5, seed=62)
    vocab = pkg.ORBVocabulary(voc)
    scale, sigma2 = synth.scale_tables()
    kps, desc, counts = mono["out"]
    bow = vocab.transform_frames_device(desc, counts, 4)
    n = len(mono["ref"])
    dev = [pkg.DeviceKeyFrame((mono["kun"], desc, counts), bow, f, mono["Tcw"][f], EUROC_K, scale, sigma2)
           for f in range(n)]
    refs = []
    for f, (_, d, ku) in enumerate(mono["ref"]):
        _, fv = oracle.bow_transform(voc, d, 4)
        refs.append(pkg.KeyFrame(keys_un=ku, descriptors=d, Tcw=mono["Tcw"][f], camera=EUROC_K, scale_factors=scale,
                                 level_sigma2=sigma2, feat_vec=fv))
    m = pkg.ORBmatcher(0.6, bool(check_ori))
    k1 = n - 1
    m12, cnt = m.SearchForTriangulationDevice(dev[k1], dev[:k1], False, False)
    torch.cuda.synchronize()
    m12, cnt = m12.cpu().numpy(), cnt.cpu().numpy()
    total = 0
    for p in range(k1):
        rn, rm = oracle.search_for_triangulation(refs[k1], refs[p], m.pair_geometry(refs[k1], refs[p]), False, False,
                                                 check_ori)
        assert cnt[p] == rn and np.array_equal(m12[p, :refs[k1].N], rm), (p, cnt[p], rn)
        total += rn
    assert total > 0
