"""GPU parity of Frame::ComputeStereoMatches (orb_compute_stereo_matches*, HIP) against the CPU
oracle (oracle/orb_stereo_oracle.cpp): mvuRight / mvDepth bit-exact, same kept count."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EUROC_BF, EUROC_B = 47.90639384423901, 0.110074


def _oracle_pair(oracle, left, right, nf=1200):
    exl, exr = oracle.OracleExtractor(nf, 1.2, 8, 20, 7), oracle.OracleExtractor(nf, 1.2, 8, 20, 7)
    kl, dl, _ = exl(left, (0, 0))
    kr, dr, _ = exr(right, (0, 0))
    return kl, dl, kr, dr, [exl.level_padded(l) for l in range(8)], [exr.level_padded(l) for l in range(8)], exl.params()


@pytest.mark.parametrize("seed,bf", [(200, EUROC_BF), (231, EUROC_BF), (232, 8.0), (233, EUROC_BF)])
def test_stereo_matches_single_frame(pkg, oracle, synth, seed, bf):
    left, right, _ = synth.stereo_pair(752, 480, seed=seed)
    exl = pkg.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480)
    exr = pkg.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480)
    kl, dl, _ = exl(left, None, (0, 0))
    kr, dr, _ = exr(right, None, (0, 0))
    ur, dp, kept = pkg.compute_stereo_matches(exl, exr, kl, dl, kr, dr, bf, EUROC_B)
    okl, odl, okr, odr, pl, pr, p = _oracle_pair(oracle, left, right)
    assert np.array_equal(kl.view(np.uint8), okl.view(np.uint8)) and np.array_equal(dl, odl)
    rur, rdp, rkept = oracle.compute_stereo_matches(okl, odl, okr, odr, pl, pr, p["scale"], p["inv_scale"], bf, EUROC_B)
    assert kept == rkept
    assert np.array_equal(ur.view(np.uint32), rur.view(np.uint32)), np.flatnonzero(ur != rur)[:10]
    assert np.array_equal(dp.view(np.uint32), rdp.view(np.uint32))


def test_stereo_matches_batch_device(pkg, oracle, synth):
    import torch
    pairs = [synth.stereo_pair(752, 480, seed=300 + i) for i in range(5)]
    L = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    R = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    exl = pkg.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480, max_batch=8)
    exr = pkg.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480, max_batch=8)
    out_l = exl.extract_batch_device(L, (0, 0))
    out_r = exr.extract_batch_device(R, (0, 0))
    u, d, kept = pkg.compute_stereo_matches_batch_device(exl, exr, out_l, out_r, EUROC_BF, EUROC_B)
    torch.cuda.synchronize()
    u, d, kept = u.cpu().numpy(), d.cpu().numpy(), kept.cpu().numpy()
    for f, (left, right, _) in enumerate(pairs):
        okl, odl, okr, odr, pl, pr, p = _oracle_pair(oracle, left, right)
        rur, rdp, rkept = oracle.compute_stereo_matches(okl, odl, okr, odr, pl, pr, p["scale"], p["inv_scale"],
                                                        EUROC_BF, EUROC_B)
        n = len(okl)
        assert int(out_l[2][f, 0]) == n
        assert kept[f] == rkept, f
        assert np.array_equal(u[f, :n].view(np.uint32), rur.view(np.uint32)), f
        assert np.array_equal(d[f, :n].view(np.uint32), rdp.view(np.uint32)), f


def test_stereo_matches_edge_cases(pkg, oracle, synth):
    left, right, _ = synth.stereo_pair(752, 480, seed=200)
    exl = pkg.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480)
    exr = pkg.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480)
    kl, dl, _ = exl(left, None, (0, 0))
    kr, dr, _ = exr(right, None, (0, 0))
    # no right keypoints
    ur, dp, kept = pkg.compute_stereo_matches(exl, exr, kl, dl, kr[:0], None, EUROC_BF, EUROC_B)
    assert kept == 0 and (ur == -1).all() and (dp == -1).all()
    # no left keypoints
    ur, dp, kept = pkg.compute_stereo_matches(exl, exr, kl[:0], None, kr, dr, EUROC_BF, EUROC_B)
    assert kept == 0 and len(ur) == 0
    # top rows identical (zero disparity: the 0.01 clamp, bestuR = uL - 0.01), the rest a real pair
    right2 = right.copy()
    right2[:160] = left[:160]
    exr2 = pkg.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480)
    kr2, dr2, _ = exr2(right2, None, (0, 0))
    ur, dp, kept = pkg.compute_stereo_matches(exl, exr2, kl, dl, kr2, dr2, EUROC_BF, EUROC_B)
    okl, odl, okr, odr, pl, pr, p = _oracle_pair(oracle, left, right2)
    rur, rdp, rkept = oracle.compute_stereo_matches(okl, odl, okr, odr, pl, pr, p["scale"], p["inv_scale"], EUROC_BF,
                                                    EUROC_B)
    assert kept == rkept > 0 and np.array_equal(ur, rur) and np.array_equal(dp, rdp)
    clamped = ur == (kl["x"].astype(np.float64) - 0.01).astype(np.float32)
    assert clamped.any()
    # mismatched frame sizes are rejected
    exs = pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=752, max_height=480)
    exs(synth.polygon_frame(640, 480, seed=1), None, (0, 0))
    with pytest.raises(pkg.OrbGpuError):
        pkg.compute_stereo_matches(exl, exs, kl, dl, kr, dr, EUROC_BF, EUROC_B)
