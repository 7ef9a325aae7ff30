"""Frame::ComputeStereoMatches oracle (oracle/orb_stereo_oracle.cpp) against an independent
pure-Python restatement of reference src/Frame.cc:1102-1358, on synthetic EuRoC-shaped stereo pairs.

The reference ships no stereo fixtures, so parity with the real reference is
unpinned; this pins the C restatement against a second, loop-by-loop reading of the source.
"""
from __future__ import annotations

import math

import numpy as np
import pytest

EUROC_B = 0.110074  # Examples/Stereo/EuRoC.yaml: Camera.bf / fx


def _popcount_dist(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def python_stereo(kl, dl, kr, dr, planes_l, planes_r, scale, inv_scale, bf, b):
    """Loop-by-loop restatement (float32 via numpy scalars where the reference uses float)."""
    f32 = np.float32
    n = len(kl)
    ur = np.full(n, -1.0, np.float32)
    dp = np.full(n, -1.0, np.float32)
    n_rows = planes_l[0].shape[0] - 38
    rows = [[] for _ in range(n_rows)]
    for ir in range(len(kr)):
        y = f32(kr[ir]["y"])
        r = f32(2.0) * f32(scale[kr[ir]["octave"]])
        for yi in range(math.floor(f32(y - r)), math.ceil(f32(y + r)) + 1):
            if 0 <= yi < n_rows:
                rows[yi].append(ir)
    max_d = f32(f32(bf) / f32(b))
    pairs = []
    for il in range(n):
        kp = kl[il]
        lvl = int(kp["octave"])
        vl, ul = f32(kp["y"]), f32(kp["x"])
        cand = rows[int(vl)]
        if not cand:
            continue
        min_u, max_u = f32(ul - max_d), f32(ul - f32(0))
        if max_u < 0:
            continue
        best, best_i = 100, 0
        for ir in cand:
            o = int(kr[ir]["octave"])
            if o < lvl - 1 or o > lvl + 1:
                continue
            u = f32(kr[ir]["x"])
            if min_u <= u <= max_u:
                d = _popcount_dist(dl[il], dr[ir])
                if d < best:
                    best, best_i = d, ir
        if best >= 75:
            continue
        sf = f32(inv_scale[lvl])
        rnd = lambda v: f32(math.floor(abs(float(v)) + 0.5) * (1 if v >= 0 else -1))  # std::round
        su_l, sv_l = rnd(f32(ul * sf)), rnd(f32(vl * sf))
        su_r = rnd(f32(f32(kr[best_i]["x"]) * sf))
        lw = planes_r[lvl].shape[1] - 38
        if su_r < 0 or su_r + 11 >= lw:
            continue
        il_img = planes_l[lvl][19:-19, 19:-19].astype(np.int32)
        ir_img = planes_r[lvl][19:-19, 19:-19].astype(np.int32)
        cu_l, cv_l, cu_r = int(su_l), int(sv_l), int(su_r)
        patch = il_img[cv_l - 5:cv_l + 6, cu_l - 5:cu_l + 6]
        dists = []
        best_s, best_inc = None, 0
        for inc in range(-5, 6):
            s = f32(np.abs(patch - ir_img[cv_l - 5:cv_l + 6, cu_r + inc - 5:cu_r + inc + 6]).sum())
            if best_s is None or s < best_s:
                best_s, best_inc = s, inc
            dists.append(s)
        if best_inc in (-5, 5):
            continue
        d1, d2, d3 = dists[best_inc + 4], dists[best_inc + 5], dists[best_inc + 6]
        delta = f32(f32(d1 - d3) / f32(f32(2.0) * f32(f32(d1 + d3) - f32(f32(2.0) * d2))))
        if delta < -1 or delta > 1:
            continue
        best_u = f32(f32(scale[lvl]) * f32(f32(f32(su_r) + f32(best_inc)) + delta))
        disp = f32(ul - best_u)
        if f32(0) <= disp < max_d:
            if disp <= 0:
                disp = f32(0.01)
                best_u = f32(float(ul) - 0.01)
            dp[il] = f32(f32(bf) / disp)
            ur[il] = best_u
            pairs.append((int(best_s), il))
    if not pairs:
        return ur, dp, 0
    pairs.sort()
    median = f32(pairs[len(pairs) // 2][0])
    th = f32(f32(f32(1.5) * f32(1.4)) * median)
    kept = len(pairs)
    for d, il in reversed(pairs):
        if f32(d) < th:
            break
        ur[il] = dp[il] = -1.0
        kept -= 1
    return ur, dp, kept


def _extract_pair(oracle, synth, seed, nf=1200, w=752, h=480, dmin=4, dmax=48):
    left, right, _ = synth.stereo_pair(w, h, seed=seed, dmin=dmin, dmax=dmax)
    exl, exr = oracle.OracleExtractor(nf, 1.2, 8, 20, 7), oracle.OracleExtractor(nf, 1.2, 8, 20, 7)
    kl, dl, _ = exl(left, (0, 0))
    kr, dr, _ = exr(right, (0, 0))
    pl = [exl.level_padded(l) for l in range(8)]
    pr = [exr.level_padded(l) for l in range(8)]
    return kl, dl, kr, dr, pl, pr, exl.params()


@pytest.mark.parametrize("seed,bf", [(200, 47.90639384423901), (231, 47.90639384423901), (232, 8.0)])
def test_stereo_oracle_matches_python(oracle, synth, seed, bf):
    kl, dl, kr, dr, pl, pr, p = _extract_pair(oracle, synth, seed)
    ur, dp, kept = oracle.compute_stereo_matches(kl, dl, kr, dr, pl, pr, p["scale"], p["inv_scale"], bf, EUROC_B)
    pur, pdp, pkept = python_stereo(kl, dl, kr, dr, pl, pr, p["scale"], p["inv_scale"], bf, EUROC_B)
    assert kept == pkept == int((ur >= 0).sum())
    assert np.array_equal(ur.view(np.uint32), pur.view(np.uint32))
    assert np.array_equal(dp.view(np.uint32), pdp.view(np.uint32))
    if bf > 40:
        assert kept > 100  # the synthetic pair has real stereo structure


def test_stereo_oracle_quality(oracle, synth):
    """Kept matches recover the generator's disparity (per 16-row x 64-col block) to ~1 px."""
    left, right, disp = synth.stereo_pair(752, 480, seed=200)
    kl, dl, kr, dr, pl, pr, p = _extract_pair(oracle, synth, 200)
    ur, dp, kept = oracle.compute_stereo_matches(kl, dl, kr, dr, pl, pr, p["scale"], p["inv_scale"],
                                                 47.90639384423901, EUROC_B)
    good = np.flatnonzero(ur >= 0)
    truth = disp[(kl["y"][good] // 16).astype(int), (kl["x"][good] // 64).astype(int)]
    err = np.abs((kl["x"][good] - ur[good]) - truth)
    assert np.median(err) < 1.0


def test_stereo_oracle_edge_cases(oracle, synth):
    kl, dl, kr, dr, pl, pr, p = _extract_pair(oracle, synth, 200)
    # no right keypoints: nothing matches (and no cull on an empty set)
    ur, dp, kept = oracle.compute_stereo_matches(kl, dl, kr[:0], dr[:0], pl, pr, p["scale"], p["inv_scale"],
                                                 47.9, EUROC_B)
    assert kept == 0 and (ur == -1).all() and (dp == -1).all()
    # right == left: SAD 0 everywhere, so the median cull (SAD >= 1.5*1.4*0) drops every match
    ur, dp, kept = oracle.compute_stereo_matches(kl, dl, kl, dl, pl, pl, p["scale"], p["inv_scale"], 47.9, EUROC_B)
    assert kept == 0 and (ur == -1).all()
    # top rows identical, the rest a real pair: zero-disparity matches take the 0.01 clamp and survive
    left, right, _ = synth.stereo_pair(752, 480, seed=200)
    right[:160] = left[:160]
    exl, exr = oracle.OracleExtractor(1200, 1.2, 8, 20, 7), oracle.OracleExtractor(1200, 1.2, 8, 20, 7)
    kl, dl, _ = exl(left, (0, 0))
    kr, dr, _ = exr(right, (0, 0))
    pl = [exl.level_padded(l) for l in range(8)]
    pr = [exr.level_padded(l) for l in range(8)]
    ur, dp, kept = oracle.compute_stereo_matches(kl, dl, kr, dr, pl, pr, p["scale"], p["inv_scale"], 47.9, EUROC_B)
    pur, pdp, pkept = python_stereo(kl, dl, kr, dr, pl, pr, p["scale"], p["inv_scale"], 47.9, EUROC_B)
    assert kept == pkept > 0 and np.array_equal(ur, pur) and np.array_equal(dp, pdp)
    assert (ur == (kl["x"].astype(np.float64) - 0.01).astype(np.float32)).any()
