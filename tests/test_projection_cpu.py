"""CPU checks of the SearchByProjection(Frame, Frame) oracle against an independent pure-Python
restatement of src/ORBmatcher.cc:1951-2185 + Frame::GetFeaturesInArea (src/Frame.cc:859-951).
float32 arithmetic, fma contractions emulated in float64 (products of floats are exact there)."""
from __future__ import annotations

import math

import numpy as np
import pytest

f32 = np.float32


def fma32(a, b, c):
    return f32(float(a) * float(b) + float(c))


def _transform(T, x):
    T = T.reshape(-1)
    return [f32(fma32(T[4 * i + 2], x[2], fma32(T[4 * i], x[0], f32(T[4 * i + 1] * x[1]))) + T[4 * i + 3])
            for i in range(3)]


def py_search(C, L, th, mono, check_ori):
    grid = {}
    for i, kp in enumerate(C.mvKeysUn):
        px = int(np.round(f32(f32(kp["x"] - f32(C.mnMinX)) * f32(C.mfGridElementWidthInv))))
        py = int(np.round(f32(f32(kp["y"] - f32(C.mnMinY)) * f32(C.mfGridElementHeightInv))))
        if 0 <= px < 64 and 0 <= py < 48:
            grid.setdefault((px, py), []).append(i)
    T = C.Tcw.reshape(-1)
    twc = [f32(-fma32(T[8 + i], T[11], fma32(T[i], T[3], f32(T[4 + i] * T[7])))) for i in range(3)]
    tlc = _transform(L.Tcw, twc)
    fwd = tlc[2] > f32(C.mb) and not mono
    bwd = -tlc[2] > f32(C.mb) and not mono
    mp = L.map_points
    D = np.unpackbits(mp["desc"][:, None, :] ^ C.mDescriptors[None, :, :], axis=2).sum(axis=2)
    assign = np.full(C.N, -1)
    hist = {}
    n = 0
    for i in range(L.N):
        if not mp["valid"][i]:
            continue
        xc = _transform(C.Tcw, mp["xyz"][i].astype(f32))
        invz = f32(1.0 / float(xc[2]))
        if invz < 0:
            continue
        u = f32(f32(f32(C.fx) * xc[0]) / xc[2]) + f32(C.cx)
        v = f32(f32(f32(C.fy) * xc[1]) / xc[2]) + f32(C.cy)
        u, v = f32(u), f32(v)
        if u < C.mnMinX or u > C.mnMaxX or v < C.mnMinY or v > C.mnMaxY:
            continue
        o = int(L.mvKeysUn[i]["octave"])
        r = f32(f32(th) * C.mvScaleFactors[o])
        lo, hi = (o, -1) if fwd else ((0, o) if bwd else (o - 1, o + 1))
        x0 = max(0, math.floor(f32(f32(f32(u - f32(C.mnMinX)) - r) * f32(C.mfGridElementWidthInv))))
        x1 = min(63, math.ceil(f32(f32(f32(u - f32(C.mnMinX)) + r) * f32(C.mfGridElementWidthInv))))
        y0 = max(0, math.floor(f32(f32(f32(v - f32(C.mnMinY)) - r) * f32(C.mfGridElementHeightInv))))
        y1 = min(47, math.ceil(f32(f32(f32(v - f32(C.mnMinY)) + r) * f32(C.mfGridElementHeightInv))))
        if x0 >= 64 or x1 < 0 or y0 >= 48 or y1 < 0:
            continue
        check = lo > 0 or hi >= 0
        best, bi = 256, -1
        for ix in range(x0, x1 + 1):
            for iy in range(y0, y1 + 1):
                for j in grid.get((ix, iy), []):
                    kp = C.mvKeysUn[j]
                    if check and (kp["octave"] < lo or (hi >= 0 and kp["octave"] > hi)):
                        continue
                    if not (abs(f32(kp["x"] - u)) < r and abs(f32(kp["y"] - v)) < r):
                        continue
                    if assign[j] >= 0 and mp["observed"][assign[j]]:
                        continue
                    if C.mvuRight is not None and C.mvuRight[j] > 0:
                        ur = fma32(-f32(C.mbf), invz, u)
                        if abs(f32(ur - C.mvuRight[j])) > r:
                            continue
                    if D[i, j] < best:
                        best, bi = int(D[i, j]), j
        if best <= 100:
            assign[bi] = i
            n += 1
            if check_ori:
                rot = f32(L.mvKeysUn[i]["angle"] - C.mvKeysUn[bi]["angle"])
                if rot < 0:
                    rot = f32(rot + f32(360))
                b = int(np.floor(float(f32(rot * f32(f32(1) / f32(30)))) + 0.5))
                hist.setdefault(0 if b == 30 else b, []).append(bi)
    if check_ori:
        sizes = [len(hist.get(b, [])) for b in range(30)]
        m1 = m2 = m3 = 0
        i1 = i2 = i3 = -1
        for b, s in enumerate(sizes):
            if s > m1:
                m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, b
            elif s > m2:
                m3, m2, i3, i2 = m2, s, i2, b
            elif s > m3:
                m3, i3 = s, b
        if m2 < f32(0.1) * f32(m1):
            i2 = i3 = -1
        elif m3 < f32(0.1) * f32(m1):
            i3 = -1
        for b, lst in hist.items():
            if b not in (i1, i2, i3):
                for j in lst:
                    assign[j] = -1
                    n -= 1
    return n, assign


@pytest.mark.parametrize("th,mono,ori,stereo", [(7, False, True, True), (15, True, True, False), (7, False, False, True)])
def test_projection_oracle_matches_python(pkg, oracle, synth, th, mono, ori, stereo):
    cur, last = synth.tracking_pair(n_points=500, clutter=120, seed=41, stereo=stereo)
    C, L = pkg.Frame(**cur), pkg.Frame(**last)
    n, m = oracle.search_by_projection_frame(C, L, th, mono, ori)
    pn, pm = py_search(C, L, th, mono, ori)
    assert n == pn and np.array_equal(m, pm), f"{int((m != pm).sum())} differences"
    assert n > 100


def py_search_local(F, P, th, far, th_far, ratio, taken=None):
    grid = {}
    for i, kp in enumerate(F.mvKeysUn):
        px = int(np.round(f32(f32(kp["x"] - f32(F.mnMinX)) * f32(F.mfGridElementWidthInv))))
        py = int(np.round(f32(f32(kp["y"] - f32(F.mnMinY)) * f32(F.mfGridElementHeightInv))))
        if 0 <= px < 64 and 0 <= py < 48:
            grid.setdefault((px, py), []).append(i)
    D = np.unpackbits(P.desc[:, None, :] ^ F.mDescriptors[None, :, :], axis=2).sum(axis=2)
    owner = np.zeros(F.N, bool) if taken is None else taken.astype(bool).copy()
    match = np.full(F.N, -1)
    n = 0
    for i in range(P.n):
        if not P.track_in_view[i] or (far and P.track_depth[i] > f32(th_far)) or P.is_bad[i]:
            continue
        lvl = int(P.track_level[i])
        r = f32(2.5) if float(P.track_view_cos[i]) > 0.998 else f32(4.0)
        if f32(th) != f32(1.0):
            r = f32(r * f32(th))
        rad = f32(r * F.mvScaleFactors[lvl])
        x, y, xr = (f32(v) for v in P.track_proj[i])
        x0 = max(0, math.floor(f32(f32(f32(x - f32(F.mnMinX)) - rad) * f32(F.mfGridElementWidthInv))))
        x1 = min(63, math.ceil(f32(f32(f32(x - f32(F.mnMinX)) + rad) * f32(F.mfGridElementWidthInv))))
        y0 = max(0, math.floor(f32(f32(f32(y - f32(F.mnMinY)) - rad) * f32(F.mfGridElementHeightInv))))
        y1 = min(47, math.ceil(f32(f32(f32(y - f32(F.mnMinY)) + rad) * f32(F.mfGridElementHeightInv))))
        if x0 >= 64 or x1 < 0 or y0 >= 48 or y1 < 0:
            continue
        b1, l1, b2, l2, bi = 256, -1, 256, -1, -1
        for ix in range(x0, x1 + 1):
            for iy in range(y0, y1 + 1):
                for j in grid.get((ix, iy), []):
                    kp = F.mvKeysUn[j]
                    if kp["octave"] < lvl - 1 or kp["octave"] > lvl:
                        continue
                    if not (abs(f32(kp["x"] - x)) < rad and abs(f32(kp["y"] - y)) < rad):
                        continue
                    if owner[j]:
                        continue
                    if F.mvuRight is not None and F.mvuRight[j] > 0 and abs(f32(xr - F.mvuRight[j])) > rad:
                        continue
                    d = int(D[i, j])
                    if d < b1:
                        b2, l2, b1, l1, bi = b1, l1, d, int(kp["octave"]), j
                    elif d < b2:
                        b2, l2 = d, int(kp["octave"])
        if b1 <= 100:
            if l1 == l2 and f32(b1) > f32(f32(ratio) * f32(b2)):
                continue
            match[bi] = i
            owner[bi] = bool(P.observed[i])
            n += 1
    return n, match


@pytest.mark.parametrize("th,far", [(1, False), (3, False), (5, True)])
def test_local_projection_oracle_matches_python(pkg, oracle, synth, th, far):
    cur, _ = synth.tracking_pair(n_points=400, clutter=100, seed=43)
    F = pkg.Frame(**cur)
    P = pkg.LocalMapPoints(**synth.local_map_points(cur, n_points=500, seed=44))
    taken = (np.random.default_rng(3).random(F.N) < 0.05).astype(np.uint8)
    n, m = oracle.search_by_projection_local(F, P, th, far, 10.0, 0.8, taken)
    pn, pm = py_search_local(F, P, th, far, 10.0, 0.8, taken)
    assert n == pn and np.array_equal(m, pm), f"{int((m != pm).sum())} differences"
    assert n > 50
