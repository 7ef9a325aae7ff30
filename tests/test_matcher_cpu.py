"""CPU checks of the SearchForTriangulation oracle and the matcher's host logic (no GPU needed).

The oracle (oracle/orb_matcher_oracle.cpp) is cross-checked against an independent pure-Python
restatement of src/ORBmatcher.cc:1046-1324 written over plain dicts/lists.  float32 products and
g++'s fma contractions are emulated in float64, where a product of two floats is exact, and the
result is rounded once to float32.  No reference fixture exists for this function (SURVEY.md
sec. 8c), so it is parity-unpinned beyond the reference's own constants (TH_LOW, HISTO_LENGTH, the
3.84 and 100 thresholds).
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

f32 = np.float32


def fma32(a, b, c):
    return f32(float(a) * float(b) + float(c))


def _F12(k1, k2, g):
    def inv(m):
        def cof(i, j):
            i1, i2, j1, j2 = (i + 1) % 3, (i + 2) % 3, (j + 1) % 3, (j + 2) % 3
            return fma32(m[i1][j1], m[i2][j2], -f32(f32(m[i1][j2]) * f32(m[i2][j1])))
        c = [cof(0, 0), cof(1, 0), cof(2, 0)]
        det = fma32(c[2], m[2][0], fma32(c[0], m[0][0], f32(c[1] * f32(m[1][0]))))
        invdet = f32(f32(1.0) / det)
        return [[f32(cof(j, i) * invdet) for j in range(3)] for i in range(3)]

    def mul(a, b):
        return [[fma32(a[i][2], b[2][j], fma32(a[i][0], b[0][j], f32(f32(a[i][1]) * f32(b[1][j]))))
                 for j in range(3)] for i in range(3)]

    K1t = [[f32(k1.fx), f32(0), f32(0)], [f32(0), f32(k1.fy), f32(0)], [f32(k1.cx), f32(k1.cy), f32(1)]]
    K2 = [[f32(k2.fx), f32(0), f32(k2.cx)], [f32(0), f32(k2.fy), f32(k2.cy)], [f32(0), f32(0), f32(1)]]
    t = [f32(v) for v in g.t12]
    tx = [[f32(0), -t[2], t[1]], [t[2], f32(0), -t[0]], [-t[1], t[0], f32(0)]]
    R = [[f32(g.R12[3 * i + j]) for j in range(3)] for i in range(3)]
    return mul(mul(mul(inv(K1t), tx), R), inv(K2))


def py_search_for_triangulation(k1, k2, g, only_stereo, coarse, check_ori):
    F = _F12(k1, k2, g)
    fv1, fv2 = k1.mFeatVec, k2.mFeatVec
    ur1 = k1.mvuRight if k1.mvuRight is not None else np.full(k1.N, -1, f32)
    ur2 = k2.mvuRight if k2.mvuRight is not None else np.full(k2.N, -1, f32)
    mp1 = k1.has_mappoint if k1.has_mappoint is not None else np.zeros(k1.N, np.uint8)
    mp2 = k2.has_mappoint if k2.has_mappoint is not None else np.zeros(k2.N, np.uint8)
    D = np.unpackbits(k1.mDescriptors[:, None, :] ^ k2.mDescriptors[None, :, :], axis=2).sum(axis=2)
    m12 = np.full(k1.N, -1, np.int32)
    hist = {}
    ep = [f32(g.ep[0]), f32(g.ep[1])]
    for node in sorted(set(fv1) & set(fv2)):
        for i1 in fv1[node]:
            if mp1[i1]:
                continue
            st1 = ur1[i1] >= 0
            if only_stereo and not st1:
                continue
            kp1 = k1.mvKeysUn[i1]
            best, bi = 50, -1
            for i2 in fv2[node]:
                if mp2[i2]:
                    continue
                st2 = ur2[i2] >= 0
                if only_stereo and not st2:
                    continue
                d = int(D[i1, i2])
                if d > 50 or d > best:
                    continue
                kp2 = k2.mvKeysUn[i2]
                if not st1 and not st2:
                    ex, ey = f32(ep[0] - kp2["x"]), f32(ep[1] - kp2["y"])
                    if fma32(ex, ex, f32(ey * ey)) < f32(f32(100) * k2.mvScaleFactors[kp2["octave"]]):
                        continue
                ok = coarse
                if not ok:
                    x1, y1, x2, y2 = kp1["x"], kp1["y"], kp2["x"], kp2["y"]
                    a = f32(fma32(x1, F[0][0], f32(y1 * F[1][0])) + F[2][0])
                    b = f32(fma32(x1, F[0][1], f32(y1 * F[1][1])) + F[2][1])
                    c = f32(fma32(x1, F[0][2], f32(y1 * F[1][2])) + F[2][2])
                    num = f32(fma32(a, x2, f32(b * y2)) + c)
                    den = fma32(a, a, f32(b * b))
                    ok = den != 0 and float(f32(f32(num * num) / den)) < 3.84 * float(k2.mvLevelSigma2[kp2["octave"]])
                if ok:
                    best, bi = d, i2
            if bi >= 0:
                m12[i1] = bi
                if check_ori:
                    rot = f32(kp1["angle"] - k2.mvKeysUn[bi]["angle"])
                    if rot < 0:
                        rot = f32(rot + f32(360))
                    v = float(f32(rot * f32(f32(1) / f32(30))))
                    b_ = int(np.floor(v + 0.5))  # std::round: half away from zero (v >= 0)
                    hist.setdefault(0 if b_ == 30 else b_, []).append(i1)
    if check_ori:
        sizes = [len(hist.get(i, [])) for i in range(30)]
        m1 = m2 = m3 = 0
        i1_ = i2_ = i3_ = -1
        for i, s in enumerate(sizes):
            if s > m1:
                m3, m2, m1, i3_, i2_, i1_ = m2, m1, s, i2_, i1_, i
            elif s > m2:
                m3, m2, i3_, i2_ = m2, s, i2_, i
            elif s > m3:
                m3, i3_ = s, i
        if m2 < f32(0.1) * f32(m1):
            i2_ = i3_ = -1
        elif m3 < f32(0.1) * f32(m1):
            i3_ = -1
        for b_, lst in hist.items():
            if b_ not in (i1_, i2_, i3_):
                m12[lst] = -1
    return int((m12 >= 0).sum()), m12


@pytest.fixture(scope="module")
def scene(pkg, synth):
    kfs = synth.keyframe_scene(n_kf=3, n_points=500, clutter=80, seed=77)
    return [pkg.KeyFrame(**k) for k in kfs]


def test_pair_geometry_matches_float64(pkg, scene):
    k1, k2 = scene[0], scene[2]
    g = pkg.ORBmatcher.pair_geometry(k1, k2)
    T1 = np.vstack([k1.Tcw.astype(np.float64), [0, 0, 0, 1]])
    T2 = np.vstack([k2.Tcw.astype(np.float64), [0, 0, 0, 1]])
    T12 = T1 @ np.linalg.inv(T2)
    assert np.allclose(np.array(g.R12).reshape(3, 3), T12[:3, :3], atol=1e-6)
    assert np.allclose(np.array(g.t12), T12[:3, 3], atol=1e-5)
    Cw = np.linalg.inv(T1)[:3, 3]
    C2 = T2[:3, :3] @ Cw + T2[:3, 3]
    ep = [k2.fx * C2[0] / C2[2] + k2.cx, k2.fy * C2[1] / C2[2] + k2.cy]
    assert np.allclose(np.array(g.ep), ep, rtol=1e-5)


@pytest.mark.parametrize("only_stereo,coarse,check_ori", [(0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 1, 1)])
def test_oracle_matches_python_restatement(pkg, oracle, scene, only_stereo, coarse, check_ori):
    k1 = scene[0]
    for k2 in scene[1:]:
        g = pkg.ORBmatcher.pair_geometry(k1, k2)
        n, m = oracle.search_for_triangulation(k1, k2, g, only_stereo, coarse, check_ori)
        pn, pm = py_search_for_triangulation(k1, k2, g, only_stereo, coarse, check_ori)
        assert n == pn and np.array_equal(m, pm), f"{int((m != pm).sum())} differences"
        assert n > 0 or only_stereo


def test_oracle_match_quality(pkg, oracle, synth):
    """Sanity: most returned pairs are true correspondences of the synthetic scene."""
    kfs = synth.keyframe_scene(n_kf=2, n_points=800, clutter=0, seed=5, mappoint_frac=0.0)
    # ground truth: both keyframes list the visible points in the same generator order before the
    # permutation, so recover identity through the descriptors' nearest base (distance <= 40 flips)
    k1, k2 = pkg.KeyFrame(**kfs[0]), pkg.KeyFrame(**kfs[1])
    g = pkg.ORBmatcher.pair_geometry(k1, k2)
    n, m = oracle.search_for_triangulation(k1, k2, g, False, False, False)
    assert n > 100
    d = np.unpackbits(k1.mDescriptors[m >= 0] ^ k2.mDescriptors[m[m >= 0]], axis=1).sum(axis=1)
    assert (d <= 50).all()


def test_matcher_without_gpu_fails_loudly(pkg):
    lib = pkg._lib.load()
    if lib.orb_device_count() > 0:
        pytest.skip("a GPU is visible")
    h = ctypes.c_void_p()
    assert lib.orb_matcher_create(0.6, 0, ctypes.byref(h)) == pkg._lib.ORB_ERR_DEVICE


def _distinctive_py(desc, offsets):
    """Pure-Python reading of MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:438-529)."""
    out = []
    for p in range(len(offsets) - 1):
        rows = desc[offsets[p]:offsets[p + 1]]
        N = len(rows)
        if N == 0:
            out.append(-1)
            continue
        D = [[int(np.unpackbits(rows[i] ^ rows[j]).sum()) for j in range(N)] for i in range(N)]
        best_m, best_i = 2 ** 31 - 1, 0
        for i in range(N):
            med = sorted(D[i])[int(0.5 * (N - 1))]
            if med < best_m:
                best_m, best_i = med, i
        out.append(best_i)
    return np.array(out, np.int32)


def test_oracle_distinctive_descriptors(oracle):
    """The oracle's ComputeDistinctiveDescriptors against a pure-Python reading, including the
    median index truncation (even N) and first-index ties (copies of one descriptor)."""
    rng = np.random.default_rng(17)
    sizes = [0, 1, 2, 3, 4, 5, 8, 13, 30, 0, 64, 2]
    rows = []
    for n in sizes:
        base = rng.integers(0, 256, 32, dtype=np.uint8)
        blk = np.repeat(base[None], n, 0)
        for r in range(n):  # noisy copies of one base, a few exact duplicates
            if r % 4:
                blk[r] ^= (rng.random(32) < 0.15).astype(np.uint8) * rng.integers(1, 256, 32, dtype=np.uint8)
        rows.append(blk)
    desc = np.concatenate(rows) if rows else np.zeros((0, 32), np.uint8)
    offsets = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    assert np.array_equal(oracle.compute_distinctive_descriptors(desc, offsets), _distinctive_py(desc, offsets))
