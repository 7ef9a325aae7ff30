"""Frame::UndistortKeyPoints oracle (oracle/orb_undistort_oracle.cpp, src/Frame.cc:1003-1051): the C
restatement of OpenCV 4.x's cv::undistortPoints against an independent numpy reading of the same
algorithm (bit for bit: both evaluate in IEEE double without contraction), a round trip through the
forward distortion model, and the reference's k1 == 0 copy.  Parity with a real OpenCV build is
unpinned: the reference ships no undistorted keypoints and OpenCV is absent here."""
from __future__ import annotations

import numpy as np

EUROC_K = (458.654, 457.296, 367.215, 248.375)            # Examples/Monocular/EuRoC.yaml:18-21
EUROC_D = (-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05)  # :28-31


def _np_undistort(u, v, K, dist):
    """cvUndistortPointsInternal, R empty, P = K, TermCriteria(COUNT, 5): the OpenCV source's order."""
    fx, fy, cx, cy = (np.float64(np.float32(t)) for t in K)
    k = np.zeros(5)
    k[:len(dist)] = np.asarray(dist, np.float32).astype(np.float64)
    u = np.asarray(u, np.float32).astype(np.float64)
    v = np.asarray(v, np.float32).astype(np.float64)
    ifx, ify = 1.0 / fx, 1.0 / fy
    x0 = x = (u - cx) * ifx
    y0 = y = (v - cy) * ify
    for _ in range(5):
        r2 = x * x + y * y
        icdist = 1.0 / (1.0 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2)
        assert (icdist >= 0).all()
        dx = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x)
        dy = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y
        x = (x0 - dx) * icdist
        y = (y0 - dy) * icdist
    return (fx * x + cx).astype(np.float32), (fy * y + cy).astype(np.float32)


def _kps(n, seed):
    from oracle import oracle
    rng = np.random.default_rng(seed)
    k = np.zeros(n, oracle.KEYPOINT_DTYPE)
    k["x"] = rng.uniform(0, 752, n).astype(np.float32)
    k["y"] = rng.uniform(0, 480, n).astype(np.float32)
    k["size"], k["angle"], k["response"] = 31.0, rng.uniform(0, 360, n), rng.uniform(0, 100, n)
    k["octave"], k["class_id"] = rng.integers(0, 8, n), -1
    return k


def test_undistort_oracle_matches_numpy_reading(oracle):
    k = _kps(5000, 1)
    for dist in (EUROC_D, EUROC_D + (0.011,), (0.05, -0.2, 0.001, -0.002, 0.1)):
        got = oracle.undistort_keypoints(k, EUROC_K, dist)
        ex, ey = _np_undistort(k["x"], k["y"], EUROC_K, dist)
        assert np.array_equal(got["x"].view(np.uint32), ex.view(np.uint32))
        assert np.array_equal(got["y"].view(np.uint32), ey.view(np.uint32))
        # every other field is mvKeys' own
        for f in ("size", "angle", "response", "octave", "class_id"):
            assert np.array_equal(got[f], k[f])


def test_undistort_round_trip(oracle):
    """Distorting the undistorted point with the forward model (k1 k2 p1 p2) lands near the input:
    five iterations converge to a fraction of a pixel inside the EuRoC image."""
    k = _kps(2000, 2)
    got = oracle.undistort_keypoints(k, EUROC_K, EUROC_D)
    fx, fy, cx, cy = EUROC_K
    k1, k2, p1, p2 = EUROC_D
    x = (got["x"].astype(np.float64) - cx) / fx
    y = (got["y"].astype(np.float64) - cy) / fy
    r2 = x * x + y * y
    rad = 1 + k1 * r2 + k2 * r2 * r2
    xd = x * rad + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
    yd = y * rad + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
    err = np.hypot(xd * fx + cx - k["x"], yd * fy + cy - k["y"])
    centre = np.hypot(k["x"] - cx, k["y"] - cy) < 250
    assert err[centre].max() < 0.05, err[centre].max()
    assert np.median(err) < 0.05


def test_undistort_zero_k1_copies(oracle):
    """mDistCoef[0] == 0: mvKeysUn = mvKeys (src/Frame.cc:1007-1011), whatever the other coefficients."""
    k = _kps(100, 3)
    got = oracle.undistort_keypoints(k, EUROC_K, (0.0, 0.1, 0.01, 0.01))
    assert np.array_equal(got.view(np.uint8), k.view(np.uint8))
    assert len(oracle.undistort_keypoints(k[:0], EUROC_K, EUROC_D)) == 0
