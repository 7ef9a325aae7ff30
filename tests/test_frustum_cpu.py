"""Frame::isInFrustum + MapPoint::PredictScale oracle (oracle/orb_frustum_oracle.cpp) against an
independent numpy float32 reading of reference src/Frame.cc:667-773 and src/MapPoint.cc:658-731.
The contractions g++ applies (fma) are emulated in double and rounded to float, so the float
outputs are compared to 1 ulp; the flags and predicted levels exactly.  PredictScale is float
arithmetic with glibc's logf (the reference's unqualified log(float) under `using namespace std`,
Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:36), which decides the level on the scale steps."""
from __future__ import annotations

import math
import pathlib
import subprocess

import numpy as np
import pytest

f32 = np.float32
ROOT = pathlib.Path(__file__).resolve().parents[1]


def predict_scale(ratio, lsf, nlev):
    """(int)ceilf(logf(ratio) / lsf) clamped to [0, nlev) (src/MapPoint.cc:715-731), float throughout."""
    from orbslam3_amd.keyframe import logf
    q = f32(logf(ratio) / f32(lsf))
    if not np.isfinite(q):
        return 0  # (int) of +-inf / NaN is INT_MIN on x86
    return min(max(math.ceil(float(q)), 0), nlev - 1)


def _fma(a, b, c):  # float32 fma via double (a*b exact in double)
    return f32(np.float64(a) * np.float64(b) + np.float64(c))


def _dot3(a, b):
    return _fma(a[2], b[2], _fma(a[0], b[0], f32(a[1] * b[1])))


def python_is_in_frustum(Tcw, Ow, cam, bf, bounds, lsf, nlev, P, N, mn, mx, cos_lim):
    fx, fy, cx, cy = (f32(c) for c in cam)
    n = len(P)
    out = dict(track_in_view=np.zeros(n, np.uint8), track_proj=np.zeros((n, 3), np.float32),
               track_depth=np.zeros(n, np.float32), track_level=np.zeros(n, np.int32),
               track_view_cos=np.zeros(n, np.float32))
    out["track_proj"][:, :2] = -1
    for i in range(n):
        p = P[i]
        Pc = [f32(_fma(Tcw[r, 2], p[2], _fma(Tcw[r, 0], p[0], f32(Tcw[r, 1] * p[1]))) + Tcw[r, 3]) for r in range(3)]
        pc_dist = f32(np.sqrt(_dot3(Pc, Pc)))
        invz = f32(f32(1.0) / Pc[2])
        if Pc[2] < 0:
            continue
        u = f32(f32(fx * Pc[0]) / Pc[2]) + cx
        v = f32(f32(fy * Pc[1]) / Pc[2]) + cy
        u, v = f32(u), f32(v)
        if u < bounds[0] or u > bounds[1] or v < bounds[2] or v > bounds[3]:
            continue
        out["track_proj"][i, :2] = (u, v)
        PO = [f32(p[k] - Ow[k]) for k in range(3)]
        dist = f32(np.sqrt(_dot3(PO, PO)))
        if dist < f32(f32(0.8) * mn[i]) or dist > f32(f32(1.2) * mx[i]):
            continue
        vc = f32(_dot3(PO, N[i]) / dist)
        if vc < f32(cos_lim):
            continue
        ratio = f32(mx[i] / dist)
        lev = predict_scale(ratio, lsf, nlev)
        out["track_in_view"][i] = 1
        out["track_proj"][i, 2] = _fma(-f32(bf), invz, u)
        out["track_depth"][i] = pc_dist
        out["track_level"][i] = lev
        out["track_view_cos"][i] = vc
    return out


def _ulp_close(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    return np.all(np.abs(a.view(np.int32).astype(np.int64) - b.view(np.int32).astype(np.int64)) <= 1)


@pytest.mark.parametrize("seed,cos_lim", [(61, 0.5), (62, 0.0), (63, 0.9)])
def test_frustum_oracle_matches_numpy(pkg, synth, oracle, seed, cos_lim):
    Tcw, Ow, P, N, mn, mx = synth.frustum_points(1500, seed=seed)
    fr = pkg.frustum_frame(Tcw, Ow, synth.EUROC_K, synth.EUROC_BF, (0, 752, 0, 480))
    r = oracle.is_in_frustum(fr, P, N, mn, mx, cos_lim)
    q = python_is_in_frustum(Tcw, Ow, synth.EUROC_K, synth.EUROC_BF, (0, 752, 0, 480), fr.log_scale_factor, 8, P, N,
                             mn, mx, cos_lim)
    assert np.array_equal(r["track_in_view"], q["track_in_view"])
    assert np.array_equal(r["track_level"], q["track_level"])
    for k in ("track_proj", "track_depth", "track_view_cos"):
        assert _ulp_close(r[k], q[k]), k
    assert 0.2 * len(P) < r["track_in_view"].sum() < 0.8 * len(P)


def scale_step_points(synth, nlev=8):
    """Map points whose ratio mfMaxDistance / dist is exactly a scale factor 1.2^k (a frame at its
    reference keyframe's distance), one float ulp either side, and a few off-step ratios.  Camera at
    the origin looking down +z, points on the axis at distance 2 (exact), so ratio = max_dist / 2."""
    scale, _ = synth.scale_tables(nlev)
    ratios = []
    for s_ in list(scale) + [f32(0.9), f32(0.84), f32(1.1), f32(5.0)]:
        s_ = f32(s_)
        ratios += [s_, np.nextafter(s_, f32(np.inf)), np.nextafter(s_, f32(0))]
    ratios = np.array(ratios, np.float32)
    n = len(ratios)
    P = np.tile(np.array([0, 0, 2], np.float32), (n, 1))
    N = np.tile(np.array([0, 0, 1], np.float32), (n, 1))
    mx = (ratios * f32(2)).astype(np.float32)
    mn = np.full(n, 0.1, np.float32)
    T = np.concatenate([np.eye(3), np.zeros((3, 1))], 1).astype(np.float32)
    return T, np.zeros(3, np.float32), P, N, mn, mx, ratios


def test_predict_scale_on_scale_steps(pkg, synth, oracle):
    """the level on exact scale steps follows float logf, e.g. ratio 1.2f -> level 1."""
    T, Ow, P, N, mn, mx, ratios = scale_step_points(synth)
    fr = pkg.frustum_frame(T, Ow, synth.EUROC_K, synth.EUROC_BF, (0, 752, 0, 480))
    r = oracle.is_in_frustum(fr, P, N, mn, mx, 0.5)
    assert r["track_in_view"].all()
    exp = [predict_scale(q, fr.log_scale_factor, 8) for q in ratios]
    assert list(r["track_level"]) == exp
    # ratio 1 -> logf = 0 -> level 0; ratio 1.2f -> logf(1.2f) / logf(1.2f) = 1 -> level 1 (in double
    # the quotient is 1 + 2e-8 and the level 2)
    assert r["track_level"][0] == 0 and r["track_level"][3] == 1


def test_predict_scale_thresholds_exhaustive():
    """The kernel's threshold form of PredictScale equals ceilf(logf(r) / lsf) for every float ratio
    a map point produces (tests/native/predict_scale_check.cpp; glibc's logf monotone there)."""
    out = ROOT / "build" / "tests"
    out.mkdir(parents=True, exist_ok=True)
    exe = out / "predict_scale_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off",
                    str(ROOT / "tests" / "native" / "predict_scale_check.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "\nOK " in "\n" + r.stdout, r.stdout + r.stderr
