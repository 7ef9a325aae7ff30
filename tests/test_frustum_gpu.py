"""GPU parity of Frame::isInFrustum (orb_is_in_frustum, HIP) against the oracle -- every field
bit-exact -- and the tracking chain isInFrustum -> SearchByProjection(Frame, local MapPoints) on the
GPU against the same chain on the oracle."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed,cos_lim", [(61, 0.5), (62, 0.0), (63, 0.9), (64, -1.0)])
def test_is_in_frustum_parity(pkg, oracle, synth, seed, cos_lim):
    Tcw, Ow, P, N, mn, mx = synth.frustum_points(20000, seed=seed)
    fr = pkg.frustum_frame(Tcw, Ow, synth.EUROC_K, synth.EUROC_BF, (0, 752, 0, 480))
    got = pkg.is_in_frustum(fr, P, N, mn, mx, cos_lim)
    exp = oracle.is_in_frustum(fr, P, N, mn, mx, cos_lim)
    for k in exp:
        assert np.array_equal(np.asarray(got[k]).view(np.uint8), np.asarray(exp[k]).view(np.uint8)), k
    assert got["track_in_view"].sum() > 1000


def _local_points_from_frame(synth, cur, n_extra=800, seed=5):
    rng = np.random.default_rng(seed)
    kps, desc = cur["keys_un"], cur["descriptors"]
    fx, fy, cx, cy = synth.EUROC_K
    T = np.asarray(cur["Tcw"], np.float64).reshape(3, 4)
    R, t = T[:, :3], T[:, 3]
    Ow = -R.T @ t
    pick = rng.choice(len(kps), size=min(1200, len(kps)), replace=False)
    z = rng.uniform(2, 12, len(pick))
    Xc = np.stack([(kps["x"][pick] - cx) * z / fx, (kps["y"][pick] - cy) * z / fy, z], 1)
    Xw = (Xc - t) @ R
    Xw = np.concatenate([Xw, Ow + rng.normal(0, 6.0, (n_extra, 3))])
    view = Xw - Ow
    d = np.linalg.norm(view, axis=1)
    nrm = view / d[:, None] + rng.normal(0, 0.2, view.shape)
    nrm /= np.linalg.norm(nrm, axis=1)[:, None]
    scale, _ = synth.scale_tables(8)
    oct_ = np.concatenate([kps["octave"][pick], rng.integers(0, 8, n_extra)])
    mx = d * scale[oct_] * rng.uniform(0.9, 1.1, len(d))
    mn = mx / scale[7]
    D = np.concatenate([desc[pick], rng.integers(0, 256, (n_extra, 32), dtype=np.uint8)])
    flips = np.packbits((rng.random((len(D), 256)) < 0.03).astype(np.uint8), axis=1)
    D = D ^ flips
    f = np.float32
    return (T.astype(f), Ow.astype(f), Xw.astype(f), nrm.astype(f), mn.astype(f), mx.astype(f), D)


@pytest.mark.parametrize("seed,th", [(71, 1), (72, 3)])
def test_tracking_chain_frustum_then_local_search(pkg, oracle, synth, seed, th):
    cur, _ = synth.tracking_pair(seed=seed)
    F = pkg.Frame(**cur)
    T, Ow, Xw, nrm, mn, mx, D = _local_points_from_frame(synth, cur, seed=seed)
    fr = pkg.frustum_frame(T, Ow, synth.EUROC_K, synth.EUROC_BF, (0, 752, 0, 480))
    n = len(Xw)
    fixed = dict(is_bad=np.zeros(n, np.uint8), observed=np.ones(n, np.uint8), desc=D)
    track_gpu = pkg.is_in_frustum(fr, Xw, nrm, mn, mx, 0.5)
    track_ref = oracle.is_in_frustum(fr, Xw, nrm, mn, mx, 0.5)
    m = pkg.ORBmatcher(0.8, True)
    n_gpu, got = m.SearchByProjection(F, pkg.LocalMapPoints(**track_gpu, **fixed), th, False, 10.0, None)
    n_ref, exp = oracle.search_by_projection_local(F, pkg.LocalMapPoints(**track_ref, **fixed), th, False, 10.0, 0.8,
                                                   None)
    assert n_gpu == n_ref > 100 and np.array_equal(got, exp)


def test_predict_scale_on_scale_steps_gpu(pkg, oracle, synth):
    """on the GPU the level on exact scale steps (ratio == 1.2f^k, +-1 ulp) follows the
    reference's float ceilf(logf(ratio) / mfLogScaleFactor), bit-equal to the oracle's glibc logf."""
    from test_frustum_cpu import predict_scale, scale_step_points
    T, Ow, P, N, mn, mx, ratios = scale_step_points(synth)
    fr = pkg.frustum_frame(T, Ow, synth.EUROC_K, synth.EUROC_BF, (0, 752, 0, 480))
    got = pkg.is_in_frustum(fr, P, N, mn, mx, 0.5)
    exp = oracle.is_in_frustum(fr, P, N, mn, mx, 0.5)
    assert np.array_equal(got["track_level"], exp["track_level"])
    assert list(got["track_level"]) == [predict_scale(q, fr.log_scale_factor, 8) for q in ratios]
    assert got["track_level"][3] == 1  # ratio 1.2f -> level 1 (double arithmetic would give 2)
