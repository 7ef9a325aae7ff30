"""CPU checks of the local BA oracle (oracle/orb_ba_oracle.cpp) against an independent numpy model.

g2o's first LM trial is restated here from scratch:
- residuals of EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ;
- central-difference Jacobians on the SE3Quat manifold (pose <- exp(d) * pose, point <- point + d);
- Huber weights;
- lambda = 1e-5 * max diag(H);
- one dense (H + lambda I) step over all free variables, with no Schur complement.

The oracle's state after optimize(1) must equal that step when the trial is accepted.  This pins
the oracle's Jacobian signs, the Schur elimination, the oplus convention and the LM bookkeeping.
The reference ships no BA fixtures, so parity with a real g2o build is
unpinned beyond this.
"""
from __future__ import annotations

import numpy as np
import pytest

f32 = np.float32


def _quat_to_rot(q):
    x, y, z, w = q / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def _exp(d):
    w, u = d[:3], d[3:]
    th = np.linalg.norm(w)
    O = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
    if th < 1e-5:
        R = V = np.eye(3) + O + O @ O
    else:
        R = np.eye(3) + np.sin(th) / th * O + (1 - np.cos(th)) / th ** 2 * O @ O
        V = np.eye(3) + (1 - np.cos(th)) / th ** 2 * O + (th - np.sin(th)) / th ** 3 * O @ O
    return R, V @ u


def _residual(R, t, X, edge, cam, smooth=False):
    Xc = R @ X + t
    fx, fy, cx, cy, bf = (float(cam[k]) for k in ("fx", "fy", "cx", "cy", "bf"))
    if not edge["stereo"]:
        return np.array([edge["obs"][0] - (fx * Xc[0] / Xc[2] + cx), edge["obs"][1] - (fy * Xc[1] / Xc[2] + cy)])
    invz = 1.0 / Xc[2] if smooth else float(f32(1.0 / Xc[2]))
    u = Xc[0] * invz * fx + cx
    v = Xc[1] * invz * fy + cy
    ur = u - (bf * invz if smooth else float(f32(f32(bf) * f32(invz))))
    return np.array([edge["obs"][0] - u, edge["obs"][1] - v, edge["obs"][2] - ur])


def _huber(e2, delta):
    dsqr = float(f32(float(delta) * float(delta)))
    if e2 <= dsqr:
        return e2, 1.0
    s = np.sqrt(e2)
    return 2 * s * float(delta) - dsqr, float(delta) / s


def _first_step(prob):
    pose, point, edges, cams = prob["pose"], prob["point"], prob["edges"], prob["pose_camera"]
    Rs = [_quat_to_rot(p[3:]) for p in pose]
    free = [i for i in np.argsort(prob["pose_id"], kind="stable") if not prob["pose_fixed"][i]]
    pidx = {p: k for k, p in enumerate(free)}
    lorder = np.argsort(prob["point_id"], kind="stable")
    lidx = {p: k for k, p in enumerate(lorder)}
    n = 6 * len(free)
    N = n + 3 * len(lorder)
    H = np.zeros((N, N))
    b = np.zeros(N)
    chi = 0.0
    dm, ds = f32(np.sqrt(5.991)), f32(np.sqrt(7.815))
    h = 1e-6
    for e in edges:
        k, p = int(e["pose"]), int(e["point"])
        cam = cams[k]
        r = _residual(Rs[k], pose[k, :3], point[p], e, cam)
        info = float(e["inv_sigma2"])
        rho0, rho1 = _huber(float(r @ r) * info, ds if e["stereo"] else dm)
        chi += rho0
        D = len(r)
        J = np.zeros((D, N))
        # d e / d point
        for j in range(3):
            dX = np.zeros(3)
            dX[j] = h
            J[:, n + 3 * lidx[p] + j] = (_residual(Rs[k], pose[k, :3], point[p] + dX, e, cam, True) -
                                        _residual(Rs[k], pose[k, :3], point[p] - dX, e, cam, True)) / (2 * h)
        if k in pidx:
            for j in range(6):
                d = np.zeros(6)
                d[j] = h
                Rp, tp = _exp(d)
                Rm, tm = _exp(-d)
                J[:, 6 * pidx[k] + j] = (_residual(Rp @ Rs[k], Rp @ pose[k, :3] + tp, point[p], e, cam, True) -
                                        _residual(Rm @ Rs[k], Rm @ pose[k, :3] + tm, point[p], e, cam, True)) / (2 * h)
        W = rho1 * info
        H += W * J.T @ J
        b += -info * rho1 * J.T @ r
    lam = 1e-5 * np.abs(np.diag(H)).max()
    dx = np.linalg.solve(H + lam * np.eye(N), b)
    new_pose = pose.copy()
    for k, i in pidx.items():
        Re, te = _exp(dx[6 * i:6 * i + 6])
        new_pose[k, :3] = Re @ pose[k, :3] + te
        new_pose[k, 3:] = _quat_from(Re @ Rs[k])
    new_point = point.copy()
    for p, l in lidx.items():
        new_point[p] += dx[n + 3 * l:n + 3 * l + 3]
    return new_pose, new_point, chi, lam


def _quat_from(R):
    from scipy.spatial.transform import Rotation
    q = Rotation.from_matrix(R).as_quat()  # x, y, z, w
    return q if q[3] >= 0 else -q


@pytest.mark.parametrize("stereo_frac", [0.0, 0.5])
def test_oracle_first_step_matches_dense_numeric_lm(oracle, synth, stereo_frac):
    prob = synth.local_ba_problem(n_kf=5, n_points=60, obs_per_point=4, stereo_frac=stereo_frac, n_fixed=1,
                                  seed=21, outlier_frac=0.1)
    exp_pose, exp_point, chi, lam = _first_step(prob)
    pose, point, _, _, res = oracle.local_ba(prob, 1)
    assert res["iterations"] == 1 and res["trials"] == 1, res  # the first trial is accepted
    assert res["initial_chi2"] == pytest.approx(chi, rel=1e-12)
    assert np.allclose(pose[:, :3], exp_pose[:, :3], atol=1e-6)
    q = np.where((np.sum(pose[:, 3:] * exp_pose[:, 3:], 1) < 0)[:, None], -pose[:, 3:], pose[:, 3:])
    assert np.allclose(q, exp_pose[:, 3:], atol=1e-7)
    assert np.allclose(point, exp_point, atol=1e-6)


def test_oracle_lm_bookkeeping(oracle, synth):
    prob = synth.local_ba_problem(n_kf=8, n_points=200, obs_per_point=5, stereo_frac=0.3, seed=4)
    _, _, _, _, r10 = oracle.local_ba(prob, 10)
    assert 1 <= r10["iterations"] <= 10 and r10["trials"] >= r10["iterations"]
    assert r10["final_chi2"] < r10["initial_chi2"]
    _, _, _, _, r0 = oracle.local_ba(prob, 0)
    assert r0["iterations"] == 0 and r0["trials"] == 0
    pose, point, _, _, rs = oracle.local_ba(prob, 10, stop_flag=np.ones(1, np.int32))
    assert rs["stopped"] == 1 and np.array_equal(point, prob["point"])


def test_stop_flag_must_be_shared_memory(pkg):
    """pbStopFlag is polled memory another thread writes; a converting copy would never
    see the request, so anything but an np.int32 array or a ctypes.c_int32 is refused."""
    import ctypes
    from orbslam3_amd.optimizer import stop_flag_address
    a = np.zeros(1, np.int32)
    assert stop_flag_address(a) == a.ctypes.data
    c = ctypes.c_int32(0)
    assert stop_flag_address(c) == ctypes.addressof(c)
    assert stop_flag_address(None) is None
    for bad in (np.zeros(1, bool), np.zeros(1, np.int64), 1, True, np.zeros((2, 2), np.int32)[:, 0], np.zeros(0, np.int32)):
        with pytest.raises(TypeError):
            stop_flag_address(bad)
