"""Deterministic synthetic inputs for the ORB front-end (no image data ships with the reference).

SURVEY.md sec. 8(d): EuRoC-shaped gray frames made of random filled rectangles and triangles with
additive noise (FAST corners at polygon vertices at roughly EuRoC density), a "blurred noise"
texture that stresses NMS and the quad-tree, and a stereo right view made by shifting the left
view by a piecewise-constant disparity field.
"""
from __future__ import annotations

import numpy as np


def polygon_frame(width: int = 640, height: int = 480, seed: int = 1, n_shapes: int = 400,
                  noise_sigma: float = 3.0) -> np.ndarray:
    """`n_shapes` random rectangles/triangles of uniform random intensity, then N(0, sigma) noise."""
    rng = np.random.default_rng(seed)
    img = np.full((height, width), rng.integers(0, 256), dtype=np.float32)
    yy, xx = np.mgrid[0:height, 0:width]
    for _ in range(n_shapes):
        val = float(rng.integers(0, 256))
        cx, cy = rng.integers(0, width), rng.integers(0, height)
        sx, sy = rng.integers(4, max(5, width // 6)), rng.integers(4, max(5, height // 6))
        x0, x1 = max(0, cx - sx // 2), min(width, cx + sx // 2 + 1)
        y0, y1 = max(0, cy - sy // 2), min(height, cy + sy // 2 + 1)
        if rng.integers(0, 2) == 0:
            img[y0:y1, x0:x1] = val
        else:
            p = rng.integers([x0, y0], [x1 + 1, y1 + 1], size=(3, 2)).astype(np.float32)
            X, Y = xx[y0:y1, x0:x1].astype(np.float32), yy[y0:y1, x0:x1].astype(np.float32)

            def edge(a, b):
                return (b[0] - a[0]) * (Y - a[1]) - (b[1] - a[1]) * (X - a[0])

            e0, e1, e2 = edge(p[0], p[1]), edge(p[1], p[2]), edge(p[2], p[0])
            inside = ((e0 >= 0) & (e1 >= 0) & (e2 >= 0)) | ((e0 <= 0) & (e1 <= 0) & (e2 <= 0))
            img[y0:y1, x0:x1][inside] = val
    img += rng.normal(0.0, noise_sigma, size=img.shape).astype(np.float32)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def blurred_noise_frame(width: int = 640, height: int = 480, seed: int = 2, sigma: float = 1.5) -> np.ndarray:
    """White noise smoothed by a separable Gaussian (sigma px), rescaled to 0..255."""
    rng = np.random.default_rng(seed)
    img = rng.random((height, width), dtype=np.float32)
    r = int(np.ceil(3 * sigma))
    k = np.exp(-0.5 * (np.arange(-r, r + 1) / sigma) ** 2).astype(np.float32)
    k /= k.sum()
    img = np.apply_along_axis(lambda v: np.convolve(np.pad(v, r, mode="reflect"), k, "valid"), 1, img)
    img = np.apply_along_axis(lambda v: np.convolve(np.pad(v, r, mode="reflect"), k, "valid"), 0, img)
    img = (img - img.min()) / max(1e-6, float(img.max() - img.min()))
    return np.clip(np.rint(img * 255), 0, 255).astype(np.uint8)


def stereo_pair(width: int = 752, height: int = 480, seed: int = 200, dmin: int = 4, dmax: int = 48):
    """Left = polygon frame; right = left shifted left by a per-(16-row band, 64-col block) disparity."""
    left = polygon_frame(width, height, seed=seed)
    rng = np.random.default_rng(seed + 1)
    disp = rng.integers(dmin, dmax + 1, size=((height + 15) // 16, (width + 63) // 64))
    right = np.empty_like(left)
    for y in range(height):
        for bx in range(disp.shape[1]):
            d = int(disp[y // 16, bx])
            x0, x1 = bx * 64, min(width, bx * 64 + 64)
            src = np.clip(np.arange(x0, x1) + d, 0, width - 1)
            right[y, x0:x1] = left[y, src]
    noise = rng.normal(0.0, 2.0, size=right.shape)
    right = np.clip(np.rint(right.astype(np.float32) + noise), 0, 255).astype(np.uint8)
    return left, right, disp


def stereo_sequence(n: int, width: int = 752, height: int = 480, seed: int = 210, step_px: int = 6, disparity: int = 13,
                    noise: float = 2.0):
    """C3 as a keyframe stream: n rectified stereo pairs of one fronto-parallel textured plane seen by a
    camera translating along x.  With the plane at depth Z = bf / disparity, frame k is the crop of a
    wide polygon canvas at x = step_px * k (left) and step_px * k + disparity (right, u_R = u_L - d), so
    every frame pair shares most of its corners and the epipolar geometry of the poses is exact:
    Tcw_k = [I | -(k * step_px * Z / fx, 0, 0)].  Returns (left [n, H, W], right [n, H, W], Tcw [n, 3, 4],
    Z)."""
    fx = EUROC_K[0]
    Z = EUROC_BF / disparity
    canvas = polygon_frame(width + step_px * (n - 1) + disparity + 8, height, seed=seed,
                           n_shapes=int(400 * (width + step_px * n) / width))
    rng = np.random.default_rng(seed + 1)
    left = np.stack([canvas[:, step_px * k: step_px * k + width] for k in range(n)])
    right = np.stack([canvas[:, step_px * k + disparity: step_px * k + disparity + width] for k in range(n)])
    right = np.clip(np.rint(right.astype(np.float32) + rng.normal(0.0, noise, right.shape)), 0, 255).astype(np.uint8)
    Tcw = np.zeros((n, 3, 4), np.float32)
    for k in range(n):
        Tcw[k, :, :3] = np.eye(3)
        Tcw[k, 0, 3] = -k * step_px * Z / fx
    return np.ascontiguousarray(left), np.ascontiguousarray(right), Tcw, Z


def frame_batch(n: int, width: int = 640, height: int = 480, seed0: int = 100) -> np.ndarray:
    return np.stack([polygon_frame(width, height, seed=seed0 + i) for i in range(n)])


# ---- keyframes for the matcher ------------------------------------------

EUROC_K = (458.654, 457.296, 367.215, 248.375)  # Examples/Stereo/EuRoC.yaml camera (left)
EUROC_BF = 47.90639384423901                     # fx * baseline (0.110074 m)


def scale_tables(nlevels: int = 8, scale: float = 1.2):
    """mvScaleFactors / mvLevelSigma2 as the extractor computes them (float32 chain)."""
    s = np.zeros(nlevels, np.float32)
    s[0] = 1.0
    for l in range(1, nlevels):
        s[l] = np.float32(float(s[l - 1]) * float(np.float32(scale)))
    return s, (s * s).astype(np.float32)


class SyntheticVocabulary:
    """k=10, two-level synthetic DBoW2-like tree: a feature's node is the level-2 word reached by
    greedy Hamming argmin (first minimum) -- node ids 11..110 as DBoW2 numbers a 10-ary tree.
    Stands in for ORBvoc.txt (absent: .MISSING_LARGE_BLOBS) to build FeatureVectors."""

    def __init__(self, seed: int = 201, k: int = 10):
        rng = np.random.default_rng(seed)
        self.k = k
        self.l1 = rng.integers(0, 256, (k, 32), dtype=np.uint8)
        # children are perturbations of their parent so the tree is coherent
        flips = rng.random((k, k, 256)) < 0.25
        bits = np.unpackbits(self.l1, axis=1)[:, None, :] ^ flips
        self.l2 = np.packbits(bits.astype(np.uint8), axis=2)

    @staticmethod
    def _ham(d, c):
        return np.unpackbits(d[:, None, :] ^ c[None, :, :], axis=2).sum(axis=2)

    def transform(self, desc: np.ndarray) -> dict:
        a = np.argmin(self._ham(desc, self.l1), axis=1)
        fv: dict = {}
        for i in range(len(desc)):
            b = int(np.argmin(self._ham(desc[i:i + 1], self.l2[a[i]])[0]))
            fv.setdefault(1 + self.k + self.k * int(a[i]) + b, []).append(i)
        return fv


def _rot_yaw_pitch(yaw, pitch):
    cy, sy, cp, sp = np.cos(yaw), np.sin(yaw), np.cos(pitch), np.sin(pitch)
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rx = np.array([[1, 0, 0], [0, cp, -sp], [0, sp, cp]])
    return Ry @ Rx


def keyframe_scene(n_kf: int = 4, n_points: int = 1500, seed: int = 201, width: int = 752, height: int = 480,
                   stereo_frac: float = 0.5, mappoint_frac: float = 0.3, clutter: int = 250, nlevels: int = 8,
                   baseline: float = 0.2, yaw_deg: float = 3.0, pixel_noise: float = 0.7):
    """Keyframes observing one random point cloud (depth 2..10 m) from poses along a 0.2 m-step arc.

    Each visible point gives a keypoint with a random octave, noisy projection, an angle shared by the
    point (+ noise) and the point's base descriptor with 0..40 flipped bits; plus random clutter
    keypoints; a fraction has a stereo coordinate (mvuRight = u - bf/z) and a fraction already has a
    MapPoint.  FeatureVectors come from SyntheticVocabulary.  Returns a list of dicts of KeyFrame
    fields (keys_un, descriptors, Tcw, camera, scale_factors, level_sigma2, u_right, has_mappoint,
    feat_vec)."""
    from ._lib import KEYPOINT_DTYPE
    rng = np.random.default_rng(seed)
    voc = SyntheticVocabulary(seed)
    fx, fy, cx, cy = EUROC_K
    scale, sigma2 = scale_tables(nlevels)
    P = np.stack([rng.uniform(-4, 4, n_points), rng.uniform(-2.5, 2.5, n_points), rng.uniform(2, 10, n_points)], 1)
    base = rng.integers(0, 256, (n_points, 32), dtype=np.uint8)
    ang0 = rng.uniform(0, 360, n_points)
    out = []
    for k in range(n_kf):
        R = _rot_yaw_pitch(np.deg2rad(yaw_deg * k), np.deg2rad(0.5 * k))
        C = np.array([baseline * k, 0.02 * k, 0.05 * k])  # camera centre
        t = -R @ C
        Xc = P @ R.T + t
        z = Xc[:, 2]
        u = fx * Xc[:, 0] / z + cx
        v = fy * Xc[:, 1] / z + cy
        vis = np.flatnonzero((z > 0.5) & (u >= 20) & (u < width - 20) & (v >= 20) & (v < height - 20))
        nv = len(vis)
        n = nv + clutter
        kps = np.zeros(n, KEYPOINT_DTYPE)
        octv = rng.integers(0, nlevels, n)
        kps["octave"] = octv
        kps["x"][:nv] = u[vis] + rng.normal(0, pixel_noise, nv) * scale[octv[:nv]]
        kps["y"][:nv] = v[vis] + rng.normal(0, pixel_noise, nv) * scale[octv[:nv]]
        kps["x"][nv:] = rng.uniform(20, width - 20, clutter)
        kps["y"][nv:] = rng.uniform(20, height - 20, clutter)
        kps["angle"][:nv] = np.mod(ang0[vis] + rng.normal(0, 4, nv) + 2.0 * k, 360)
        kps["angle"][nv:] = rng.uniform(0, 360, clutter)
        kps["size"] = 31 * scale[octv]
        kps["response"] = rng.integers(7, 120, n)
        kps["class_id"] = -1
        desc = np.empty((n, 32), np.uint8)
        bits = np.unpackbits(base[vis], axis=1)
        nflip = rng.integers(0, 41, nv)
        for i in range(nv):
            bits[i, rng.choice(256, nflip[i], replace=False)] ^= 1
        desc[:nv] = np.packbits(bits, axis=1)
        desc[nv:] = rng.integers(0, 256, (clutter, 32), dtype=np.uint8)
        # a few exact duplicates so that distance ties occur inside nodes
        dup = rng.choice(n, size=min(20, n // 2), replace=False)
        desc[dup[1::2]] = desc[dup[0::2]]
        ur = np.full(n, -1.0, np.float32)
        st = rng.random(nv) < stereo_frac
        ur[:nv][st] = (kps["x"][:nv][st] - EUROC_BF / z[vis][st]).astype(np.float32)
        perm = rng.permutation(n)
        kps, desc, ur = kps[perm], desc[perm], ur[perm]
        Tcw = np.concatenate([R, t[:, None]], 1).astype(np.float32)
        out.append(dict(keys_un=kps, descriptors=desc, Tcw=Tcw, camera=EUROC_K, scale_factors=scale,
                        level_sigma2=sigma2, u_right=ur,
                        has_mappoint=(rng.random(n) < mappoint_frac).astype(np.uint8),
                        feat_vec=voc.transform(desc)))
    return out


# ---- local bundle adjustment problems ----------------------------------

BA_EDGE_DTYPE = np.dtype([("point", "<i4"), ("pose", "<i4"), ("stereo", "<i4"), ("inv_sigma2", "<f4"),
                          ("obs", "<f8", (3,))])
BA_CAMERA_DTYPE = np.dtype([("fx", "<f4"), ("fy", "<f4"), ("cx", "<f4"), ("cy", "<f4"), ("bf", "<f4")])


def rot_to_quat(R):
    """Rotation matrix -> quaternion (x, y, z, w) with w >= 0."""
    R = np.asarray(R, np.float64)
    t = np.trace(R)
    if t > 0:
        s = np.sqrt(t + 1.0) * 2
        q = np.array([(R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s, 0.25 * s])
    else:
        i = int(np.argmax(np.diag(R)))
        j, k = (i + 1) % 3, (i + 2) % 3
        s = np.sqrt(R[i, i] - R[j, j] - R[k, k] + 1.0) * 2
        q = np.zeros(4)
        q[i] = 0.25 * s
        q[3] = (R[k, j] - R[j, k]) / s
        q[j] = (R[j, i] + R[i, j]) / s
        q[k] = (R[k, i] + R[i, k]) / s
    q /= np.linalg.norm(q)
    return q if q[3] >= 0 else -q


def quat_to_rot(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def _small_rot(rng, sigma):
    w = rng.normal(0, sigma, 3)
    th = np.linalg.norm(w)
    if th < 1e-12:
        return np.eye(3)
    k = w / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def local_ba_problem(n_kf: int = 50, n_points: int = 2000, obs_per_point: int = 6, stereo_frac: float = 0.0,
                     n_fixed: int = 2, seed: int = 7, outlier_frac: float = 0.05, width: int = 752, height: int = 480,
                     nlevels: int = 8):
    """C5: keyframes along a 10 m arc facing a point cloud 2-10 m deep; each point observed by ~6
    keyframes (~12k edges for 2000 points); octave U{0..7}, information 1/1.44^octave, pixel noise
    N(0, 1)*scale, 5 % outliers (+-20 px), poses perturbed by 0.01 rad / 0.02 m and points by
    0.05 m, `n_fixed` fixed keyframes, EuRoC pinhole intrinsics.  Returns a dict of the arrays of
    orb_ba_problem_t plus the ground truth."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = EUROC_K
    scale, sigma2 = scale_tables(nlevels)
    inv_sigma2 = (np.float32(1.0) / sigma2).astype(np.float32)
    # ground truth: camera centres on an arc, looking roughly at the cloud centre (0, 0, 8)
    phis = np.linspace(-0.5, 0.5, n_kf)
    Rs, ts = [], []
    for k, ph in enumerate(phis):
        C = np.array([10.0 * np.sin(ph) * 0.5, 0.3 * np.sin(3 * ph), -10.0 * (1 - np.cos(ph)) * 0.5])
        yaw = -ph * 0.5
        Rwc = np.array([[np.cos(yaw), 0, np.sin(yaw)], [0, 1, 0], [-np.sin(yaw), 0, np.cos(yaw)]])
        Rcw = Rwc.T
        Rs.append(Rcw)
        ts.append(-Rcw @ C)
    P = np.stack([rng.uniform(-5, 5, n_points), rng.uniform(-2.5, 2.5, n_points), rng.uniform(4, 12, n_points)], 1)
    edges = []
    for p in range(n_points):
        vis = []
        for k in range(n_kf):
            Xc = Rs[k] @ P[p] + ts[k]
            if Xc[2] < 1.0:
                continue
            u, v = fx * Xc[0] / Xc[2] + cx, fy * Xc[1] / Xc[2] + cy
            if 10 <= u < width - 10 and 10 <= v < height - 10:
                vis.append((k, u, v, Xc[2]))
        if not vis:
            continue
        sel = rng.choice(len(vis), size=min(obs_per_point, len(vis)), replace=False)
        for s in sorted(sel, key=lambda i: vis[i][0]):
            k, u, v, z = vis[s]
            octv = int(rng.integers(0, nlevels))
            sc = float(scale[octv])
            uo, vo = u + rng.normal(0, 1.0) * sc, v + rng.normal(0, 1.0) * sc
            if rng.random() < outlier_frac:
                uo += rng.uniform(-20, 20)
                vo += rng.uniform(-20, 20)
            st = rng.random() < stereo_frac
            ur = uo - EUROC_BF / z + rng.normal(0, 1.0) * sc if st else 0.0
            edges.append((p, k, int(st), inv_sigma2[octv], (uo, vo, ur)))
    E = np.zeros(len(edges), BA_EDGE_DTYPE)
    for i, (p, k, st, info, obs) in enumerate(edges):
        E[i] = (p, k, st, info, obs)
    pose_gt = np.zeros((n_kf, 7))
    pose0 = np.zeros((n_kf, 7))
    fixed = np.zeros(n_kf, np.uint8)
    fixed[:n_fixed] = 1
    for k in range(n_kf):
        pose_gt[k, :3] = ts[k]
        pose_gt[k, 3:] = rot_to_quat(Rs[k])
        if fixed[k]:
            pose0[k] = pose_gt[k]
        else:
            Rp = _small_rot(rng, 0.01) @ Rs[k]
            pose0[k, :3] = ts[k] + rng.normal(0, 0.02, 3)
            pose0[k, 3:] = rot_to_quat(Rp)
    cams = np.zeros(n_kf, BA_CAMERA_DTYPE)
    cams[:] = (fx, fy, cx, cy, EUROC_BF)
    point0 = P + rng.normal(0, 0.05, P.shape)
    return dict(pose=pose0, pose_id=np.arange(n_kf, dtype=np.int64), pose_fixed=fixed, pose_camera=cams,
                point=point0, point_id=np.arange(n_points, dtype=np.int64) + n_kf + 1, edges=E,
                pose_gt=pose_gt, point_gt=P)


def tracking_pair(n_points: int = 1200, seed: int = 31, width: int = 752, height: int = 480, stereo: bool = True,
                  clutter: int = 300, outlier_frac: float = 0.05, unobserved_frac: float = 0.15, dup_frac: float = 0.05,
                  forward: float = 0.02, nlevels: int = 8):
    """Two consecutive frames for SearchByProjection(CurrentFrame, LastFrame): the last frame tracks
    map points (xyz, descriptor, observed flag, a few outliers); the current frame sees them again
    after a small motion, with noisy keypoints, perturbed descriptors, stereo u_right and clutter.
    A few map points share descriptors and nearby positions so that current keypoints are contested
    (exercises the in-order 'already matched' rule).  Returns dicts for Frame(**cur), Frame(**last)."""
    from ._lib import KEYPOINT_DTYPE
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = EUROC_K
    scale, _ = scale_tables(nlevels)
    P = np.stack([rng.uniform(-4, 4, n_points), rng.uniform(-2.5, 2.5, n_points), rng.uniform(2, 12, n_points)], 1)
    base = rng.integers(0, 256, (n_points, 32), dtype=np.uint8)
    ndup = int(dup_frac * n_points)
    src = rng.choice(n_points, ndup, replace=False)
    dst = rng.choice(n_points, ndup, replace=False)
    P[dst] = P[src] + rng.normal(0, 0.004, (ndup, 3))
    base[dst] = base[src]
    ang = rng.uniform(0, 360, n_points)
    octv = rng.integers(0, nlevels, n_points)

    def frame(R, t, noise, flips):
        Xc = P @ R.T + t
        z = Xc[:, 2]
        u = fx * Xc[:, 0] / z + cx
        v = fy * Xc[:, 1] / z + cy
        vis = np.flatnonzero((z > 0.3) & (u >= 0) & (u < width) & (v >= 0) & (v < height))
        nv = len(vis)
        kps = np.zeros(nv + clutter, KEYPOINT_DTYPE)
        o = octv[vis].copy()
        o = np.clip(o + rng.integers(-1, 2, nv), 0, nlevels - 1)
        kps["octave"][:nv] = o
        kps["x"][:nv] = np.clip(u[vis] + rng.normal(0, noise, nv) * scale[o], 0, width - 1)
        kps["y"][:nv] = np.clip(v[vis] + rng.normal(0, noise, nv) * scale[o], 0, height - 1)
        kps["angle"][:nv] = np.mod(ang[vis] + rng.normal(0, 3, nv), 360)
        kps["x"][nv:] = rng.uniform(0, width - 1, clutter)
        kps["y"][nv:] = rng.uniform(0, height - 1, clutter)
        kps["octave"][nv:] = rng.integers(0, nlevels, clutter)
        kps["angle"][nv:] = rng.uniform(0, 360, clutter)
        kps["size"] = 31 * scale[kps["octave"]]
        kps["class_id"] = -1
        bits = np.unpackbits(base[vis], axis=1)
        for i in range(nv):
            bits[i, rng.choice(256, int(rng.integers(0, flips)), replace=False)] ^= 1
        desc = np.concatenate([np.packbits(bits, axis=1), rng.integers(0, 256, (clutter, 32), dtype=np.uint8)])
        ur = np.full(nv + clutter, -1.0, np.float32)
        if stereo:
            st = rng.random(nv) < 0.6
            ur[:nv][st] = (kps["x"][:nv][st] - EUROC_BF / z[vis][st] + rng.normal(0, 0.5, st.sum())).astype(np.float32)
        perm = rng.permutation(nv + clutter)
        ids = np.concatenate([vis, np.full(clutter, -1)])[perm]
        Tcw = np.concatenate([R, t[:, None]], 1).astype(np.float32)
        return kps[perm], desc[perm], ur[perm], ids, Tcw

    R0, t0 = np.eye(3), np.zeros(3)
    R1 = _rot_yaw_pitch(np.deg2rad(0.8), np.deg2rad(0.3))
    t1 = np.array([0.03, -0.01, -forward])
    lk, ld, lur, lids, lT = frame(R0, t0, 0.3, 12)
    ck, cd, cur_, cids, cT = frame(R1, t1, 0.5, 30)
    valid = (lids >= 0) & (rng.random(len(lids)) > outlier_frac)
    xyz = np.zeros((len(lids), 3), np.float32)
    mdesc = np.zeros((len(lids), 32), np.uint8)
    xyz[lids >= 0] = P[lids[lids >= 0]] + rng.normal(0, 0.01, ((lids >= 0).sum(), 3))
    mdesc[lids >= 0] = base[lids[lids >= 0]]
    observed = (rng.random(len(lids)) > unobserved_frac).astype(np.uint8)
    common = dict(camera=EUROC_K, scale_factors=scale, width=width, height=height, bf=EUROC_BF if stereo else 0.0)
    last = dict(keys_un=lk, descriptors=ld, Tcw=lT, u_right=lur if stereo else None,
                map_points=dict(valid=valid.astype(np.uint8), observed=observed, xyz=xyz, desc=mdesc), **common)
    cur = dict(keys_un=ck, descriptors=cd, Tcw=cT, u_right=cur_ if stereo else None, **common)
    return cur, last


def local_map_points(cur: dict, n_points: int = 1500, seed: int = 51, width: int = 752, height: int = 480,
                     nlevels: int = 8, bad_frac: float = 0.03, unobserved_frac: float = 0.1, dup_frac: float = 0.05):
    """Local map points for SearchByProjection(Frame, vector<MapPoint*>): the tracking fields
    isInFrustum would write for the current frame `cur` (from tracking_pair): projection (u, v, u_R),
    view cosine, depth and predicted level; descriptors close to the frame's keypoints for most
    points; a few bad / unobserved / duplicated points."""
    rng = np.random.default_rng(seed)
    kps = cur["keys_un"]
    desc = cur["descriptors"]
    n = n_points
    pick = rng.integers(0, len(kps), n)
    proj = np.zeros((n, 3), np.float32)
    proj[:, 0] = np.clip(kps["x"][pick] + rng.normal(0, 2.0, n), 0, width - 1)
    proj[:, 1] = np.clip(kps["y"][pick] + rng.normal(0, 2.0, n), 0, height - 1)
    depth = rng.uniform(1.5, 15, n).astype(np.float32)
    proj[:, 2] = proj[:, 0] - np.float32(EUROC_BF) / depth
    lvl = np.clip(kps["octave"][pick] + rng.integers(-1, 2, n), 0, nlevels - 1).astype(np.int32)
    bits = np.unpackbits(desc[pick], axis=1)
    for i in range(n):
        bits[i, rng.choice(256, int(rng.integers(0, 45)), replace=False)] ^= 1
    mdesc = np.packbits(bits, axis=1)
    ndup = int(dup_frac * n)
    a, b = rng.choice(n, ndup, replace=False), rng.choice(n, ndup, replace=False)
    mdesc[b], proj[b], lvl[b] = mdesc[a], proj[a], lvl[a]
    return dict(track_in_view=(rng.random(n) > 0.1).astype(np.uint8), is_bad=(rng.random(n) < bad_frac).astype(np.uint8),
                observed=(rng.random(n) > unobserved_frac).astype(np.uint8), track_proj=proj,
                track_view_cos=rng.choice(np.array([0.999, 0.99], np.float32), n), track_depth=depth,
                track_level=lvl, desc=mdesc)


def pose_opt_batch(n_frames: int = 64, n_points: int = 600, stereo_frac: float = 0.5, outlier_frac: float = 0.08,
                   seed: int = 41, width: int = 752, height: int = 480, nlevels: int = 8, rot_err: float = 0.01,
                   trans_err: float = 0.03, points_per_frame=None):
    """Tracking frames for Optimizer::PoseOptimization: per frame a true pose, ~n_points matched map
    points 1.5-12 m in front, observations at octave U{0..7} with N(0, 1)*scale pixel noise, stereo
    u_right for `stereo_frac` of them, `outlier_frac` gross outliers (+-15..60 px), and the initial
    pose (the motion model's prediction) off by ~rot_err rad / trans_err m.  EuRoC intrinsics.
    Returns (frames POSE_FRAME_DTYPE, edges POSE_EDGE_DTYPE, true poses [n, 7])."""
    from ._lib import POSE_EDGE_DTYPE, POSE_FRAME_DTYPE
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = EUROC_K
    scale, sigma2 = scale_tables(nlevels)
    inv_sigma2 = (np.float32(1.0) / sigma2).astype(np.float32)
    frames = np.zeros(n_frames, POSE_FRAME_DTYPE)
    all_edges = []
    truth = np.zeros((n_frames, 7))
    for f in range(n_frames):
        yaw, pitch = rng.uniform(-0.3, 0.3), rng.uniform(-0.1, 0.1)
        Rcw = _small_rot(rng, 0.05) @ np.array([[np.cos(yaw), 0, -np.sin(yaw)], [0, 1, 0], [np.sin(yaw), 0, np.cos(yaw)]])
        Rcw = np.array([[1, 0, 0], [0, np.cos(pitch), -np.sin(pitch)], [0, np.sin(pitch), np.cos(pitch)]]) @ Rcw
        tcw = rng.normal(0, 1.0, 3)
        truth[f, :3], truth[f, 3:] = tcw, rot_to_quat(Rcw)
        npf = n_points if points_per_frame is None else int(points_per_frame[f])
        e0 = len(all_edges)
        while len(all_edges) - e0 < npf:
            z = rng.uniform(1.5, 12.0)
            u, v = rng.uniform(20, width - 20), rng.uniform(20, height - 20)
            Xc = np.array([(u - cx) * z / fx, (v - cy) * z / fy, z])
            Xw = Rcw.T @ (Xc - tcw)
            octv = int(rng.integers(0, nlevels))
            sc = float(scale[octv])
            uo, vo = u + rng.normal(0, 1.0) * sc, v + rng.normal(0, 1.0) * sc
            if rng.random() < outlier_frac:
                uo += rng.choice([-1, 1]) * rng.uniform(15, 60)
                vo += rng.choice([-1, 1]) * rng.uniform(15, 60)
            st = rng.random() < stereo_frac
            ur = uo - EUROC_BF / z + rng.normal(0, 1.0) * sc if st else -1.0
            all_edges.append((Xw, (uo, vo, ur if st else 0.0), inv_sigma2[octv], int(st)))
        Rp = _small_rot(rng, rot_err) @ Rcw
        frames[f]["pose"][:3] = tcw + rng.normal(0, trans_err, 3)
        frames[f]["pose"][3:] = rot_to_quat(Rp)
        frames[f]["cam"] = (fx, fy, cx, cy, EUROC_BF)
        frames[f]["edge_begin"] = e0
        frames[f]["n_edges"] = npf
    edges = np.zeros(len(all_edges), POSE_EDGE_DTYPE)
    for i, (xw, obs, info, st) in enumerate(all_edges):
        edges[i]["xw"], edges[i]["obs"], edges[i]["inv_sigma2"], edges[i]["stereo"] = xw, obs, info, st
    return frames, edges, truth


def tracking_chain_scene(n_points: int = 1800, seed: int = 81, width: int = 752, height: int = 480,
                         stereo: bool = True, clutter: int = 300, tracked_frac: float = 0.7, outlier_frac: float = 0.06,
                         unobserved_frac: float = 0.1, bad_frac: float = 0.02, nlevels: int = 8,
                         pred_rot: float = 0.004, pred_trans: float = 0.02, step: float = 0.05):
    """One frame of Tracking::TrackWithMotionModel -> TrackLocalMap: a map of points (position,
    descriptor, normal, mfMinDistance / mfMaxDistance from the octave of their reference observation,
    observed / bad flags), the last frame (pose 0) holding `tracked_frac` of the points it sees (a few of
    them at positions off by ~0.1 m: PoseOptimization's outliers), the current frame at the true pose 1
    (noisy keypoints at octave +-1, perturbed descriptors, stereo u_right for 60 %, clutter) and the
    motion model's prediction of its pose, off the truth by ~pred_rot rad / pred_trans m.  The local
    map is every point; last_row[j] names the last frame's keypoint that holds point j (-1: none).
    Returns dict(cur=Frame kwargs, last=Frame kwargs with map_points, local=dict of local map arrays,
    pose7_pred, pose7_true, level_sigma2)."""
    from ._lib import KEYPOINT_DTYPE
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = EUROC_K
    scale, sigma2 = scale_tables(nlevels)
    P = np.stack([rng.uniform(-4, 4, n_points), rng.uniform(-2.5, 2.5, n_points), rng.uniform(2, 12, n_points)], 1)
    base = rng.integers(0, 256, (n_points, 32), dtype=np.uint8)
    ang = rng.uniform(0, 360, n_points)
    octv = rng.integers(0, nlevels, n_points)
    R0, t0 = np.eye(3), np.zeros(3)
    R1 = _rot_yaw_pitch(np.deg2rad(0.6), np.deg2rad(0.2))
    C1 = np.array([0.02, -0.005, step])
    t1 = -R1 @ C1

    def frame(R, t, noise, flips, oct_jitter):
        Xc = P @ R.T + t
        z = Xc[:, 2]
        u = fx * Xc[:, 0] / z + cx
        v = fy * Xc[:, 1] / z + cy
        vis = np.flatnonzero((z > 0.3) & (u >= 0) & (u < width) & (v >= 0) & (v < height))
        nv = len(vis)
        kps = np.zeros(nv + clutter, KEYPOINT_DTYPE)
        o = np.clip(octv[vis] + (rng.integers(-1, 2, nv) if oct_jitter else 0), 0, nlevels - 1)
        kps["octave"][:nv] = o
        kps["x"][:nv] = np.clip(u[vis] + rng.normal(0, noise, nv) * scale[o], 0, width - 1)
        kps["y"][:nv] = np.clip(v[vis] + rng.normal(0, noise, nv) * scale[o], 0, height - 1)
        kps["angle"][:nv] = np.mod(ang[vis] + rng.normal(0, 3, nv), 360)
        kps["x"][nv:] = rng.uniform(0, width - 1, clutter)
        kps["y"][nv:] = rng.uniform(0, height - 1, clutter)
        kps["octave"][nv:] = rng.integers(0, nlevels, clutter)
        kps["angle"][nv:] = rng.uniform(0, 360, clutter)
        kps["size"] = 31 * scale[kps["octave"]]
        kps["response"] = rng.uniform(5, 100, nv + clutter)
        kps["class_id"] = -1
        bits = np.unpackbits(base[vis], axis=1)
        for i in range(nv):
            bits[i, rng.choice(256, int(rng.integers(0, flips)), replace=False)] ^= 1
        desc = np.concatenate([np.packbits(bits, axis=1), rng.integers(0, 256, (clutter, 32), dtype=np.uint8)])
        ur = np.full(nv + clutter, -1.0, np.float32)
        if stereo:
            st = rng.random(nv) < 0.6
            ur[:nv][st] = (kps["x"][:nv][st] - EUROC_BF / z[vis][st] + rng.normal(0, 0.5, st.sum())).astype(np.float32)
        perm = rng.permutation(nv + clutter)
        ids = np.concatenate([vis, np.full(clutter, -1)])[perm]
        return kps[perm], desc[perm], ur[perm], ids

    lk, ld, lur, lids = frame(R0, t0, 0.3, 12, False)
    ck, cd, cur_ur, _ = frame(R1, t1, 0.5, 30, True)
    # map point positions (the map's estimate): small noise, a few gross errors
    Pm = (P + rng.normal(0, 0.01, P.shape)).astype(np.float32)
    gross = rng.random(n_points) < outlier_frac
    Pm[gross] += rng.normal(0, 0.1, (int(gross.sum()), 3)).astype(np.float32)
    observed = (rng.random(n_points) > unobserved_frac).astype(np.uint8)
    has = lids >= 0
    valid = has & (rng.random(len(lids)) < tracked_frac)
    xyz = np.zeros((len(lids), 3), np.float32)
    mdesc = np.zeros((len(lids), 32), np.uint8)
    obs_rows = np.zeros(len(lids), np.uint8)
    xyz[has], mdesc[has], obs_rows[has] = Pm[lids[has]], base[lids[has]], observed[lids[has]]
    last_row = np.full(n_points, -1, np.int32)
    last_row[lids[valid]] = np.flatnonzero(valid)
    # MapPoint::UpdateNormalAndDepth from the pose-0 observation (src/MapPoint.cc:619-668)
    d0 = np.linalg.norm(Pm, axis=1)
    normal = (Pm / d0[:, None]).astype(np.float32)
    max_dist = (d0 * scale[octv]).astype(np.float32)
    min_dist = (max_dist / scale[nlevels - 1]).astype(np.float32)
    # the motion model's prediction, as the float SE3 a Frame holds (Sophus SE3f)
    Rp = _small_rot(rng, pred_rot) @ R1
    tp = t1 + rng.normal(0, pred_trans, 3)
    pose7_pred = np.concatenate([tp.astype(np.float32), rot_to_quat(Rp).astype(np.float32)]).astype(np.float64)
    Tp = np.concatenate([quat_to_rot(pose7_pred[3:]), pose7_pred[:3, None]], 1).astype(np.float32)
    common = dict(camera=EUROC_K, scale_factors=scale, width=width, height=height, bf=EUROC_BF if stereo else 0.0)
    last = dict(keys_un=lk, descriptors=ld, Tcw=np.concatenate([R0, t0[:, None]], 1).astype(np.float32),
                u_right=lur if stereo else None,
                map_points=dict(valid=valid.astype(np.uint8), observed=obs_rows, xyz=xyz, desc=mdesc), **common)
    cur = dict(keys_un=ck, descriptors=cd, Tcw=Tp, u_right=cur_ur if stereo else None, **common)
    local = dict(pos=Pm, normal=normal, min_dist=min_dist, max_dist=max_dist, desc=base.copy(), observed=observed,
                 is_bad=((rng.random(n_points) < bad_frac) & (last_row < 0)).astype(np.uint8), last_row=last_row)
    truth = np.concatenate([t1, rot_to_quat(R1)])
    return dict(cur=cur, last=last, local=local, pose7_pred=pose7_pred, pose7_true=truth, level_sigma2=sigma2)


def dbow_vocabulary(k: int = 10, L: int = 4, seed: int = 11, flip: float = 0.2, leaf_early: float = 0.05,
                    stop_frac: float = 0.02, weighting: int = 0, scoring: int = 0, kmin=None):
    """A DBoW2-shaped vocabulary tree (stand-in for ORBvoc.txt, absent: .MISSING_LARGE_BLOBS):
    breadth-first node ids (root 0), k children at the root and k-3..k below, children = the
    parent's descriptor with `flip` of its bits flipped (a coherent tree), a few nodes ending early
    as leaves (an unbalanced tree, like real vocabularies) and `stop_frac` stop words (weight 0).
    Built level by level (k=10, L=6 -- ORBvoc's shape, ~1.1M nodes -- takes seconds).  Returns the
    dict orb_vocabulary_view_t takes, plus `leaves` (node ids of the words)."""
    rng = np.random.default_rng(seed)
    desc_levels = [np.zeros((1, 32), np.uint8)]
    nkids = []            # per level: children count of each node of that level
    frontier = desc_levels[0]
    for depth in range(L):
        m = len(frontier)
        if depth == 0:
            kk = np.full(1, k)
        else:
            kk = rng.integers(max(2, k - 3) if kmin is None else kmin, k + 1, m)
            kk[rng.random(m) < leaf_early] = 0
        nkids.append(kk)
        parent = np.repeat(np.arange(m), kk)
        if depth == 0:
            child = rng.integers(0, 256, (len(parent), 32), dtype=np.uint8)
        else:
            bits = np.unpackbits(frontier[parent], axis=1) ^ (rng.random((len(parent), 256)) < flip)
            child = np.packbits(bits.astype(np.uint8), axis=1)
        desc_levels.append(child)
        frontier = child
    nkids.append(np.zeros(len(frontier), np.int64))
    counts = np.concatenate(nkids).astype(np.int64)
    n = len(counts)
    child_begin = np.zeros(n + 1, np.int64)
    child_begin[1:] = np.cumsum(counts)
    child_begin += 0
    # breadth-first numbering: node i's children are nodes 1 + child_begin[i] ...
    child_idx = np.arange(1, 1 + child_begin[-1], dtype=np.int32)
    desc = np.concatenate(desc_levels)
    assert len(desc) == n
    word_id = np.full(n, -1, np.int32)
    weight = np.zeros(n, np.float64)
    leaves = np.flatnonzero(counts == 0)
    leaves = leaves[leaves != 0]
    word_id[leaves] = np.arange(len(leaves), dtype=np.int32)
    weight[leaves] = np.where(rng.random(len(leaves)) < stop_frac, 0.0, rng.uniform(0.2, 6.0, len(leaves)))
    return dict(k=k, L=L, weighting=weighting, scoring=scoring, child_begin=child_begin.astype(np.int32),
                child_idx=child_idx, desc=desc, word_id=word_id, weight=weight, leaves=leaves.astype(np.int32))


def bow_descriptors(voc: dict, n: int, seed: int = 12, noise: float = 0.08):
    """Descriptors near random vocabulary words (leaf descriptor + `noise` bit flips), with some
    exact ties between siblings avoided by nothing: first-minimum rules are exercised."""
    rng = np.random.default_rng(seed)
    leaves = voc["leaves"]
    pick = voc["desc"][leaves[rng.integers(0, len(leaves), n)]]
    bits = np.unpackbits(pick, axis=1) ^ (rng.random((n, 256)) < noise)
    return np.packbits(bits.astype(np.uint8), axis=1)


def frustum_points(n: int = 3000, seed: int = 61, width: int = 752, height: int = 480, nlevels: int = 8):
    """Local map points around a tracking frame for Frame::isInFrustum: most in front and inside the
    image, some behind the camera, outside the image, outside their scale-invariance distance range
    or seen at a grazing angle.  mfMaxDistance / mfMinDistance as MapPoint::UpdateNormalAndDepth sets
    them (dist * levelScaleFactor, / scaleFactors[nLevels - 1]).  Returns (Tcw 3x4, Ow, pos, normal,
    min_dist, max_dist), float32."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = EUROC_K
    scale, _ = scale_tables(nlevels)
    Rcw = _rot_yaw_pitch(rng.uniform(-0.5, 0.5), rng.uniform(-0.2, 0.2))
    tcw = rng.normal(0, 1.0, 3)
    Ow = -Rcw.T @ tcw
    z = rng.uniform(0.5, 20.0, n)
    u = rng.uniform(-150, width + 150, n)
    v = rng.uniform(-100, height + 100, n)
    Xc = np.stack([(u - cx) * z / fx, (v - cy) * z / fy, z], 1)
    behind = rng.random(n) < 0.05
    Xc[behind, 2] *= -1
    P = (Xc - tcw) @ Rcw  # Rcw^T (Xc - t)
    view = P - Ow
    d = np.linalg.norm(view, axis=1)
    nrm = view / d[:, None]
    tilt = rng.random(n) < 0.15  # the reference keyframes saw the point from elsewhere
    nrm[tilt] = nrm[tilt] + rng.normal(0, 0.8, (int(tilt.sum()), 3))
    nrm /= np.linalg.norm(nrm, axis=1)[:, None]
    ref = d * rng.uniform(0.6, 1.6, n)  # distance from the reference keyframe
    lvl = rng.integers(0, nlevels, n)
    max_dist = ref * scale[lvl]
    min_dist = max_dist / scale[nlevels - 1]
    Tcw = np.concatenate([Rcw, tcw[:, None]], 1)
    f32 = lambda a: np.ascontiguousarray(a, np.float32)
    return f32(Tcw), f32(Ow), f32(P), f32(nrm), f32(min_dist), f32(max_dist)
