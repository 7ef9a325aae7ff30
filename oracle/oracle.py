"""ctypes binding of the CPU oracle (oracle/_build/liborb_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, and only as the checker / the timed CPU baseline -- never by the product package.
"""
from __future__ import annotations

import ctypes
import pathlib
import subprocess

import numpy as np

ORACLE_DIR = pathlib.Path(__file__).resolve().parent
LIB_PATH = ORACLE_DIR / "_build" / "liborb_oracle.so"

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])

_vp, _i, _f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
_PROTOS = {
    "oracle_node_sort": (None, [_vp, _vp, _i, _vp]),
    "oracle_orb_create": (_vp, [_i, _f, _i, _i, _i]),
    "oracle_orb_destroy": (None, [_vp]),
    "oracle_orb_params": (None, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "oracle_orb_extract": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp, _vp, _i, ctypes.POINTER(_i)]),
    "oracle_orb_level_dims": (None, [_vp, _i, ctypes.POINTER(_i), ctypes.POINTER(_i), ctypes.POINTER(_i),
                                     ctypes.POINTER(_i)]),
    "oracle_orb_level_copy": (None, [_vp, _i, _vp]),
    "oracle_orb_level_candidates": (_i, [_vp, _i, _vp, _i]),
    "oracle_orb_level_cell_thresholds": (_i, [_vp, _i, _vp, _i]),
    "oracle_orb_level_keys": (_i, [_vp, _i, _vp, _i]),
    "oracle_resize_linear_u8": (None, [_vp, _i, _i, _i, _vp, _i, _i, _i]),
    "oracle_fast9": (_i, [_vp, _i, _i, _i, _i, _vp, _i]),
    "oracle_distribute": (_i, [_vp, _i, _i, _i, _i, _i, _i, _vp, _i]),
    "oracle_fast_atan2": (_f, [_f, _f]),
    "oracle_gaussian_blur": (None, [_vp, _i, _i, _i, _vp]),
    "oracle_descriptor_distance": (_i, [_vp, _vp]),
    "oracle_compute_distinctive_descriptors": (None, [_vp, _vp, _i, _vp]),
    "oracle_hamming_knn2": (None, [_vp, _i, _vp, _i, _vp, _vp, _vp]),
    "oracle_search_for_triangulation": (_i, [_vp, _vp, _vp, _i, _i, _i, _vp]),
    "oracle_local_ba": (_i, [_vp, _vp, _vp, _vp, _vp]),
    "oracle_search_by_projection_frame": (_i, [_vp, _vp, _f, _i, _i, _vp]),
    "oracle_search_by_projection_local": (_i, [_vp, _vp, _vp, _f, _i, _f, _f, _vp]),
    "oracle_pose_optimization": (_i, [_i, _vp, _vp, _vp, _vp, _vp]),
    "oracle_is_in_frustum": (_i, [_vp, _i, _vp, _vp, _vp, _vp, _f, _vp, _vp, _vp, _vp, _vp]),
    "oracle_bow_transform": (_i, [_vp, _vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "oracle_undistort_keypoints": (None, [_vp, _i, _vp, _vp, _i, _vp]),
    "oracle_pose7_to_frame": (None, [_vp, _vp, _vp]),
    "oracle_pose7_float_roundtrip": (None, [_vp, _vp]),
    "oracle_compute_stereo_matches": (_i, [_vp, _i, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _i, _vp, _vp, _f, _f,
                                           _vp, _vp]),
}

_LIB = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)


def load() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            build()
        lib = ctypes.CDLL(str(LIB_PATH))
        for name, (res, args) in _PROTOS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = lib
    return _LIB


def node_sort(counts, ulx):
    """libstdc++ std::sort with compareNodes (src/ORBextractor.cc:676-697, 950) of (count, UL.x) records:
    the record indices in sorted order."""
    import numpy as np
    c = np.ascontiguousarray(counts, np.int32)
    x = np.ascontiguousarray(ulx, np.int32)
    out = np.zeros(len(c), np.int32)
    load().oracle_node_sort(c.ctypes.data, x.ctypes.data, len(c), out.ctypes.data)
    return out


class OracleExtractor:
    """CPU restatement of ORB_SLAM3::ORBextractor (oracle/orb_extractor_oracle.cpp)."""

    def __init__(self, nfeatures=1000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7):
        self.lib = load()
        self.nlevels = nlevels
        self.h = ctypes.c_void_p(self.lib.oracle_orb_create(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST))
        self.nfeatures = nfeatures

    def __del__(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.lib.oracle_orb_destroy(self.h)
            self.h = None

    def params(self):
        n = self.nlevels
        arrs = [np.zeros(n, np.float32) for _ in range(4)]
        per = np.zeros(n, np.int32)
        umax = np.zeros(16, np.int32)
        self.lib.oracle_orb_params(self.h, *[a.ctypes.data for a in arrs], per.ctypes.data, umax.ctypes.data)
        return {"scale": arrs[0], "inv_scale": arrs[1], "sigma2": arrs[2], "inv_sigma2": arrs[3],
                "per_level": per, "umax": umax}

    def __call__(self, image: np.ndarray, lapping=(0, 0)):
        img = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = img.shape
        cap = 4 * self.nfeatures + 256
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = ctypes.c_int()
        rc = self.lib.oracle_orb_extract(self.h, img.ctypes.data, w, h, w, int(lapping[0]), int(lapping[1]),
                                         kps.ctypes.data, desc.ctypes.data, cap, ctypes.byref(n))
        if rc < -1:
            raise RuntimeError(f"oracle extract failed {rc}")
        k = n.value
        return kps[:k].copy(), desc[:k].copy(), rc

    def level_padded(self, level: int) -> np.ndarray:
        w, h, pw, ph = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self.lib.oracle_orb_level_dims(self.h, level, ctypes.byref(w), ctypes.byref(h), ctypes.byref(pw),
                                       ctypes.byref(ph))
        out = np.zeros((ph.value, pw.value), np.uint8)
        self.lib.oracle_orb_level_copy(self.h, level, out.ctypes.data)
        return out

    def level_candidates(self, level: int) -> np.ndarray:
        n = self.lib.oracle_orb_level_candidates(self.h, level, None, 0)
        out = np.zeros(n, KEYPOINT_DTYPE)
        self.lib.oracle_orb_level_candidates(self.h, level, out.ctypes.data, n)
        return out

    def level_cell_thresholds(self, level: int) -> np.ndarray:
        n = self.lib.oracle_orb_level_cell_thresholds(self.h, level, None, 0)
        out = np.zeros(n, np.int32)
        self.lib.oracle_orb_level_cell_thresholds(self.h, level, out.ctypes.data, n)
        return out

    def level_keys(self, level: int) -> np.ndarray:
        n = self.lib.oracle_orb_level_keys(self.h, level, None, 0)
        out = np.zeros(n, KEYPOINT_DTYPE)
        self.lib.oracle_orb_level_keys(self.h, level, out.ctypes.data, n)
        return out


def fast9(window: np.ndarray, threshold: int) -> np.ndarray:
    lib = load()
    win = np.ascontiguousarray(window, dtype=np.uint8)
    h, w = win.shape
    cap = w * h
    out = np.zeros(cap, KEYPOINT_DTYPE)
    n = lib.oracle_fast9(win.ctypes.data, w, w, h, threshold, out.ctypes.data, cap)
    return out[:n].copy()


def distribute(cand: np.ndarray, min_x: int, max_x: int, min_y: int, max_y: int, n_features: int) -> np.ndarray:
    lib = load()
    c = np.ascontiguousarray(cand, dtype=KEYPOINT_DTYPE)
    cap = len(c) + 8
    out = np.zeros(cap, KEYPOINT_DTYPE)
    m = lib.oracle_distribute(c.ctypes.data, len(c), min_x, max_x, min_y, max_y, n_features, out.ctypes.data, cap)
    return out[:m].copy()


def resize_linear(src: np.ndarray, dw: int, dh: int) -> np.ndarray:
    lib = load()
    s = np.ascontiguousarray(src, dtype=np.uint8)
    out = np.zeros((dh, dw), np.uint8)
    lib.oracle_resize_linear_u8(s.ctypes.data, s.shape[1], s.shape[1], s.shape[0], out.ctypes.data, dw, dw, dh)
    return out


def gaussian_blur(view: np.ndarray) -> np.ndarray:
    lib = load()
    v = np.ascontiguousarray(view, dtype=np.uint8)
    out = np.zeros_like(v)
    lib.oracle_gaussian_blur(v.ctypes.data, v.shape[1], v.shape[1], v.shape[0], out.ctypes.data)
    return out


def fast_atan2(y: float, x: float) -> float:
    return float(load().oracle_fast_atan2(y, x))


def descriptor_distance(a: np.ndarray, b: np.ndarray) -> int:
    a = np.ascontiguousarray(a, dtype=np.uint8)
    b = np.ascontiguousarray(b, dtype=np.uint8)
    return load().oracle_descriptor_distance(a.ctypes.data, b.ctypes.data)


def hamming_knn2(query, train):
    """Oracle best / second-best Hamming scan (index order, first index on ties); 257 = none."""
    q = np.ascontiguousarray(query, dtype=np.uint8).reshape(-1, 32)
    t = np.ascontiguousarray(train, dtype=np.uint8).reshape(-1, 32)
    n = len(q)
    out = [np.zeros(max(n, 1), np.int32) for _ in range(3)]
    load().oracle_hamming_knn2(q.ctypes.data, n, t.ctypes.data, len(t), *(o.ctypes.data for o in out))
    return tuple(o[:n] for o in out)


def compute_distinctive_descriptors(desc, offsets):
    """Oracle MapPoint::ComputeDistinctiveDescriptors per point (rows offsets[p]..offsets[p+1] of desc):
    returns best[p] (-1 for an empty point)."""
    desc = np.ascontiguousarray(desc, dtype=np.uint8).reshape(-1, 32)
    offsets = np.ascontiguousarray(offsets, dtype=np.int32)
    n = len(offsets) - 1
    best = np.zeros(max(n, 1), np.int32)
    load().oracle_compute_distinctive_descriptors(desc.ctypes.data, offsets.ctypes.data, n, best.ctypes.data)
    return best[:n]


def search_for_triangulation(kf1, kf2, geom, only_stereo: bool, coarse: bool, check_ori: bool):
    """Oracle SearchForTriangulation for one pair.  kf1/kf2: objects with .view() returning an
    orb_kf_view_t ctypes struct (the product's KeyFrame, used here as plain data); geom: the
    orb_kf_pair_geom_t struct.  Returns (nmatches, vMatches12 int32[N1])."""
    m = np.full(max(kf1.N, 1), -1, np.int32)
    n = load().oracle_search_for_triangulation(ctypes.byref(kf1.view()), ctypes.byref(kf2.view()),
                                               ctypes.byref(geom), int(only_stereo), int(coarse), int(check_ori),
                                               m.ctypes.data)
    return n, m[:kf1.N]


class _BaProblem(ctypes.Structure):
    _fields_ = [("n_poses", ctypes.c_int32), ("n_points", ctypes.c_int32), ("n_edges", ctypes.c_int32),
                ("pose", _vp), ("pose_id", _vp), ("pose_fixed", _vp), ("pose_camera", _vp), ("point", _vp),
                ("point_id", _vp), ("edges", _vp)]


class _BaOptions(ctypes.Structure):
    _fields_ = [("iterations", ctypes.c_int32), ("user_lambda_init", ctypes.c_double), ("stop_flag", _vp), ("stop_flag_bool", _vp)]


class _BaResult(ctypes.Structure):
    _fields_ = [("iterations", ctypes.c_int32), ("trials", ctypes.c_int32), ("terminated", ctypes.c_int32),
                ("stopped", ctypes.c_int32), ("initial_chi2", ctypes.c_double), ("final_chi2", ctypes.c_double),
                ("lambda_", ctypes.c_double)]


def local_ba(prob: dict, iterations: int = 10, user_lambda_init: float = 0.0, stop_flag=None):
    """Oracle g2o LM/Schur solve of a flattened LocalBundleAdjustment graph (see oracle/orb_ba_oracle.cpp).
    prob: dict of arrays (pose [n,7] t+q, pose_id, pose_fixed, pose_camera (5 x f4 records), point [m,3],
    point_id, edges (40-byte records)).  Returns (pose, point, edge_chi2, depth_ok, result dict)."""
    pose = np.ascontiguousarray(prob["pose"], dtype=np.float64).copy()
    point = np.ascontiguousarray(prob["point"], dtype=np.float64).copy()
    pid = np.ascontiguousarray(prob["pose_id"], dtype=np.int64)
    pfx = np.ascontiguousarray(prob["pose_fixed"], dtype=np.uint8)
    cam = np.ascontiguousarray(prob["pose_camera"])
    qid = np.ascontiguousarray(prob["point_id"], dtype=np.int64)
    edges = np.ascontiguousarray(prob["edges"])
    assert cam.dtype.itemsize == 20 and edges.dtype.itemsize == 40
    s = _BaProblem(len(pose), len(point), len(edges), pose.ctypes.data, pid.ctypes.data, pfx.ctypes.data,
                   cam.ctypes.data, point.ctypes.data, qid.ctypes.data, edges.ctypes.data)
    flag = None if stop_flag is None else np.ascontiguousarray(stop_flag, dtype=np.int32)
    o = _BaOptions(int(iterations), float(user_lambda_init), None if flag is None else flag.ctypes.data)
    chi2 = np.zeros(len(edges))
    depth = np.zeros(len(edges), np.uint8)
    r = _BaResult()
    load().oracle_local_ba(ctypes.byref(s), ctypes.byref(o), chi2.ctypes.data, depth.ctypes.data, ctypes.byref(r))
    res = {"iterations": r.iterations, "trials": r.trials, "terminated": r.terminated, "stopped": r.stopped,
           "initial_chi2": r.initial_chi2, "final_chi2": r.final_chi2, "lambda": r.lambda_}
    return pose, point, chi2, depth.astype(bool), res


def search_by_projection_frame(cur, last, th: float, mono: bool, check_ori: bool):
    """Oracle SearchByProjection(CurrentFrame, LastFrame, th, bMono).  cur/last: objects with .view() /
    .last_points() returning the orb_frame_view_t / orb_last_points_t ctypes structs (plain data)."""
    m = np.full(max(cur.N, 1), -1, np.int32)
    n = load().oracle_search_by_projection_frame(ctypes.byref(cur.view()), ctypes.byref(last.last_points()),
                                                 float(th), int(mono), int(check_ori), m.ctypes.data)
    return n, m[:cur.N]


def search_by_projection_local(frame, points, th: float, far: bool, th_far: float, nnratio: float, frame_taken=None):
    """Oracle SearchByProjection(Frame, vector<MapPoint*>, th, bFarPoints, thFarPoints)."""
    m = np.full(max(frame.N, 1), -1, np.int32)
    tk = None if frame_taken is None else np.ascontiguousarray(frame_taken, dtype=np.uint8)
    n = load().oracle_search_by_projection_local(ctypes.byref(frame.view()), None if tk is None else tk.ctypes.data,
                                                 ctypes.byref(points.view()), float(th), int(far), float(th_far),
                                                 float(nnratio), m.ctypes.data)
    return n, m[:frame.N]


def compute_stereo_matches(kps_l, desc_l, kps_r, desc_r, planes_l, planes_r, scale, inv_scale, bf, b):
    """Frame::ComputeStereoMatches (oracle/orb_stereo_oracle.cpp).  planes_*: per level, the padded
    plane ((h+38) x (w+38) uint8) of the left / right extractor.  Returns (mvuRight, mvDepth, kept)."""
    lib = load()
    kl = np.ascontiguousarray(kps_l, KEYPOINT_DTYPE)
    kr = np.ascontiguousarray(kps_r, KEYPOINT_DTYPE)
    dl = np.ascontiguousarray(desc_l, np.uint8).reshape(-1, 32)
    dr = np.ascontiguousarray(desc_r, np.uint8).reshape(-1, 32)
    n = len(planes_l)
    pl = [np.ascontiguousarray(p, np.uint8) for p in planes_l]
    pr = [np.ascontiguousarray(p, np.uint8) for p in planes_r]
    ptr_l = (ctypes.c_void_p * n)(*[p.ctypes.data for p in pl])
    ptr_r = (ctypes.c_void_p * n)(*[p.ctypes.data for p in pr])
    pitch = np.array([p.shape[1] for p in pl], np.int32)
    w = pitch - 38
    h = np.array([p.shape[0] - 38 for p in pl], np.int32)
    sc = np.ascontiguousarray(scale, np.float32)
    isc = np.ascontiguousarray(inv_scale, np.float32)
    ur = np.zeros(len(kl), np.float32)
    dp = np.zeros(len(kl), np.float32)
    kept = lib.oracle_compute_stereo_matches(kl.ctypes.data, len(kl), dl.ctypes.data, kr.ctypes.data, len(kr),
                                             dr.ctypes.data, ptr_l, ptr_r, pitch.ctypes.data, w.ctypes.data,
                                             h.ctypes.data, n, sc.ctypes.data, isc.ctypes.data, float(bf), float(b),
                                             ur.ctypes.data, dp.ctypes.data)
    return ur, dp, kept


def pose_optimization(frames, edges):
    """Oracle Optimizer::PoseOptimization over a batch (oracle/orb_pose_oracle.cpp).  frames / edges:
    orb_pose_frame_t / orb_pose_edge_t records (88 / 56 bytes).  Returns (poses [n, 7], outlier
    flags per edge (bool), inliers per frame)."""
    fr = np.ascontiguousarray(frames)
    ed = np.ascontiguousarray(edges)
    assert fr.dtype.itemsize == 88 and ed.dtype.itemsize == 56
    poses = np.zeros((len(fr), 7))
    outl = np.zeros(max(len(ed), 1), np.uint8)
    inl = np.zeros(max(len(fr), 1), np.int32)
    load().oracle_pose_optimization(len(fr), fr.ctypes.data, ed.ctypes.data, poses.ctypes.data, outl.ctypes.data,
                                    inl.ctypes.data)
    return poses, outl[:len(ed)].astype(bool), inl[:len(fr)]


def bow_transform(voc: dict, desc, levelsup: int = 4):
    """Oracle TemplatedVocabulary::transform (oracle/orb_bow_oracle.cpp).  Returns (bow: {word: value},
    feat_vec: {node: [features]}) like the DBoW2 std::maps."""
    lib = load()

    class View(ctypes.Structure):  # orb_vocabulary_view_t (include/orbgpu.h)
        _fields_ = [("k", ctypes.c_int32), ("L", ctypes.c_int32), ("weighting", ctypes.c_int32),
                    ("scoring", ctypes.c_int32), ("n_nodes", ctypes.c_int32), ("child_begin", ctypes.c_void_p),
                    ("child_idx", ctypes.c_void_p), ("desc", ctypes.c_void_p), ("word_id", ctypes.c_void_p),
                    ("weight", ctypes.c_void_p)]
    keep = [np.ascontiguousarray(voc["child_begin"], np.int32), np.ascontiguousarray(voc["child_idx"], np.int32),
            np.ascontiguousarray(voc["desc"], np.uint8), np.ascontiguousarray(voc["word_id"], np.int32),
            np.ascontiguousarray(voc["weight"], np.float64)]
    view = View(int(voc["k"]), int(voc["L"]), int(voc.get("weighting", 0)), int(voc.get("scoring", 0)),
                len(keep[3]), *[a.ctypes.data for a in keep])
    d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    n = len(d)
    m = max(n, 1)
    bw, bv = np.zeros(m, np.int32), np.zeros(m, np.float64)
    fn, fb, ff = np.zeros(m, np.int32), np.zeros(m + 1, np.int32), np.zeros(m, np.int32)
    nw, nn = np.zeros(1, np.int32), np.zeros(1, np.int32)
    lib.oracle_bow_transform(ctypes.addressof(view), d.ctypes.data, n, int(levelsup), bw.ctypes.data, bv.ctypes.data,
                             nw.ctypes.data, fn.ctypes.data, fb.ctypes.data, ff.ctypes.data, nn.ctypes.data)
    bow = {int(bw[i]): float(bv[i]) for i in range(int(nw[0]))}
    fv = {int(fn[j]): [int(x) for x in ff[fb[j]:fb[j + 1]]] for j in range(int(nn[0]))}
    return bow, fv


def is_in_frustum(frame, pos, normal, min_dist, max_dist, viewing_cos_limit=0.5):
    """Oracle Frame::isInFrustum (oracle/orb_frustum_oracle.cpp).  frame: an orb_frustum_frame_t
    ctypes structure.  Returns the same dict of tracking fields as the product's is_in_frustum."""
    P = np.ascontiguousarray(pos, np.float32).reshape(-1, 3)
    n = len(P)
    m = max(n, 1)
    out = dict(track_in_view=np.zeros(m, np.uint8), track_proj=np.zeros((m, 3), np.float32),
               track_depth=np.zeros(m, np.float32), track_level=np.zeros(m, np.int32),
               track_view_cos=np.zeros(m, np.float32))
    arrs = [np.ascontiguousarray(a, np.float32) for a in (normal, min_dist, max_dist)]
    load().oracle_is_in_frustum(ctypes.addressof(frame), n, P.ctypes.data, *[a.ctypes.data for a in arrs],
                                float(viewing_cos_limit), *[out[k].ctypes.data for k in ("track_in_view", "track_proj",
                                                                                           "track_depth", "track_level",
                                                                                           "track_view_cos")])
    return {k: v[:n] for k, v in out.items()}


def undistort_keypoints(kps, K, dist):
    """Frame::UndistortKeyPoints (src/Frame.cc:1003-1051): mvKeysUn from mvKeys with cv::undistortPoints
    (OpenCV 4.x, restated; parity unpinned).  K = (fx, fy, cx, cy), dist = mDistCoef (4 or 5 floats)."""
    k = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
    out = np.empty_like(k)
    Kf = np.ascontiguousarray(K, np.float32)
    d = np.ascontiguousarray(dist, np.float32)
    load().oracle_undistort_keypoints(k.ctypes.data, len(k), Kf.ctypes.data, d.ctypes.data, len(d), out.ctypes.data)
    return out


def pose7_to_frame(pose7):
    """Frame::SetPose(SE3f(q.cast<float>(), t.cast<float>())) after PoseOptimization: (Tcw 3x4 float32,
    Ow float32[3]) from the g2o SE3Quat vector (tx ty tz qx qy qz qw)."""
    p = np.ascontiguousarray(pose7, np.float64).reshape(7)
    T = np.zeros(12, np.float32)
    O = np.zeros(3, np.float32)
    load().oracle_pose7_to_frame(p.ctypes.data, T.ctypes.data, O.ctypes.data)
    return T.reshape(3, 4), O


def pose7_float_roundtrip(pose7):
    """The pose the next PoseOptimization starts from after Frame::SetPose (float cast, Sophus's
    quaternion normalisation, back to double)."""
    p = np.ascontiguousarray(pose7, np.float64).reshape(7)
    out = np.zeros(7, np.float64)
    load().oracle_pose7_float_roundtrip(p.ctypes.data, out.ctypes.data)
    return out
