"""CPU tests: pin the ORB oracle to the reference's own constants
and cross-check its OpenCV restatements against independent formulations."""
from __future__ import annotations

import json
import math
import pathlib

import numpy as np
import pytest

GOLDEN = pathlib.Path(__file__).resolve().parent / "golden"


def test_scale_tables_and_budget(oracle):
    p = oracle.OracleExtractor(1000, 1.2, 8, 20, 7).params()
    # mvScaleFactor as the reference computes it in float
    expect = [1.0, 1.2000000477, 1.4400000572, 1.7280001640, 2.0736002922, 2.4883203506, 2.9859845638,
              3.5831816196]
    np.testing.assert_allclose(p["scale"], np.float32(expect), rtol=0, atol=1e-7)
    np.testing.assert_array_equal(p["sigma2"], p["scale"] * p["scale"])
    np.testing.assert_array_equal(p["inv_scale"], np.float32(1.0) / p["scale"])
    assert list(p["per_level"]) == [217, 181, 151, 126, 105, 87, 73, 60]
    assert list(p["umax"]) == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
    # the disc has 749 pixels
    assert 31 + 2 * sum(2 * u + 1 for u in p["umax"][1:]) == 749


@pytest.mark.parametrize("nf,expect", [(1200, [261, 217, 181, 151, 126, 105, 87, 72]),
                                       (5000, [1086, 905, 754, 628, 524, 436, 364, 303])])
def test_feature_budget_other_configs(oracle, nf, expect):
    assert list(oracle.OracleExtractor(nf, 1.2, 8, 20, 7).params()["per_level"]) == expect


@pytest.mark.parametrize("w,h,sizes", [
    (640, 480, [(640, 480), (533, 400), (444, 333), (370, 278), (309, 231), (257, 193), (214, 161), (179, 134)]),
])
def test_level_sizes(oracle, synth, w, h, sizes):
    ex = oracle.OracleExtractor()
    kps, desc, rc = ex(synth.polygon_frame(w, h, seed=3))
    for l, (lw, lh) in enumerate(sizes):
        pad = ex.level_padded(l)
        assert pad.shape == (lh + 38, lw + 38)
    # keypoint size field = (int)(31 * scale) per level
    by_level = {int(k["octave"]): float(k["size"]) for k in kps}
    for l, s in zip(range(8), [31, 37, 44, 53, 64, 77, 92, 111]):
        if l in by_level:
            assert by_level[l] == s


def test_pattern_table_matches_reference_checksum(pkg):
    from orbslam3_amd import _lib
    txt = (_lib.PKG_DIR / "csrc" / "orb_pattern31.inc").read_text()
    vals = [int(v) for line in txt.splitlines() if not line.startswith("//") for v in line.split(",") if v.strip()]
    g = json.loads((GOLDEN / "pattern31.json").read_text())
    assert len(vals) == g["n"] == 1024
    assert sum(vals) == g["sum"] and sum(abs(v) for v in vals) == g["sum_abs"]
    assert sum((i + 1) * v for i, v in enumerate(vals)) == g["weighted"]
    assert vals[:8] == g["first8"] and vals[-8:] == g["last8"]
    assert max(abs(v) for v in vals) == g["max_abs"] == 13


def test_fast_atan2_accuracy(oracle):
    rng = np.random.default_rng(0)
    for _ in range(2000):
        y, x = (float(v) for v in rng.integers(-3_000_000, 3_000_000, size=2))
        a = oracle.fast_atan2(y, x)
        ref = math.degrees(math.atan2(y, x)) % 360.0
        assert 0.0 <= a < 360.0 or (a == 360.0 and y < 0 and abs(y) < 1)
        diff = abs(a - ref)
        assert min(diff, 360 - diff) < 0.3  # OpenCV documents ~0.3 degree accuracy
    assert oracle.fast_atan2(0.0, 0.0) == 0.0
    assert oracle.fast_atan2(5.0, 0.0) == 90.0


def _fast_score_np(win: np.ndarray) -> np.ndarray:
    """Threshold-independent FAST-9/16 score: max over 16 arcs x 2 polarities of the arc minimum of
    |I(p) - I(q)|, minus 1 (the formulation the HIP kernel uses)."""
    circle = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
              (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]
    h, w = win.shape
    v = win[3:h - 3, 3:w - 3].astype(np.int32)
    d = np.stack([v - win[3 + dy:h - 3 + dy, 3 + dx:w - 3 + dx].astype(np.int32) for dx, dy in circle])
    best_dark = np.full(v.shape, -1000, np.int32)
    best_bright = np.full(v.shape, 1000, np.int32)
    for k in range(16):
        arc = d[[(k + i) % 16 for i in range(9)]]
        best_dark = np.maximum(best_dark, arc.min(axis=0))
        best_bright = np.minimum(best_bright, arc.max(axis=0))
    return np.maximum(best_dark, -best_bright) - 1


def _fast_nms_np(win: np.ndarray, t: int):
    """Kernel formulation of cv::FAST(nonmax=true): keep p iff score(p) >= t and score(p) exceeds the
    raw (un-thresholded, clamped to >= 0) score of every neighbour inside the detectable region."""
    s = np.clip(_fast_score_np(win), 0, 255)
    hs, ws = s.shape
    pad = np.zeros((hs + 2, ws + 2), np.int32)
    pad[1:-1, 1:-1] = s
    out = []
    for y in range(hs):
        for x in range(ws):
            sv = s[y, x]
            if sv < t:
                continue
            nb = pad[y:y + 3, x:x + 3].copy()
            nb[1, 1] = -1
            if sv > nb.max():
                out.append((x + 3, y + 3, int(sv)))
    return out


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("t", [7, 20])
def test_fast_oracle_matches_threshold_free_score(oracle, synth, seed, t):
    rng = np.random.default_rng(seed)
    if seed % 2:
        win = synth.polygon_frame(48, 44, seed=seed, n_shapes=12)
    else:
        win = rng.integers(0, 256, size=(41, 43), dtype=np.uint8)
    got = [(int(k["x"]), int(k["y"]), int(k["response"])) for k in oracle.fast9(win, t)]
    assert got == _fast_nms_np(win, t)


def test_descriptor_distance(oracle):
    rng = np.random.default_rng(5)
    for _ in range(200):
        a = rng.integers(0, 256, 32, dtype=np.uint8)
        b = rng.integers(0, 256, 32, dtype=np.uint8)
        assert oracle.descriptor_distance(a, b) == int(np.unpackbits(a ^ b).sum())
    z = np.zeros(32, np.uint8)
    assert oracle.descriptor_distance(z, z) == 0
    assert oracle.descriptor_distance(z, np.full(32, 255, np.uint8)) == 256


def test_distribute_keeps_everything_when_budget_is_large(oracle):
    rng = np.random.default_rng(7)
    pts = set()
    while len(pts) < 300:
        pts.add((int(rng.integers(0, 600)), int(rng.integers(0, 440))))
    cand = np.zeros(len(pts), oracle.KEYPOINT_DTYPE)
    for i, (x, y) in enumerate(sorted(pts, key=lambda p: (p[1], p[0]))):
        cand[i] = (x, y, 7, -1, rng.integers(7, 200), 0, -1)
    out = oracle.distribute(cand, 16, 624, 16, 464, 10_000)
    assert sorted((int(k["x"]), int(k["y"])) for k in out) == sorted(pts)


@pytest.mark.parametrize("n", [1, 50, 217])
def test_distribute_budget(oracle, n):
    rng = np.random.default_rng(n)
    cand = np.zeros(3000, oracle.KEYPOINT_DTYPE)
    cand["x"] = rng.integers(0, 608, 3000)
    cand["y"] = rng.integers(0, 448, 3000)
    cand["response"] = rng.integers(7, 255, 3000)
    out = oracle.distribute(cand, 16, 624, 16, 464, n)
    assert n <= len(out) <= max(n + 2, 4)


def test_resize_and_blur_sanity(oracle):
    flat = np.full((100, 120), 77, np.uint8)
    assert (oracle.resize_linear(flat, 100, 83) == 77).all()
    assert (oracle.gaussian_blur(flat) == 77).all()
    ramp = np.tile(np.arange(200, dtype=np.uint8), (60, 1))
    r = oracle.resize_linear(ramp, 167, 50).astype(int)
    # interpolation of a horizontal ramp: within 1 of the exact bilinear value
    sx = (np.arange(167) + 0.5) * (200 / 167) - 0.5
    assert np.abs(r - np.clip(sx, 0, 199)[None, :]).max() <= 1.0
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (40, 50)).astype(np.uint8)
    b = oracle.gaussian_blur(img).astype(float)
    k = np.array([18, 34, 48, 56, 48, 34, 18], float) / 256
    pad = np.pad(img.astype(float), 3, mode="reflect")  # numpy "reflect" == BORDER_REFLECT_101
    hor = sum(k[i] * pad[:, i:i + 50] for i in range(7))
    ref = sum(k[i] * hor[i:i + 40, :] for i in range(7))
    assert np.abs(b - ref).max() <= 0.5 + 1e-9


def test_oracle_node_sort_is_compare_nodes():
    """oracle.node_sort orders by (count, UL.x) ascending (compareNodes, src/ORBextractor.cc:676-697)."""
    import numpy as np
    from oracle import oracle as orc
    rng = np.random.default_rng(5)
    c, x = rng.integers(2, 9, 200).astype(np.int32), rng.integers(0, 50, 200).astype(np.int32)
    o = orc.node_sort(c, x)
    assert sorted(o.tolist()) == list(range(200))
    keys = list(zip(c[o].tolist(), x[o].tolist()))
    assert keys == sorted(keys)
