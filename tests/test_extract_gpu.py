"""GPU parity of the HIP ORB extractor against the CPU oracle, stage by stage and end to end.

Bar: bit-exact (pyramid bytes, the blurred levels, FAST candidates + per-cell thresholds, quad-tree
selection order, keypoint structs, descriptors, monoIndex).  Runs on the MI355X box (-m gpu).
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frames(synth):
    left, right, _ = synth.stereo_pair(752, 480, seed=200)
    return {
        "poly640": (synth.polygon_frame(640, 480, seed=1), 1000, (0, 1000)),
        "noise640": (synth.blurred_noise_frame(640, 480, seed=2), 1000, (0, 0)),
        "stereoL752": (left, 1200, (0, 0)),
        "stereoR752": (right, 1200, (0, 0)),
        "poly1280": (synth.polygon_frame(1280, 720, seed=5), 1000, (0, 1000)),
        "init5000": (synth.polygon_frame(640, 480, seed=11), 5000, (0, 1000)),
        "odd_size": (synth.polygon_frame(643, 397, seed=13), 800, (100, 400)),
        "noise1280": (synth.blurred_noise_frame(1280, 720, seed=3), 1000, (0, 1000)),
    }


CASES = ["poly640", "noise640", "stereoL752", "stereoR752", "poly1280", "init5000", "odd_size", "noise1280"]


@pytest.fixture(scope="module")
def frames(synth):
    return _frames(synth)


def _decode(keys: np.ndarray):
    keys = keys.astype(np.uint64)
    return np.stack([(keys >> 8) & 0xFFF, keys >> 20, keys & 0xFF], axis=1).astype(np.int64)


def _first_diff(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.shape != b.shape:
        return f"shape {a.shape} vs {b.shape}"
    idx = np.argwhere(a != b)
    return f"{len(idx)} diffs, first at {idx[0].tolist()}: {a[tuple(idx[0])]} vs {b[tuple(idx[0])]}" if len(idx) else ""


def test_c1_frame_against_golden(pkg, synth):
    """C1 (seed 1, 640x480, N 1000, mono placement) on the device against the committed full dump
    (tests/golden/c1_seed1.npz): keypoint records, descriptors and monoIndex byte for byte."""
    from golden import fixtures as fx
    g = fx.load_npz("c1_seed1.npz")
    img = synth.polygon_frame(640, 480, seed=1)
    kps, desc, mono = pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=640, max_height=480)(img, None, (0, 1000))
    assert np.array_equal(kps.view(np.uint8).reshape(-1, 28), g["kps"])
    assert np.array_equal(desc, g["desc"]) and mono == int(g["mono"])
    fx.check_extract(fx.load_json("extract.json")["c1_seed1"], img, kps, desc, mono, "c1_seed1")


@pytest.mark.parametrize("case", CASES)
def test_extract_parity(pkg, oracle, frames, case):
    img, nf, lap = frames[case]
    h, w = img.shape
    ex = pkg.ORBextractor(nf, 1.2, 8, 20, 7, max_width=1280, max_height=720)
    ref = oracle.OracleExtractor(nf, 1.2, 8, 20, 7)
    kps, desc, mono = ex(img, None, lap)
    rkps, rdesc, rmono = ref(img, lap)
    lib = ex._lib
    for l in range(8):
        # 1. pyramid: the view and the 3-px REFLECT_101 border the extractor keeps (the rest of the
        #    19-px frame is never read, so it is not written)
        gp, rp = ex.level_padded(l), ref.level_padded(l)
        assert np.array_equal(gp[16:-16, 16:-16], rp[16:-16, 16:-16]), \
            f"{case} level {l} pyramid: {_first_diff(gp[16:-16, 16:-16], rp[16:-16, 16:-16])}"
        # 2. blurred level == GaussianBlur(level.clone(), 7x7, 2) of the oracle's level
        lw, lh = rp.shape[1] - 38, rp.shape[0] - 38
        gb = np.zeros((lh, lw), np.uint8)
        assert lib.orb_debug_level_blurred(ex._h, 0, l, gb.ctypes.data) == 0
        rb = oracle.gaussian_blur(rp[19:-19, 19:-19])
        assert np.array_equal(gb, rb), f"{case} level {l} blur: {_first_diff(gb, rb)}"
        # 3. FAST candidates in cell order + per-cell threshold choice
        rc = ref.level_candidates(l)
        rthr = ref.level_cell_thresholds(l)
        cap = max(1, len(rc) + 64)
        buf = np.zeros(cap, np.uint32)
        thr = np.zeros(len(rthr) + 1, np.uint8)
        n = lib.orb_debug_level_candidates(ex._h, 0, l, buf.ctypes.data, cap, thr.ctypes.data, len(thr))
        assert n == len(rc), f"{case} level {l}: {n} candidates vs oracle {len(rc)}"
        got = _decode(buf[:n])
        exp = np.stack([rc["x"], rc["y"], rc["response"]], axis=1).astype(np.int64)
        assert np.array_equal(got, exp), f"{case} level {l} candidates: {_first_diff(got, exp)}"
        assert np.array_equal(thr[:len(rthr)].astype(np.int32), rthr), f"{case} level {l} thresholds"
        # 4. quad-tree selection, in list order (level coordinates)
        rk = ref.level_keys(l)
        sbuf = np.zeros(len(rk) + 64, np.uint32)
        ns = lib.orb_debug_level_selected(ex._h, 0, l, sbuf.ctypes.data, len(sbuf))
        assert ns == len(rk), f"{case} level {l}: {ns} selected vs oracle {len(rk)}"
        sel = _decode(sbuf[:ns]) + np.array([16, 16, 0])
        exp = np.stack([rk["x"], rk["y"], rk["response"]], axis=1).astype(np.int64)
        assert np.array_equal(sel, exp), f"{case} level {l} selection: {_first_diff(sel, exp)}"
    assert lib.orb_debug_status(ex._h) == 0
    # 5. end to end: keypoints (bitwise), descriptors, monoIndex
    assert mono == rmono
    assert len(kps) == len(rkps)
    assert np.array_equal(kps.view(np.uint8), rkps.view(np.uint8)), \
        f"{case} keypoints: {_first_diff(kps.view(np.uint32).reshape(-1, 7), rkps.view(np.uint32).reshape(-1, 7))}"
    assert np.array_equal(desc, rdesc), f"{case} descriptors: {_first_diff(desc, rdesc)}"


@pytest.mark.parametrize("desc_split", ["0", "1"])
def test_batch_equals_single_calls(pkg, oracle, synth, monkeypatch, desc_split):
    """Device batch == oracle per frame; also with the early levels' quad-tree and descriptors on the
    side stream (ORBGPU_DESC_SPLIT=1: staged records placed by the final describe launch)."""
    import torch
    monkeypatch.setenv("ORBGPU_DESC_SPLIT", desc_split)
    frames = synth.frame_batch(6, 640, 480, seed0=300)
    ex = pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=640, max_height=480, max_batch=8)
    imgs = torch.from_numpy(frames).cuda()
    kps, desc, counts = ex.extract_batch_device(imgs, (0, 1000))
    torch.cuda.synchronize()
    counts = counts.cpu().numpy()
    ref = oracle.OracleExtractor(1000, 1.2, 8, 20, 7)
    for f in range(len(frames)):
        rk, rd, rm = ref(frames[f], (0, 1000))
        n = int(counts[f, 0])
        assert n == len(rk) and int(counts[f, 1]) == rm
        gk = pkg.keypoints_to_structured(kps[f], n)
        assert np.array_equal(gk.view(np.uint8), rk.view(np.uint8)), f"frame {f} keypoints"
        assert np.array_equal(desc[f, :n].cpu().numpy(), rd), f"frame {f} descriptors"


def test_empty_image_and_capacity(pkg):
    ex = pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=640, max_height=480)
    k, d, m = ex(np.zeros((0, 0), np.uint8))
    assert m == -1 and len(k) == 0 and d is None
    # a flat image has no corners at all
    k, d, m = ex(np.full((480, 640), 128, np.uint8), None, (0, 1000))
    assert len(k) == 0 and m == 0
    with pytest.raises(Exception):
        ex(np.zeros((800, 900), np.uint8))  # larger than the handle was created for


def test_mv_image_pyramid_and_getters(pkg, oracle, synth):
    img = synth.polygon_frame(640, 480, seed=21)
    ex = pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=640, max_height=480)
    ex(img, None, (0, 0))
    pyr = ex.mvImagePyramid
    assert [p.shape for p in pyr] == [(480, 640), (400, 533), (333, 444), (278, 370), (231, 309), (193, 257),
                                      (161, 214), (134, 179)]
    assert np.array_equal(pyr[0], img)
    p = oracle.OracleExtractor(1000, 1.2, 8, 20, 7).params()
    assert ex.GetLevels() == 8
    assert np.array_equal(np.float32(ex.GetScaleFactors()), p["scale"])
    assert np.array_equal(np.float32(ex.GetInverseScaleSigmaSquares()), p["inv_sigma2"])
    assert ex.mnFeaturesPerLevel == list(p["per_level"])


def test_hamming_knn2(pkg, oracle):
    import torch
    rng = np.random.default_rng(9)
    q = rng.integers(0, 256, (700, 32), dtype=np.uint8)
    t = rng.integers(0, 256, (1300, 32), dtype=np.uint8)
    t[5] = q[3]
    t[17] = q[3]  # a tie at distance 0: the first index wins
    idx, d1, d2 = pkg.ORBmatcher.knn2_device(torch.from_numpy(q).cuda(), torch.from_numpy(t).cuda())
    idx, d1, d2 = idx.cpu().numpy(), d1.cpu().numpy(), d2.cpu().numpy()
    D = np.unpackbits(q[:, None, :] ^ t[None, :, :], axis=2).sum(axis=2)
    for i in range(len(q)):
        best, second, bi = 257, 257, -1
        for j in range(len(t)):
            d = D[i, j]
            if d < best:
                second, best, bi = best, d, j
            elif d < second:
                second = d
        assert (idx[i], d1[i], d2[i]) == (bi, best, second)
    assert idx[3] == 5 and d1[3] == 0 and d2[3] == 0


@pytest.mark.parametrize("nq,nt", [(1000, 1000), (37, 70000), (5, 0), (130, 3), (100, 1024), (100, 1025)],
                         ids=["frame", "big_train", "empty", "tiny", "one_block_max", "two_chunks"])
def test_hamming_knn2_split_merge(pkg, nq, nt):
    """The train split (chunks merged in order) equals the sequential scan, ties across chunk
    boundaries included: every query's exact copy is planted at several train positions."""
    import torch
    rng = np.random.default_rng(nq + nt)
    q = rng.integers(0, 256, (nq, 32), dtype=np.uint8)
    t = rng.integers(0, 256, (max(nt, 1), 32), dtype=np.uint8)[:nt]
    for i in range(0, nq, 3):
        if nt:
            for j in rng.integers(0, nt, 3):
                t[j] = q[i]
    idx, d1, d2 = pkg.ORBmatcher.knn2_device(torch.from_numpy(q).cuda(), torch.from_numpy(t).cuda())
    idx, d1, d2 = idx.cpu().numpy(), d1.cpu().numpy(), d2.cpu().numpy()
    if nt == 0:
        assert (idx == -1).all() and (d1 == 257).all() and (d2 == 257).all()
        return
    pc = np.unpackbits(np.arange(256, dtype=np.uint8)[:, None], axis=1).sum(1).astype(np.int32)
    for i0 in range(0, nq, 8):
        D = pc[q[i0:i0 + 8, None, :] ^ t[None, :, :]].sum(axis=2)
        srt = np.sort(D, axis=1)
        assert np.array_equal(idx[i0:i0 + 8], np.argmin(D, axis=1))
        assert np.array_equal(d1[i0:i0 + 8], srt[:, 0])
        assert np.array_equal(d2[i0:i0 + 8], srt[:, 1] if nt > 1 else np.full(len(srt), 257))


@pytest.mark.parametrize("mode", [("ORBGPU_DEBUG_FLAGS", "8"), ("ORBGPU_DEBUG_FLAGS", "2"), ("ORBGPU_DEBUG_FLAGS", "16"),
                                  ("ORBGPU_DESC_SPLIT", "0")],
                         ids=["kp_scratch_keys", "kp_serial_sort", "kp_lds_sort", "no_desc_split"])
def test_quadtree_variants_parity(pkg, oracle, frames, monkeypatch, mode):
    """Quad-tree variants stay bit-exact: keys forced into the global scratch (flag 8), the single-lane
    libstdc++ sort port (flag 2), the LDS sort emulation for every candidate set (flag 16), and the
    pipeline without the side-stream describe of the early levels."""
    monkeypatch.setenv(*mode)
    for case in ["poly640", "noise1280", "init5000", "odd_size"]:
        img, nf, lap = frames[case]
        ex = pkg.ORBextractor(nf, 1.2, 8, 20, 7, max_width=1280, max_height=720)
        kps, desc, mono = ex(img, None, lap)
        rkps, rdesc, rmono = oracle.OracleExtractor(nf, 1.2, 8, 20, 7)(img, lap)
        assert ex._lib.orb_debug_status(ex._h) == 0, case
        assert mono == rmono and np.array_equal(kps.view(np.uint8), rkps.view(np.uint8)), case
        assert np.array_equal(desc, rdesc), case


def test_quadtree_node_sort_emulations(pkg, oracle):
    """The careful rounds' std::sort(compareNodes) emulations (register version for <= 64 nodes, LDS
    version otherwise) give libstdc++'s exact order, ties included (src/ORBextractor.cc:676-697, 950):
    random records with many equal (count, UL.x) pairs, sorted / reversed / constant inputs, n 0..300."""
    lib = pkg._lib.load()
    rng = np.random.default_rng(77)
    cases = []
    for n in list(range(0, 70)) + [100, 129, 200, 300]:
        for kind in range(4):
            if kind == 0:
                c, x = rng.integers(2, 6, n), rng.integers(0, 4, n) * 37
            elif kind == 1:
                c, x = rng.integers(2, 200, n), rng.integers(0, 600, n)
            elif kind == 2:
                c, x = np.sort(rng.integers(2, 9, n))[::-1].copy(), np.full(n, 5)
            else:
                c, x = np.full(n, 3), np.arange(n) % 3
            cases.append((c.astype(np.int32), x.astype(np.int32)))
    used_reg = 0
    for c, x in cases:
        exp = oracle.node_sort(c, x)
        for mode in (0, 1):
            out = np.zeros(len(c), np.int32)
            rc = lib.orb_debug_node_sort(c.ctypes.data, x.ctypes.data, len(c), mode, out.ctypes.data)
            assert rc >= 0
            used_reg += rc
            assert np.array_equal(out, exp), (len(c), mode, c.tolist(), x.tolist())
    assert used_reg > 200  # the register version ran for most of the n <= 64 cases


def test_sparse_corners_parity(pkg, oracle):
    """Few corners per level: the quad-tree stops because no node can be split further (src:912-918,
    nodes == prevSize) rather than at N, single-key roots and levels with one or no candidate."""
    rng = np.random.default_rng(31)
    for n_rect in (1, 3, 12):
        img = np.full((480, 640), 90, np.uint8)
        for _ in range(n_rect):
            x0, y0 = int(rng.integers(40, 560)), int(rng.integers(40, 400))
            img[y0:y0 + int(rng.integers(12, 60)), x0:x0 + int(rng.integers(12, 60))] = int(rng.integers(150, 255))
        ex = pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=640, max_height=480)
        kps, desc, mono = ex(img, None, (0, 1000))
        rkps, rdesc, rmono = oracle.OracleExtractor(1000, 1.2, 8, 20, 7)(img, (0, 1000))
        assert ex._lib.orb_debug_status(ex._h) == 0
        assert mono == rmono and len(kps) == len(rkps) > 0, n_rect
        assert np.array_equal(kps.view(np.uint8), rkps.view(np.uint8)), n_rect
        assert np.array_equal(desc, rdesc), n_rect


@pytest.mark.parametrize("env", [{"ORBGPU_CHUNK": "2"}, {"ORBGPU_STREAMS": "2", "ORBGPU_CHUNK": "3"},
                                 {"ORBGPU_FAST_SPLIT": "3"}, {"ORBGPU_FAST_PER_LEVEL": "1"}, {"ORBGPU_QT_SPLIT": "1"},
                                 {"ORBGPU_FAST_STAMPS": "1", "ORBGPU_PYR_STAMPS": "1"}, {"ORBGPU_PYR_PAIR": "1"}],
                         ids=["chunk2", "streams2_chunk3", "fast_split3", "fast_per_level", "qt_split", "phase_stamps",
                              "two_level_pyramid"])
def test_schedule_switches_parity(pkg, oracle, synth, monkeypatch, env):
    """Every per-handle schedule switch (read when the handle is created; orb_extract.hip
    orb_extractor_create) changes only how the batch is cut into launches and streams: a 7-frame batch
    (a chunk size that does not divide it) stays bit-exact against the oracle."""
    import torch
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    frames = synth.frame_batch(7, 640, 480, seed0=1400)
    ex = pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=640, max_height=480, max_batch=8)
    kps, desc, counts = ex.extract_batch_device(torch.from_numpy(frames).cuda(), (0, 1000))
    torch.cuda.synchronize()
    assert ex._lib.orb_debug_status(ex._h) == 0
    counts = counts.cpu().numpy()
    ref = oracle.OracleExtractor(1000, 1.2, 8, 20, 7)
    for f in range(len(frames)):
        rk, rd, rm = ref(frames[f], (0, 1000))
        n = int(counts[f, 0])
        assert n == len(rk) and int(counts[f, 1]) == rm, f
        assert np.array_equal(pkg.keypoints_to_structured(kps[f], n).view(np.uint8), rk.view(np.uint8)), f
        assert np.array_equal(desc[f, :n].cpu().numpy(), rd), f


def test_batch_outputs_to_pinned_host(pkg, synth):
    """orb_extract_batch_device writing keypoints, descriptors and counts straight into pinned host
    memory (the PCIe bench's download-free form) gives the bytes of the device-output call."""
    import ctypes
    import torch
    frames = synth.frame_batch(4, 640, 480, seed0=1600)
    ex = pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=640, max_height=480, max_batch=4)
    imgs = torch.from_numpy(frames).cuda()
    kps, desc, counts = ex.extract_batch_device(imgs, (0, 1000))
    cap = kps.shape[1]
    hk = torch.empty(kps.shape, dtype=kps.dtype).pin_memory()
    hd = torch.empty(desc.shape, dtype=desc.dtype).pin_memory()
    hc = torch.empty(counts.shape, dtype=counts.dtype).pin_memory()
    st = torch.cuda.current_stream()
    rc = ex._lib.orb_extract_batch_device(ex._h, imgs.data_ptr(), 4, 640, 480, 640, 640 * 480, 0, 1000,
                                          hk.data_ptr(), hd.data_ptr(), cap, hc.data_ptr(), ctypes.c_void_p(st.cuda_stream))
    assert rc >= 0
    torch.cuda.synchronize()
    c = counts.cpu()
    assert torch.equal(hc, c)
    for f in range(4):
        n = int(c[f, 0])
        assert torch.equal(hk[f, :n].view(torch.int32), kps[f, :n].cpu().view(torch.int32)), f
        assert torch.equal(hd[f, :n], desc[f, :n].cpu()), f


def test_set_overlap_parity(pkg, oracle, synth):
    """orb_extractor_set_overlap: a batch as one chain on the caller's stream (0) and with the early
    levels on the side streams (1, the default) give the oracle's keypoints and descriptors; bad modes
    are rejected."""
    import torch
    frames = synth.frame_batch(5, 640, 480, seed0=1500)
    ex = pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=640, max_height=480, max_batch=8)
    ref = oracle.OracleExtractor(1000, 1.2, 8, 20, 7)
    imgs = torch.from_numpy(frames).cuda()
    for on in (False, True, False):
        ex.set_overlap(on)
        kps, desc, counts = ex.extract_batch_device(imgs, (0, 1000))
        torch.cuda.synchronize()
        counts = counts.cpu().numpy()
        for f in range(len(frames)):
            rk, rd, rm = ref(frames[f], (0, 1000))
            n = int(counts[f, 0])
            assert n == len(rk) and int(counts[f, 1]) == rm, (on, f)
            assert np.array_equal(pkg.keypoints_to_structured(kps[f], n).view(np.uint8), rk.view(np.uint8)), (on, f)
            assert np.array_equal(desc[f, :n].cpu().numpy(), rd), (on, f)
    assert ex._lib.orb_extractor_set_overlap(ex._h, 2) < 0


@pytest.mark.parametrize("w,h,kind,nf,scale,nlevels,ini,mn", [
    (1280, 720, "poly", 1500, 1.5, 6, 25, 10),   # level ratio > 1.25: the wide-box resize path
    (1280, 720, "noise", 800, 2.0, 4, 20, 7),    # ratio 2, few levels
    (752, 480, "poly", 1000, 1.1, 12, 15, 5),    # 12 levels (kMaxLevels), low thresholds
    (104, 110, "noise", 200, 1.2, 2, 20, 7),     # one cell column per level: 72- and 55-px FAST windows
    (640, 480, "poly", 1000, 1.2, 7, 20, 7),     # odd level count (with ORBGPU_PYR_PAIR=1: three two-level passes, then one)
])
@pytest.mark.parametrize("pair", ["0", "1", "2"], ids=["level_passes", "two_level_passes", "first_two_levels"])
def test_extract_parity_other_parameters(pkg, oracle, synth, monkeypatch, w, h, kind, nf, scale, nlevels, ini, mn, pair):
    """ORBextractor parameters other than the 1.2 / 8 / 20 / 7 of the bench configs (the reference
    reads them from the settings file, src/Tracking.cc:1346-1362): pyramid levels, keypoints (bitwise)
    and descriptors against the oracle, with the level-by-level pyramid and with the two-level passes
    (ORBGPU_PYR_PAIR=1; level ratios above ~1.25 do not fit its boxes and keep the level passes)."""
    monkeypatch.setenv("ORBGPU_PYR_PAIR", pair)
    img = synth.polygon_frame(w, h, seed=21) if kind == "poly" else synth.blurred_noise_frame(w, h, seed=22)
    ex = pkg.ORBextractor(nf, scale, nlevels, ini, mn, max_width=w, max_height=h)
    ref = oracle.OracleExtractor(nf, scale, nlevels, ini, mn)
    kps, desc, mono = ex(img, None, (0, 1000))
    rkps, rdesc, rmono = ref(img, (0, 1000))
    for l in range(nlevels):
        gp, rp = ex.level_padded(l), ref.level_padded(l)
        assert np.array_equal(gp[16:-16, 16:-16], rp[16:-16, 16:-16]), f"level {l}: {_first_diff(gp[16:-16, 16:-16], rp[16:-16, 16:-16])}"
    assert mono == rmono and len(kps) == len(rkps) > 0
    assert np.array_equal(kps.view(np.uint8), rkps.view(np.uint8)), \
        _first_diff(kps.view(np.uint32).reshape(-1, 7), rkps.view(np.uint32).reshape(-1, 7))
    assert np.array_equal(desc, rdesc), _first_diff(desc, rdesc)


def test_scale_factor_above_two_is_rejected(pkg, synth):
    """The pyramid tiles' LDS source boxes cover level ratios up to 2: a larger scale factor fails
    loudly instead of reading past the box."""
    img = synth.polygon_frame(1280, 720, seed=23)
    ex = pkg.ORBextractor(500, 3.0, 3, 20, 7, max_width=1280, max_height=720)
    with pytest.raises(pkg.OrbGpuError):
        ex(img, None, (0, 0))
    with pytest.raises(pkg.OrbGpuError):  # and again: the rejected geometry is not reused
        ex(img, None, (0, 0))
