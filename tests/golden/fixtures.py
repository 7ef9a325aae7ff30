"""Golden fixtures of the hot path: what the CPU oracle outputs on the seeded
synthetic workloads, committed so that a change to the oracle, to the synthetic generators or to the
product shows up as a diff against a frozen record, not only as a disagreement between two live
computations.

The reference ships no images and no expected keypoints / descriptors / BA results (SURVEY.md §4,
§8c), so these records pin against drift; they do not pin against the reference itself.  Parity with
the reference rests on the oracle's restatement.

Records (tests/golden/*.json, *.npz), written by tests/golden/gen_golden.py:
  extract.json     per frame: input SHA-256, keypoint count, monoIndex, SHA-256 of the keypoint records
                   (cv::KeyPoint layout, 28 B each) and of the descriptors (32 B each):
                   C1 (seed 1 polygon + seed 2 blurred noise, 640x480, N 1000, mono), C2 (64 frames,
                   seeds 100..163), C3 (6 stereo pairs 752x480, N 1200, stereo placement), C4 (4 frames
                   1280x720, seeds 1000..1003)
  c1_seed1.npz     the C1 frame's full keypoints and descriptors
  sft_c3.json      SearchForTriangulation on the C3 keyframe chain (tests/test_chain_gpu.py's scene):
                   count and SHA-256 of vMatches12 per (keyframe, neighbour, flags)
  ba_c5.npz        LocalBA C5 (mono seed 7, 50/50 seed 8): the problem's SHA-256 and the oracle's
                   solution (poses, points, edge chi2, depth flags, LM path); the full small problem
                   (6 keyframes, 150 points) with its solution
  tracking.json    the oracle tracking chain on scenes 81 / 82 (stereo) / 83 (mono) and on the
                   TrackWithMotionModel gate scenes: status, match counts, SHA-256 of the matches and
                   outlier flags, the final pose
"""
from __future__ import annotations

import hashlib
import json
import pathlib

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent

EUROC_BF, EUROC_B = 47.90639384423901, 0.110074
SFT_FLAGS = [(0, 0, 0), (0, 0, 1), (1, 0, 1), (0, 1, 0)]


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8).tobytes()).hexdigest()


def load_json(name: str) -> dict:
    return json.loads((HERE / name).read_text())


def load_npz(name: str):
    return np.load(HERE / name, allow_pickle=False)


# ---- extraction
def extract_cases(synth):
    """(name, image, nfeatures, lapping) of every recorded frame."""
    cases = [("c1_seed1", synth.polygon_frame(640, 480, seed=1), 1000, (0, 1000)),
             ("c1_noise_seed2", synth.blurred_noise_frame(640, 480, seed=2), 1000, (0, 1000))]
    cases += [(f"c2_seed{100 + i}", synth.polygon_frame(640, 480, seed=100 + i), 1000, (0, 1000)) for i in range(64)]
    L, R, _, _ = synth.stereo_sequence(6, seed=214)
    for f in range(6):
        cases.append((f"c3_left{f}", L[f], 1200, (0, 0)))
        cases.append((f"c3_right{f}", R[f], 1200, (0, 0)))
    cases += [(f"c4_seed{1000 + i}", synth.polygon_frame(1280, 720, seed=1000 + i), 1000, (0, 1000)) for i in range(4)]
    return cases


def extract_record(img, kps_struct, desc, mono) -> dict:
    return {"image_sha256": sha(img), "n": int(len(kps_struct)), "mono": int(mono),
            "kps_sha256": sha(kps_struct), "desc_sha256": sha(np.asarray(desc, np.uint8).reshape(-1, 32))}


def check_extract(rec: dict, img, kps_struct, desc, mono, what: str = "") -> None:
    got = extract_record(img, kps_struct, desc, mono)
    assert got["image_sha256"] == rec["image_sha256"], f"{what}: synthetic input changed"
    for k in ("n", "mono", "kps_sha256", "desc_sha256"):
        assert got[k] == rec[k], f"{what}: {k} {got[k]} != golden {rec[k]}"


# ---- SearchForTriangulation on the C3 keyframe chain
def c3_keyframes(pkg, synth, oracle):
    """The oracle side of tests/test_chain_gpu.py's chain: 6 stereo keyframes (extraction, stereo
    matches, BoW) as plain-data KeyFrames."""
    n = 6
    L, R, Tcw, _ = synth.stereo_sequence(n, seed=214)
    voc = synth.dbow_vocabulary(10, 6, seed=61)
    scale, sigma2 = synth.scale_tables()
    rng = np.random.default_rng(3)
    has_mp = (rng.random((n, 1200 + 16 * 8)) < 0.2).astype(np.uint8)
    kfs = []
    for f in range(n):
        exa, exb = oracle.OracleExtractor(1200, 1.2, 8, 20, 7), oracle.OracleExtractor(1200, 1.2, 8, 20, 7)
        kl, dl, _ = exa(L[f], (0, 0))
        kr, dr, _ = exb(R[f], (0, 0))
        p = exa.params()
        ur, _, _ = oracle.compute_stereo_matches(kl, dl, kr, dr, [exa.level_padded(l) for l in range(8)],
                                                 [exb.level_padded(l) for l in range(8)], p["scale"], p["inv_scale"],
                                                 EUROC_BF, EUROC_B)
        _, fv = oracle.bow_transform(voc, dl, 4)
        kfs.append(pkg.KeyFrame(keys_un=kl, descriptors=dl, Tcw=Tcw[f], camera=synth.EUROC_K, scale_factors=scale,
                                level_sigma2=sigma2, u_right=ur, has_mappoint=has_mp[f, :len(kl)], feat_vec=fv))
    return kfs, has_mp


def sft_key(k1: int, k2: int, flags) -> str:
    return f"{k1}-{k2}-" + "".join(str(int(v)) for v in flags)


def sft_records(pkg, oracle, kfs) -> dict:
    out = {}
    n = len(kfs)
    for flags in SFT_FLAGS:
        only_stereo, coarse, check_ori = flags
        for k1 in (n - 1, 0):
            for k2 in range(n):
                if k2 == k1:
                    continue
                g = pkg.ORBmatcher.pair_geometry(kfs[k1], kfs[k2])
                rn, rm = oracle.search_for_triangulation(kfs[k1], kfs[k2], g, only_stereo, coarse, check_ori)
                out[sft_key(k1, k2, flags)] = {"n": int(rn), "matches_sha256": sha(np.asarray(rm, np.int32))}
    return out


# ---- LocalBA
BA_CASES = {"c5_mono_seed7": dict(stereo_frac=0.0, seed=7), "c5_mixed_seed8": dict(stereo_frac=0.5, seed=8)}
BA_SMALL = dict(n_kf=6, n_points=150, obs_per_point=4, stereo_frac=0.3, n_fixed=1, seed=3)


def problem_sha(prob: dict) -> str:
    h = hashlib.sha256()
    for k in sorted(prob):
        v = prob[k]
        if isinstance(v, np.ndarray):
            h.update(k.encode())
            h.update(np.ascontiguousarray(v).view(np.uint8).tobytes())
        elif isinstance(v, (int, float)):
            h.update(f"{k}={v!r}".encode())
    return h.hexdigest()


def ba_path(res: dict) -> np.ndarray:
    return np.array([res["iterations"], res["trials"], res["terminated"], res["stopped"]], np.int64)


# ---- tracking chain: the parity scenes, and scenes for TrackWithMotionModel's decisions (the 2 th
# retry recovering, exactly 20 after it, failing twice, nmatchesMap < 10)
TRACK_SCENES = {"scene81": dict(seed=81), "scene82": dict(seed=82), "scene83": dict(seed=83, stereo=False),
                "gate_retry": dict(seed=81, pred_rot=0.05, pred_trans=0.3),
                "gate_exactly_20": dict(seed=81, pred_rot=0.1, pred_trans=0.5),
                "gate_fails_twice": dict(seed=83, pred_rot=0.1, pred_trans=0.5),
                "gate_few_map_points": dict(seed=84, unobserved_frac=0.99)}


def track_th(kw: dict) -> int:
    return 7 if kw.get("stereo", True) else 15


def tracking_record(o: dict) -> dict:
    return {"n1": int(o["n1"]), "n2": int(o["n2"]), "I1": int(o["I1"]), "I2": int(o["I2"]),
            "n_kept": int(o["n_kept"]), "n_map": int(o["n_map"]),
            "m1_sha256": sha(np.asarray(o["m1"], np.int32)), "m2_sha256": sha(np.asarray(o["m2"], np.int32)),
            "O1_sha256": sha(np.asarray(o["O1"], np.uint8)), "O2_sha256": sha(np.asarray(o["O2"], np.uint8)),
            "pose2": [float(v) for v in np.asarray(o["pose2"], np.float64)], "status": int(o["status"])}
