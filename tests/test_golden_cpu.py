"""The CPU oracle and the synthetic generators against the committed golden fixtures
(tests/golden/fixtures.py): a change to either shows up here as a diff against a frozen record.  The GPU
parity tests assert the device outputs against the same records (test_workloads_gpu, test_extract_gpu,
test_chain_gpu, test_ba_gpu, test_tracking_chain_gpu)."""
from __future__ import annotations

import json

import numpy as np
import pytest

from golden import fixtures as fx


@pytest.fixture(scope="module")
def extract_golden():
    return fx.load_json("extract.json")


def test_extract_records_cover_every_config(extract_golden):
    names = set(extract_golden)
    assert {"c1_seed1", "c1_noise_seed2"} <= names
    assert sum(n.startswith("c2_") for n in names) == 64
    assert sum(n.startswith("c3_") for n in names) == 12
    assert sum(n.startswith("c4_") for n in names) == 4


def test_oracle_extraction_matches_golden(oracle, synth, extract_golden):
    for name, img, nf, lap in fx.extract_cases(synth):
        k, d, m = oracle.OracleExtractor(nf, 1.2, 8, 20, 7)(img, lap)
        fx.check_extract(extract_golden[name], img, k, d, m, name)


def test_c1_full_dump(oracle, synth):
    g = fx.load_npz("c1_seed1.npz")
    k, d, m = oracle.OracleExtractor(1000, 1.2, 8, 20, 7)(synth.polygon_frame(640, 480, seed=1), (0, 1000))
    assert np.array_equal(k.view(np.uint8).reshape(-1, 28), g["kps"])
    assert np.array_equal(d, g["desc"]) and int(g["mono"]) == m
    # the record's keypoints are sane cv::KeyPoints: 8 octaves, sizes 31 * scale, responses >= minThFAST
    kp = g["kps"].view(k.dtype).reshape(-1)
    assert set(np.unique(kp["octave"])) == set(range(8)) and (kp["response"] >= 7).all()


def test_oracle_sft_matches_golden(pkg, oracle, synth):
    golden = fx.load_json("sft_c3.json")
    kfs, _ = fx.c3_keyframes(pkg, synth, oracle)
    got = fx.sft_records(pkg, oracle, kfs)
    assert got.keys() == golden.keys()
    for key in golden:
        assert got[key] == golden[key], key
    assert sum(v["n"] for v in golden.values()) > 1000


def test_oracle_local_ba_matches_golden(oracle, synth):
    g = fx.load_npz("ba_c5.npz")
    meta = json.loads(g["meta_json"].tobytes())
    for name, kw in fx.BA_CASES.items():
        prob = synth.local_ba_problem(**kw)
        assert fx.problem_sha(prob) == meta[name]["problem_sha256"], f"{name}: synthetic problem changed"
        pose, point, chi2, depth, res = oracle.local_ba(prob, 10)
        # one thread, fixed summation order: the oracle reproduces its record bit for bit
        assert np.array_equal(pose, g[f"{name}__pose"]) and np.array_equal(point, g[f"{name}__point"]), name
        assert np.array_equal(chi2, g[f"{name}__chi2"]), name
        assert np.array_equal(np.asarray(depth, np.uint8), g[f"{name}__depth"]), name
        assert np.array_equal(fx.ba_path(res), g[f"{name}__path"]), name


def test_small_ba_problem_round_trip(oracle, synth):
    """The small problem is stored whole: the stored arrays rebuild the generator's problem byte for
    byte, and the oracle's solution of the STORED problem equals the record."""
    g = fx.load_npz("ba_c5.npz")
    meta = json.loads(g["meta_json"].tobytes())
    prob = synth.local_ba_problem(**fx.BA_SMALL)
    stored = {}
    for k, v in prob.items():
        if not isinstance(v, np.ndarray):
            stored[k] = v
        elif v.dtype.names:
            dt = np.dtype([tuple(x) for x in meta[f"small_problem__{k}__dtype"]])
            stored[k] = g[f"small_problem__{k}__bytes"].reshape(-1).view(dt)
        else:
            stored[k] = g[f"small_problem__{k}"]
        assert np.asarray(stored[k]).tobytes() == np.asarray(v).tobytes(), k
    assert fx.problem_sha(stored) == meta["small"]["problem_sha256"]
    pose, point, chi2, depth, res = oracle.local_ba(stored, 10)
    assert np.array_equal(pose, g["small__pose"]) and np.array_equal(point, g["small__point"])
    assert np.array_equal(chi2, g["small__chi2"]) and np.array_equal(fx.ba_path(res), g["small__path"])


def test_oracle_tracking_chain_matches_golden(pkg, synth):
    from oracle import tracking_chain
    golden = fx.load_json("tracking.json")
    assert golden.keys() == fx.TRACK_SCENES.keys()
    for name, kw in fx.TRACK_SCENES.items():
        sc = synth.tracking_chain_scene(**kw)
        C, L = pkg.Frame(**sc["cur"]), pkg.Frame(**sc["last"])
        o = tracking_chain.track(pkg, C, L, sc["local"], sc["pose7_pred"], sc["level_sigma2"], fx.track_th(kw), 1)
        assert fx.tracking_record(o) == golden[name], name
    # every TrackWithMotionModel outcome is recorded
    assert {golden[n]["status"] for n in golden} == {0, 1, 3, 4}
