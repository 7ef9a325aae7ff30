"""The device-resident tracking chain (tracking.TrackingChain: Tracking::TrackWithMotionModel ->
TrackLocalMap, src/Tracking.cc:4112-4217, 4234-4300, 4742-4825) against the same chain on the oracle:
SearchByProjection(LastFrame) -> PoseOptimization -> outlier discard -> isInFrustum at the optimised
pose (skipping the points the frame holds) -> SearchByProjection(local map) -> PoseOptimization.

Two checks per scene.  Stage by stage: each oracle stage is fed the device's previous outputs, and its
outputs must equal the device's bit for bit (matches, graphs, outlier flags, the discard's counts) --
the poses within PoseOptimization's 1e-6 bar.  End to end: the oracle chain run on its own poses gives
the same matches and outlier flags."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _device(pkg, sc, C, L, cap=None, last_cap=None, local=None):
    import torch
    dev = torch.device("cuda")

    def up(a, dt):
        return torch.from_numpy(np.ascontiguousarray(a, dt)).to(dev)

    def dframe(F, pad=37, cap=None):
        # capacity past the count, filled with junk keypoints the chain must not read
        rng = np.random.default_rng(F.N)
        if cap is not None:
            pad = cap - F.N
        cap_f = F.N + pad
        k = np.concatenate([F.mvKeysUn, F.mvKeysUn[rng.integers(0, F.N, pad)]])
        d = np.concatenate([F.mDescriptors, rng.integers(0, 256, (pad, 32), dtype=np.uint8)])
        kps = up(k.view(np.float32).reshape(1, cap_f, 7), np.float32)
        desc = up(d.reshape(1, cap_f, 32), np.uint8)
        counts = up(np.array([[F.N, 0]]), np.int32)
        ur = None if F.mvuRight is None else up(np.concatenate([F.mvuRight, np.full(pad, 100, np.float32)]).reshape(1, cap_f),
                                                np.float32)
        return pkg.DeviceFrame(kps, desc, counts, 0, F.Tcw, sc["cur"]["camera"], F.mvScaleFactors, sc["level_sigma2"],
                               int(F.mnMaxX), int(F.mnMaxY), F.mbf, ur)

    cur, last = dframe(C, cap=cap), dframe(L, cap=last_cap if last_cap is not None else cap)
    mp = L.map_points
    pad = last.cap - L.N

    def padded(a, v):
        return np.concatenate([a, np.full((pad,) + a.shape[1:], v, a.dtype)])
    lastp = pkg.DeviceLastPoints(last, up(padded(mp["valid"], 1), np.uint8), up(padded(mp["observed"], 1), np.uint8),
                                 up(padded(mp["xyz"], 1.0), np.float32), up(padded(mp["desc"], 0), np.uint8))
    local = pkg.DeviceLocalMap.from_host(dev, **(sc["local"] if local is None else local))
    return cur, lastp, local


def _frames(pkg, sc):
    return pkg.Frame(**sc["cur"]), pkg.Frame(**sc["last"])


def _oracle_stages(pkg, sc, C, L, th_motion, th_local, pose1=None):
    from oracle import tracking_chain
    return tracking_chain.track(pkg, C, L, sc["local"], sc["pose7_pred"], sc["level_sigma2"], th_motion, th_local,
                                pose1=pose1)


@pytest.mark.parametrize("seed,stereo", [(81, True), (82, True), (83, False)])
def test_tracking_chain_vs_oracle(pkg, oracle, synth, seed, stereo):
    import torch
    sc = synth.tracking_chain_scene(seed=seed, stereo=stereo)
    C, L = _frames(pkg, sc)
    th_motion = 7 if stereo else 15
    cur, last, local = _device(pkg, sc, C, L)
    chain = pkg.TrackingChain(cur.cap, th_motion=th_motion, th_local=1)
    r = chain.track(cur, last, local, sc["pose7_pred"]).sync()
    # stage by stage, the oracle fed the device's pose
    o = _oracle_stages(pkg, sc, C, L, th_motion, 1, pose1=r["pose1"])
    assert r["n1"] == o["n1"] > 100
    assert np.array_equal(r["edges1"].view(np.uint8), o["e1"].view(np.uint8))
    assert np.array_equal(r["edge_kp1"], o["kp1"])
    assert np.array_equal(r["outlier1"], o["O1"]) and o["O1"].sum() > 0
    assert np.abs(r["pose1"] - o["pose1"]).max() < 1e-6
    assert r["inliers"][0] == o["I1"]
    assert np.array_equal(r["m1"][:C.N], o["m1"])
    assert (r["n_kept"], r["n_map"]) == (o["n_kept"], o["n_map"])
    assert np.array_equal(chain.taken[:C.N].cpu().numpy(), o["taken"])
    tiv = local.track_in_view[:local.n].cpu().numpy()
    assert np.array_equal(tiv, o["in_view"])
    assert (o["in_view"] == 0).sum() > (o["tf"]["track_in_view"] == 0).sum()  # the held points were skipped
    for k in ("track_proj", "track_depth", "track_level", "track_view_cos"):
        got = getattr(local, k)[:local.n].cpu().numpy()
        assert np.array_equal(got[tiv == 1], o["tf"][k][tiv == 1]), k
    assert r["n2"] == o["n2"] > 50
    assert np.array_equal(r["m2"][:C.N], o["m2"])
    assert np.array_equal(r["edges2"].view(np.uint8), o["e2"].view(np.uint8))
    assert np.array_equal(r["edge_kp2"], o["kp2"])
    assert np.array_equal(r["outlier2"], o["O2"])
    assert np.abs(r["pose2"] - o["pose2"]).max() < 1e-6
    assert r["inliers"][1] == o["I2"]
    # end to end: the oracle on its own poses
    e = _oracle_stages(pkg, sc, C, L, th_motion, 1)
    for k in ("m1", "m2", "O1", "O2"):
        assert np.array_equal(e[k], o[k]), k
    assert np.abs(e["pose2"] - r["pose2"]).max() < 1e-6
    # and against the committed record of the oracle chain (tests/golden/tracking.json)
    from golden import fixtures as fx
    g = fx.load_json("tracking.json")[f"scene{seed}"]  # (scene83 is the mono one)
    dev = fx.tracking_record(dict(n1=r["n1"], n2=r["n2"], I1=r["inliers"][0], I2=r["inliers"][1], n_kept=r["n_kept"],
                                  n_map=r["n_map"], m1=r["m1"][:C.N], m2=r["m2"][:C.N], O1=r["outlier1"],
                                  O2=r["outlier2"], pose2=g["pose2"], status=r["status"]))
    assert dev == g, seed
    assert np.abs(r["pose2"] - np.asarray(g["pose2"])).max() < 1e-6
    # and the chain tracked: the final pose is closer to the truth than the prediction
    t = sc["pose7_true"]
    assert np.linalg.norm(r["pose2"][:3] - t[:3]) < 0.5 * np.linalg.norm(sc["pose7_pred"][:3] - t[:3])
    torch.cuda.synchronize()


def test_tracking_chain_reuse_and_no_local_map(pkg, oracle, synth):
    """A chain object tracks several frames in turn (buffers reused, state from the previous frame not
    leaking), and an empty local map leaves the second search without matches."""
    import torch
    chain = None
    for seed in (84, 85):
        sc = synth.tracking_chain_scene(seed=seed, n_points=1200)
        C, L = _frames(pkg, sc)
        cur, last, local = _device(pkg, sc, C, L)
        chain = chain or pkg.TrackingChain(max(cur.cap, 4096))
        r = chain.track(cur, last, local, sc["pose7_pred"]).sync()
        o = _oracle_stages(pkg, sc, C, L, 7, 1, pose1=r["pose1"])
        assert np.array_equal(r["m1"][:C.N], o["m1"]) and np.array_equal(r["m2"][:C.N], o["m2"])
        assert (r["m1"][C.N:cur.cap] == -1).all() and (r["m2"][C.N:cur.cap] == -1).all()
        assert np.abs(r["pose2"] - o["pose2"]).max() < 1e-6
    sc = synth.tracking_chain_scene(seed=86, n_points=1200)
    C, L = _frames(pkg, sc)
    cur, last, _ = _device(pkg, sc, C, L)
    empty = pkg.DeviceLocalMap.from_host(torch.device("cuda"), **{k: v[:0] for k, v in sc["local"].items()})
    r = chain.track(cur, last, empty, sc["pose7_pred"]).sync()
    assert r["n2"] == 0 and (r["m2"][:cur.cap] == -1).all()
    assert r["n1"] > 100 and len(r["edges2"]) == r["n_kept"]


@pytest.mark.parametrize("stereo,seeds", [(True, (81, 82, 84)), (False, (83, 86))])
def test_tracking_chain_batch_equals_single(pkg, synth, stereo, seeds):
    """orb_tracking_chain_batch_device: one launch per stage over the frames (a batch with a free slot);
    every frame's outputs equal the single chain's on the same inputs, bit for bit (poses included)."""
    scenes = [synth.tracking_chain_scene(seed=s, stereo=stereo) for s in seeds]
    fr = [_frames(pkg, sc) for sc in scenes]
    cap = max(max(C.N, L.N) for C, L in fr) + 37
    devs = [_device(pkg, sc, C, L, cap=cap) for sc, (C, L) in zip(scenes, fr)]
    th = 7 if stereo else 15
    single = []
    for sc, (cur, last, local) in zip(scenes, devs):
        ch = pkg.TrackingChain(cap, th_motion=th, th_local=1)
        single.append(ch.track(cur, last, local, sc["pose7_pred"]).sync())
    batch = pkg.TrackingChainBatch(cap, len(seeds) + 1, th_motion=th, th_local=1)
    res = batch.track([(cur, last, local, sc["pose7_pred"]) for sc, (cur, last, local) in zip(scenes, devs)]).sync()
    assert len(res) == len(seeds)
    for r, o in zip(res, single):
        for k in ("n1", "n2", "n_kept", "n_map"):
            assert r[k] == o[k], k
        for k in ("m1", "m2", "edge_kp1", "edge_kp2", "outlier1", "outlier2", "inliers"):
            assert np.array_equal(np.asarray(r[k]), np.asarray(o[k])), k
        for k in ("edges1", "edges2"):
            assert np.array_equal(r[k].view(np.uint8), o[k].view(np.uint8)), k
        assert np.array_equal(r["pose1"], o["pose1"]) and np.array_equal(r["pose2"], o["pose2"])
        for k in (0, 1):  # the graphs' frame records, but for the batch's edge offset
            for f in ("pose", "n_edges"):
                assert np.array_equal(r["frames"][k][f], o["frames"][k][f]), f
        assert o["n1"] > 100 and o["n2"] > 0


def test_tracking_chain_batch_ragged(pkg, synth):
    """A batch whose frames differ in everything but cap: last-frame capacities, local map sizes (full,
    truncated, empty) and a local map without the last-frame links; grids sized for the largest frame
    must leave the others' results as their single chains give them."""
    specs = [(81, None, 5, True), (82, 700, 60, True), (84, 0, 0, True), (85, 1200, 17, False)]
    scenes = [synth.tracking_chain_scene(seed=s) for s, _, _, _ in specs]
    fr = [_frames(pkg, sc) for sc in scenes]
    cap = max(C.N for C, _ in fr) + 11
    devs = []
    for (seed, nloc, lpad, links), sc, (C, L) in zip(specs, scenes, fr):
        loc = {k: (v if nloc is None else v[:nloc]) for k, v in sc["local"].items() if links or k != "last_row"}
        devs.append(_device(pkg, sc, C, L, cap=cap, last_cap=L.N + lpad, local=loc))
    single = []
    for sc, (cur, last, local) in zip(scenes, devs):
        single.append(pkg.TrackingChain(cap).track(cur, last, local, sc["pose7_pred"]).sync())
    res = pkg.TrackingChainBatch(cap, len(specs)).track(
        [(cur, last, local, sc["pose7_pred"]) for sc, (cur, last, local) in zip(scenes, devs)]).sync()
    for (seed, nloc, _, _), r, o in zip(specs, res, single):
        for k in ("n1", "n2", "n_kept", "n_map"):
            assert r[k] == o[k], (seed, k)
        for k in ("m1", "m2", "edge_kp1", "edge_kp2", "outlier1", "outlier2", "inliers"):
            assert np.array_equal(np.asarray(r[k]), np.asarray(o[k])), (seed, k)
        assert np.array_equal(r["pose1"], o["pose1"]) and np.array_equal(r["pose2"], o["pose2"]), seed
        if nloc == 0:
            assert r["n2"] == 0


def test_tracking_chain_batch_many_slots(pkg, synth):
    """A batch of 48 frames (three scenes dealt round-robin, each slot with its own local map, as the
    bench's 256-frame batches run): every slot's outputs equal its scene's single chain, so the grid
    rows, the per-frame argument blocks and the scratch strides hold past a handful of frames."""
    scenes = [synth.tracking_chain_scene(seed=s) for s in (81, 82, 84)]
    fr = [_frames(pkg, sc) for sc in scenes]
    cap = max(max(C.N, L.N) for C, L in fr) + 5
    devs = [_device(pkg, sc, C, L, cap=cap) for sc, (C, L) in zip(scenes, fr)]
    single = [pkg.TrackingChain(cap).track(cur, last, local, sc["pose7_pred"]).sync()
              for sc, (cur, last, local) in zip(scenes, devs)]
    n = 48
    items = []
    for i in range(n):
        k = i % 3
        sc, (cur, last, _) = scenes[k], devs[k]
        local = _device(pkg, sc, *fr[k], cap=cap)[2]  # a local map per slot: isInFrustum writes its fields
        items.append((cur, last, local, sc["pose7_pred"]))
    res = pkg.TrackingChainBatch(cap, n).track(items).sync()
    assert len(res) == n
    for i, r in enumerate(res):
        o = single[i % 3]
        for k in ("n1", "n2", "n_kept", "n_map"):
            assert r[k] == o[k], (i, k)
        for k in ("m1", "m2", "edge_kp1", "edge_kp2", "outlier1", "outlier2", "inliers"):
            assert np.array_equal(np.asarray(r[k]), np.asarray(o[k])), (i, k)
        assert np.array_equal(r["pose1"], o["pose1"]) and np.array_equal(r["pose2"], o["pose2"]), i


# TrackWithMotionModel's decisions on the device (src/Tracking.cc:4149-4217): scenes whose motion-model
# prediction is off by enough that the th search finds < 20 matches (the 2 th search recovers; exactly 20
# passes), fails twice, or passes the search with too few observed map points (nmatchesMap < 10)
# (the scene parameters are tests/golden/fixtures.py's TRACK_SCENES, whose oracle records the
# status of each)
GATE_SCENES = {
    "retry_recovers": ("gate_retry", 1),
    "retry_exactly_20": ("gate_exactly_20", 1),
    "fails_twice": ("gate_fails_twice", 3),
    "few_map_points": ("gate_few_map_points", 4),
    "tracked": ("scene82", 0),
}


def _gate_scene(synth, name):
    from golden import fixtures as fx
    key, status = GATE_SCENES[name]
    return synth.tracking_chain_scene(**fx.TRACK_SCENES[key]), key, status


def _check_gate(r, o, C, what):
    assert r["status"] == o["status"], (what, r["status"], o["status"])
    for k in ("n1", "n2", "n_kept", "n_map"):
        assert r[k] == o[k], (what, k, r[k], o[k])
    for k in ("m1", "m2"):
        assert np.array_equal(np.asarray(r[k])[:C.N], o[k]), (what, k)
    assert np.array_equal(np.asarray(r["outlier1"]), o["O1"]) and np.array_equal(np.asarray(r["outlier2"]), o["O2"]), what
    assert list(np.asarray(r["inliers"])) == [o["I1"], o["I2"]], what
    assert np.abs(r["pose1"] - o["pose1"]).max() < 1e-6 and np.abs(r["pose2"] - o["pose2"]).max() < 1e-6, what


@pytest.mark.parametrize("name", list(GATE_SCENES))
def test_tracking_chain_motion_gate(pkg, synth, name):
    """Single chain: the status word, the matches of the search that counted (the 2 th one after a retry),
    no graph / no local-map stage after a failure, poses as documented -- equal to the oracle chain's
    TrackWithMotionModel decisions (oracle/tracking_chain.py, gate=True)."""
    from golden import fixtures as fx
    sc, key, status = _gate_scene(synth, name)
    C, L = _frames(pkg, sc)
    cur, last, local = _device(pkg, sc, C, L)
    r = pkg.TrackingChain(cur.cap).track(cur, last, local, sc["pose7_pred"]).sync()
    o = _oracle_stages(pkg, sc, C, L, 7, 1)
    assert o["status"] == status, (name, o["status"])
    _check_gate(r, o, C, name)
    g = fx.load_json("tracking.json")[key]
    assert g["status"] == r["status"] and g["n1"] == r["n1"] and g["n2"] == r["n2"]
    assert g["m1_sha256"] == fx.sha(np.asarray(r["m1"][:C.N], np.int32))
    if status & 6:  # a failed frame: nothing after the search / the first PoseOptimization
        assert r["n2"] == 0 and (r["m2"][:cur.cap] == -1).all() and int(r["frames"][1]["n_edges"]) == 0
    if status == 3:
        assert int(r["frames"][0]["n_edges"]) == 0 and np.array_equal(r["pose1"], np.asarray(sc["pose7_pred"]))


def test_tracking_chain_motion_gate_off(pkg, synth):
    """gate=False: every stage runs with th as given, as the oracle chain with its gate off."""
    sc, _, _ = _gate_scene(synth, "fails_twice")
    C, L = _frames(pkg, sc)
    cur, last, local = _device(pkg, sc, C, L)
    r = pkg.TrackingChain(cur.cap, gate=False).track(cur, last, local, sc["pose7_pred"]).sync()
    from oracle import tracking_chain
    o = tracking_chain.track(pkg, C, L, sc["local"], sc["pose7_pred"], sc["level_sigma2"], 7, 1, gate=False)
    assert r["status"] == 0 and o["status"] == 0 and r["n1"] == o["n1"] < 20
    assert np.array_equal(r["m1"][:C.N], o["m1"]) and np.array_equal(r["m2"][:C.N], o["m2"])
    assert np.abs(r["pose2"] - o["pose2"]).max() < 1e-6


def test_tracking_chain_batch_motion_gate(pkg, synth):
    """Batch: every gate case in one call (slots in mixed order, each with its own local map), each slot
    equal to the single chain bit for bit (status included)."""
    names = ["fails_twice", "tracked", "retry_recovers", "few_map_points", "retry_exactly_20", "fails_twice"]
    scenes = [_gate_scene(synth, n)[0] for n in names]
    fr = [_frames(pkg, sc) for sc in scenes]
    cap = max(max(C.N, L.N) for C, L in fr) + 3
    devs = [_device(pkg, sc, C, L, cap=cap) for sc, (C, L) in zip(scenes, fr)]
    single = [pkg.TrackingChain(cap).track(cur, last, local, sc["pose7_pred"]).sync()
              for sc, (cur, last, local) in zip(scenes, devs)]
    batch = pkg.TrackingChainBatch(cap, len(names))
    res = batch.track([(cur, last, local, sc["pose7_pred"]) for sc, (cur, last, local) in zip(scenes, devs)]).sync()
    for n, r, o in zip(names, res, single):
        assert r["status"] == o["status"] == GATE_SCENES[n][1], n
        for k in ("n1", "n2", "n_kept", "n_map"):
            assert r[k] == o[k], (n, k)
        for k in ("m1", "m2", "edge_kp1", "edge_kp2", "outlier1", "outlier2", "inliers"):
            assert np.array_equal(np.asarray(r[k]), np.asarray(o[k])), (n, k)
        assert np.array_equal(r["pose1"], o["pose1"]) and np.array_equal(r["pose2"], o["pose2"]), n
    batch.release()


def test_tracking_chain_batch_rejects_shared_local_map(pkg, synth):
    """isInFrustum writes each slot's local map, so one map in two slots of a call is refused."""
    sc = synth.tracking_chain_scene(seed=82)
    C, L = _frames(pkg, sc)
    cur, last, local = _device(pkg, sc, C, L)
    with pytest.raises(ValueError, match="two slots"):
        pkg.TrackingChainBatch(cur.cap, 2).track([(cur, last, local, sc["pose7_pred"])] * 2)


def test_tracking_chain_batch_forms(pkg, synth, monkeypatch):
    """The batch's alternative forms against the single chain: a cap above the LDS-staged candidate
    passes' limit (the frame's records no longer fit one workgroup: the thread form runs) and the
    two-frames-per-CU PoseOptimization (forced; batches of >= 512 frames take it by themselves)."""
    scenes = [synth.tracking_chain_scene(seed=s) for s in (81, 83)]
    fr = [_frames(pkg, sc) for sc in scenes]
    for cap, dual in ((3000, None), (max(max(C.N, L.N) for C, L in fr) + 3, "1")):
        devs = [_device(pkg, sc, C, L, cap=cap) for sc, (C, L) in zip(scenes, fr)]
        single = [pkg.TrackingChain(cap).track(cur, last, local, sc["pose7_pred"]).sync()
                  for sc, (cur, last, local) in zip(scenes, devs)]
        if dual:
            monkeypatch.setenv("ORBGPU_POSE_DUAL", dual)
        res = pkg.TrackingChainBatch(cap, len(scenes)).track(
            [(cur, last, local, sc["pose7_pred"]) for sc, (cur, last, local) in zip(scenes, devs)]).sync()
        monkeypatch.delenv("ORBGPU_POSE_DUAL", raising=False)
        for r, o in zip(res, single):
            for k in ("n1", "n2", "n_kept", "n_map"):
                assert r[k] == o[k], (cap, k)
            for k in ("m1", "m2", "edge_kp1", "edge_kp2"):
                assert np.array_equal(np.asarray(r[k]), np.asarray(o[k])), (cap, k)
            if dual:  # another kernel build: the 1e-6 PoseOptimization bar, identical outlier flags
                for k in ("outlier1", "outlier2", "inliers"):
                    assert np.array_equal(np.asarray(r[k]), np.asarray(o[k])), (cap, k)
                for k in ("pose1", "pose2"):
                    assert np.sqrt(np.mean((np.asarray(r[k]) - np.asarray(o[k])) ** 2)) < 1e-6, (cap, k)
            else:
                for k in ("outlier1", "outlier2", "inliers", "pose1", "pose2"):
                    assert np.array_equal(np.asarray(r[k]), np.asarray(o[k])), (cap, k)
