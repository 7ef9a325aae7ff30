"""The C3 chain device-resident end to end (BASELINE configs[2]): stereo extraction of a keyframe stream
(orb_extract_batch_device, left and right), Frame::ComputeStereoMatches (orb_compute_stereo_matches_batch_device),
KeyFrame::ComputeBoW (orb_bow_transform_frames_device) and LocalMapping::CreateNewMapPoints'
SearchForTriangulation against the covisible keyframes (orb_search_for_triangulation_device,
src/LocalMapping.cc:536-610), with no host hop between the stages.  Compared with the same chain on
the oracle: every match and count bit-exact, plus the BoW outputs of the intermediate stage."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EUROC_BF, EUROC_B = 47.90639384423901, 0.110074
FLAGS = [(0, 0, 0), (0, 0, 1), (1, 0, 1), (0, 1, 0)]


@pytest.fixture(scope="module")
def chain(pkg, synth, oracle):
    import torch
    n = 6
    L, R, Tcw, _ = synth.stereo_sequence(n, seed=214)
    voc = synth.dbow_vocabulary(10, 6, seed=61)
    scale, sigma2 = synth.scale_tables()
    rng = np.random.default_rng(3)
    exl = pkg.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480, max_batch=8)
    exr = pkg.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480, max_batch=8)
    vocab = pkg.ORBVocabulary(voc)
    out_l = exl.extract_batch_device(torch.from_numpy(L).cuda(), (0, 0))
    out_r = exr.extract_batch_device(torch.from_numpy(R).cuda(), (0, 0))
    u, _, _ = pkg.compute_stereo_matches_batch_device(exl, exr, out_l, out_r, EUROC_BF, EUROC_B)
    bow = vocab.transform_frames_device(out_l[1], out_l[2], 4)
    cap = out_l[0].shape[1]
    has_mp = (rng.random((n, cap)) < 0.2).astype(np.uint8)
    hm = torch.from_numpy(has_mp).cuda()
    dev = [pkg.DeviceKeyFrame(out_l, bow, f, Tcw[f], synth.EUROC_K, scale, sigma2, u_right=u, has_mappoint=hm)
           for f in range(n)]
    # the oracle chain
    ref = []
    for f in range(n):
        exa, exb = oracle.OracleExtractor(1200, 1.2, 8, 20, 7), oracle.OracleExtractor(1200, 1.2, 8, 20, 7)
        kl, dl, _ = exa(L[f], (0, 0))
        kr, dr, _ = exb(R[f], (0, 0))
        p = exa.params()
        ur, _, _ = oracle.compute_stereo_matches(kl, dl, kr, dr, [exa.level_padded(l) for l in range(8)],
                                                 [exb.level_padded(l) for l in range(8)], p["scale"], p["inv_scale"],
                                                 EUROC_BF, EUROC_B)
        rbow, fv = oracle.bow_transform(voc, dl, 4)
        ref.append((pkg.KeyFrame(keys_un=kl, descriptors=dl, Tcw=Tcw[f], camera=synth.EUROC_K, scale_factors=scale,
                                 level_sigma2=sigma2, u_right=ur, has_mappoint=has_mp[f, :len(kl)], feat_vec=fv), rbow))
    torch.cuda.synchronize()
    sides = {"left": (L, [t.cpu().numpy() for t in out_l]), "right": (R, [t.cpu().numpy() for t in out_r])}
    return dict(dev=dev, ref=ref, bow=[t.cpu().numpy() for t in bow], counts=out_l[2].cpu().numpy(), n=n, sides=sides)


def test_chain_extraction_golden(pkg, chain):
    """The chain's device extraction of both sides of every stereo keyframe against the committed
    records (tests/golden/extract.json, c3_left* / c3_right*)."""
    from golden import fixtures as fx
    golden = fx.load_json("extract.json")
    for side, (imgs, (kps, desc, counts)) in chain["sides"].items():
        for f in range(chain["n"]):
            n = int(counts[f, 0])
            k = np.ascontiguousarray(kps[f, :n]).view(np.uint8).reshape(n, 28).view(pkg.KEYPOINT_DTYPE).reshape(n)
            fx.check_extract(golden[f"c3_{side}{f}"], imgs[f], k, desc[f, :n], int(counts[f, 1]), f"c3_{side}{f}")


def test_chain_bow_stage(chain):
    """The FeatureVector the SearchForTriangulation stage reads, on the extractor's layout, equals the oracle's."""
    fv_node, fv_begin, fv_feat, cnt = chain["bow"][2], chain["bow"][3], chain["bow"][4], chain["bow"][5]
    bw, bv = chain["bow"][0], chain["bow"][1]
    for f, (k, rbow) in enumerate(chain["ref"]):
        assert int(chain["counts"][f, 0]) == k.N
        nn = int(cnt[f, 1])
        fv = {int(fv_node[f, j]): [int(x) for x in fv_feat[f, fv_begin[f, j]:fv_begin[f, j + 1]]] for j in range(nn)}
        assert fv == k.mFeatVec
        assert {int(bw[f, i]): float(bv[f, i]) for i in range(int(cnt[f, 0]))} == rbow


@pytest.mark.parametrize("only_stereo,coarse,check_ori", FLAGS)
def test_chain_search_for_triangulation(pkg, oracle, chain, only_stereo, coarse, check_ori):
    import torch
    n = chain["n"]
    from golden import fixtures as fx
    golden = fx.load_json("sft_c3.json")
    m = pkg.ORBmatcher(0.6, bool(check_ori))
    for k1 in (n - 1, 0):  # the newest keyframe against its predecessors, and the oldest against the rest
        nbrs = [f for f in range(n) if f != k1]
        m12, cnt = m.SearchForTriangulationDevice(chain["dev"][k1], [chain["dev"][f] for f in nbrs], only_stereo, coarse)
        torch.cuda.synchronize()
        m12, cnt = m12.cpu().numpy(), cnt.cpu().numpy()
        r1 = chain["ref"][k1][0]
        total = 0
        for p, f in enumerate(nbrs):
            r2 = chain["ref"][f][0]
            rn, rm = oracle.search_for_triangulation(r1, r2, m.pair_geometry(r1, r2), only_stereo, coarse, check_ori)
            assert cnt[p] == rn, (k1, f, cnt[p], rn)
            assert np.array_equal(m12[p, :r1.N], rm), (k1, f, int((m12[p, :r1.N] != rm).sum()))
            assert (m12[p, r1.N:] == -1).all()
            rec = golden[fx.sft_key(k1, f, (only_stereo, coarse, check_ori))]
            assert rec == {"n": int(cnt[p]), "matches_sha256": fx.sha(np.asarray(m12[p, :r1.N], np.int32))}, (k1, f)
            total += rn
        assert total > 0


def test_chain_device_matches_host_call(pkg, chain):
    """The device form equals orb_search_for_triangulation on the downloaded keyframes."""
    import torch
    n = chain["n"]
    m = pkg.ORBmatcher(0.6, False)
    m12, cnt = m.SearchForTriangulationDevice(chain["dev"][n - 1], chain["dev"][:n - 1], False, False)
    torch.cuda.synchronize()
    got = m.SearchForTriangulationMany(chain["ref"][n - 1][0], [r[0] for r in chain["ref"][:n - 1]], False, False)
    for p, (c, mm) in enumerate(got):
        assert int(cnt[p]) == c and np.array_equal(m12[p, :len(mm)].cpu().numpy(), mm)


def test_chain_batched_keyframes(pkg, chain):
    """Several new keyframes with their neighbours in one launch equal one call per keyframe."""
    import torch
    n = chain["n"]
    dev = chain["dev"]
    m = pkg.ORBmatcher(0.6, True)
    groups = [(dev[n - 1], dev[:n - 1]), (dev[2], [dev[0], dev[1], dev[3]]), (dev[0], dev[1:])]
    m12, cnt = m.SearchForTriangulationDeviceBatch(groups, False, False)
    torch.cuda.synchronize()
    p = 0
    for k1, nb in groups:
        a, c = m.SearchForTriangulationDevice(k1, nb, False, False)
        torch.cuda.synchronize()
        assert torch.equal(cnt[p:p + len(nb)], c) and torch.equal(m12[p:p + len(nb), :k1.cap], a)
        p += len(nb)


def test_chain_capacity_overflow(pkg, synth, oracle):
    """A caller-chosen cap below a frame's keypoint count: the extractor flags the frame
    ORB_ERR_CAPACITY, the BoW transform does not read its slice and reports ORB_ERR_CAPACITY, and every
    SearchForTriangulation pair with it reports ORB_ERR_CAPACITY with no matches; the frames that fit
    are unaffected and still equal the oracle chain."""
    import torch
    L, _, Tcw, _ = synth.stereo_sequence(3, seed=214)
    imgs = L.copy()
    for f in (1, 2):  # small textured windows: few keypoints, under the cap
        flat = np.full_like(imgs[f], 128)
        flat[140:300, 200:420] = imgs[f][140:300, 200:420]
        imgs[f] = flat
    voc = synth.dbow_vocabulary(10, 4, seed=61)
    scale, sigma2 = synth.scale_tables()
    ex = pkg.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480, max_batch=4)
    vocab = pkg.ORBVocabulary(voc)
    ref = [oracle.OracleExtractor(1200, 1.2, 8, 20, 7)(imgs[f], (0, 0)) for f in range(3)]
    cap = max(len(ref[1][0]), len(ref[2][0])) + 8
    assert len(ref[0][0]) > cap
    out = ex.extract_batch_device(torch.from_numpy(imgs).cuda(), (0, 0), cap=cap)
    bow = vocab.transform_frames_device(out[1], out[2], 4)
    torch.cuda.synchronize()
    counts, bcounts = out[2].cpu().numpy(), bow[5].cpu().numpy()
    assert counts[0, 0] == len(ref[0][0]) and counts[0, 1] == pkg._lib.ORB_ERR_CAPACITY
    assert (bcounts[0] == pkg._lib.ORB_ERR_CAPACITY).all()
    kfs, dev = [], []
    for f in (1, 2):
        assert counts[f, 0] == len(ref[f][0]) and counts[f, 1] >= 0
        rbow, fv = oracle.bow_transform(voc, ref[f][1], 4)
        nn = int(bcounts[f, 1])
        fvn, fvb, fvf = bow[2][f].cpu().numpy(), bow[3][f].cpu().numpy(), bow[4][f].cpu().numpy()
        assert {int(fvn[j]): [int(x) for x in fvf[fvb[j]:fvb[j + 1]]] for j in range(nn)} == fv
        kfs.append(pkg.KeyFrame(keys_un=ref[f][0], descriptors=ref[f][1], Tcw=Tcw[f], camera=synth.EUROC_K,
                                scale_factors=scale, level_sigma2=sigma2, feat_vec=fv))
    dev = [pkg.DeviceKeyFrame(out, bow, f, Tcw[f], synth.EUROC_K, scale, sigma2) for f in range(3)]
    m = pkg.ORBmatcher(0.6, True)
    for k1, nbrs in ((1, (0, 2)), (0, (1, 2))):
        m12, cnt = m.SearchForTriangulationDevice(dev[k1], [dev[f] for f in nbrs], False, True)
        torch.cuda.synchronize()
        m12, cnt = m12.cpu().numpy(), cnt.cpu().numpy()
        for p, f in enumerate(nbrs):
            if 0 in (k1, f):
                assert cnt[p] == pkg._lib.ORB_ERR_CAPACITY and (m12[p] == -1).all(), (k1, f)
                continue
            r1, r2 = kfs[k1 - 1], kfs[f - 1]
            rn, rm = oracle.search_for_triangulation(r1, r2, m.pair_geometry(r1, r2), False, True, True)
            assert cnt[p] == rn and np.array_equal(m12[p, :r1.N], rm), (k1, f, cnt[p], rn)
