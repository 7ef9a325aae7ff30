import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
from conftest import load_package
pkg = load_package()
from orbslam3_amd import synth
import test_tracking_chain_gpu as T
for B in (1, 2):
    seeds = (81, 82)[:B]
    scenes = [synth.tracking_chain_scene(seed=s, stereo=True) for s in seeds]
    fr = [T._frames(pkg, sc) for sc in scenes]
    cap = max(max(C.N, L.N) for C, L in fr) + 37
    devs = [T._device(pkg, sc, C, L, cap=cap) for sc, (C, L) in zip(scenes, fr)]
    single = []
    for sc, (cur, last, local) in zip(scenes, devs):
        ch = pkg.TrackingChain(cap, th_motion=7, th_local=1)
        single.append(ch.track(cur, last, local, sc["pose7_pred"]).sync())
    batch = pkg.TrackingChainBatch(cap, B, th_motion=7, th_local=1)
    res = batch.track([(cur, last, local, sc["pose7_pred"]) for sc, (cur, last, local) in zip(scenes, devs)]).sync()
    for b, (r, o) in enumerate(zip(res, single)):
        N = fr[b][0].N
        cnt_b = int(((r["m1"][:N] >= 0) | (r["m2"][:N] >= 0)).sum())
        cnt_o = int(((o["m1"][:N] >= 0) | (o["m2"][:N] >= 0)).sum())
        print("B", B, "b", b, "n_edges2", r["frames"][1]["n_edges"], o["frames"][1]["n_edges"], "count", cnt_b, cnt_o,
              "n_edges1", r["frames"][0]["n_edges"], o["frames"][0]["n_edges"], "kept", r["n_kept"], o["n_kept"],
              "n1", r["n1"], o["n1"], "outl1", r["outlier1"].sum(), o["outlier1"].sum())
        k = min(len(r["edge_kp2"]), len(o["edge_kp2"]))
        d = np.nonzero(r["edge_kp2"][:k] != o["edge_kp2"][:k])[0]
        print("  first kp2 diff", d[:5], r["edge_kp2"][d[:3]] if len(d) else None, o["edge_kp2"][d[:3]] if len(d) else None)
        print("  raw m1 count>=0", int((r["m1"][:N] >= 0).sum()), int((o["m1"][:N] >= 0).sum()))
