"""The benched workloads themselves, checked frame by frame against the oracle.

bench.py times C2 as 64 frames (seeds 100..163) with four extractor handles taking the steps in
turn on their own streams, each batch one chain on its handle's stream (set_overlap(False)), so one batch's quad-tree/describe tail runs beside the next batch's
pyramid/FAST, with the pyramid launch stamps on (profile "pyramid_launches").  The C4 line runs
32 frames of 1280x720 per GPU the same way.  Both are reproduced here at full size and every frame
of every handle is compared with the CPU oracle: keypoints bitwise, descriptors, monoIndex.

LocalBA beyond the C5 window: 80 and 200 free keyframes (n = 480 and 1200 pose unknowns), above the
register-resident Cholesky's 288, against the oracle at the 1e-6 pose RMSE bar.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run_in_flight(pkg, imgs, nf, w, h, lap, steps=8, handles=4, stamps=True):
    """bench.py's timed loop: `handles` extractors on their own streams, step i on handle i % handles."""
    import torch
    b = imgs.shape[0]
    exs = [pkg.ORBextractor(nf, 1.2, 8, 20, 7, max_width=w, max_height=h, max_batch=b) for _ in range(handles)]
    cap = nf + 16 * 8
    outs = [(torch.empty((b, cap, 7), dtype=torch.float32, device=imgs.device),
             torch.empty((b, cap, 32), dtype=torch.uint8, device=imgs.device),
             torch.empty((b, 2), dtype=torch.int32, device=imgs.device)) for _ in range(handles)]
    streams = [torch.cuda.Stream() for _ in range(handles)]
    if handles > 1:  # bench.throughput_mode: one chain per batch on its handle's stream
        for e in exs:
            e.set_overlap(False)
    if stamps:
        for e in exs:
            e.profile("pyramid_launches")
    for i in range(steps):
        exs[i % handles].extract_batch_device(imgs, lap, cap=cap, out=outs[i % handles], stream=streams[i % handles])
    torch.cuda.synchronize()
    for e in exs:
        assert e._lib.orb_debug_status(e._h) == 0
        if stamps:
            ms, n = e.pyramid_launch_ms()
            # 8 levels: 8 level passes, or 4 two-level passes (k_pyramid_pair) with ORBGPU_PYR_PAIR=1
            per_batch = {"1": 4, "2": 7}.get(os.environ.get("ORBGPU_PYR_PAIR", "0"), 8)
            assert n == per_batch * (steps // handles) and ms > 0
            e.profile(False)
    return outs


def _check_against_oracle(pkg, oracle, frames, outs, nf, lap, golden_names=()):
    """Every frame of every handle against the live oracle, and the frames named in golden_names against
    the committed records (tests/golden/extract.json) as well."""
    from golden import fixtures as fx
    golden = fx.load_json("extract.json")
    ref = oracle.OracleExtractor(nf, 1.2, 8, 20, 7)
    counts = [o[2].cpu().numpy() for o in outs]
    total = 0
    for f in range(len(frames)):
        rk, rd, rm = ref(frames[f], lap)
        for hnd, (kps, desc, _) in enumerate(outs):
            n = int(counts[hnd][f, 0])
            assert n == len(rk) and int(counts[hnd][f, 1]) == rm, f"handle {hnd} frame {f}: count/monoIndex"
            gk = pkg.keypoints_to_structured(kps[f], n)
            gd = desc[f, :n].cpu().numpy()
            assert np.array_equal(gk.view(np.uint8), rk.view(np.uint8)), f"handle {hnd} frame {f} keypoints"
            assert np.array_equal(gd, rd), f"handle {hnd} frame {f} descriptors"
            if f < len(golden_names):
                fx.check_extract(golden[golden_names[f]], frames[f], gk, gd, int(counts[hnd][f, 1]),
                                 f"handle {hnd} {golden_names[f]}")
        total += len(rk)
    return total


def test_c2_as_benched(pkg, oracle, synth):
    """C2 exactly as bench.py runs it: 64 frames (seeds 100..163), 4 handles in flight, 8 steps."""
    import torch
    frames = np.stack([synth.polygon_frame(640, 480, seed=100 + i) for i in range(64)])
    outs = _run_in_flight(pkg, torch.from_numpy(frames).cuda(), 1000, 640, 480, (0, 1000))
    total = _check_against_oracle(pkg, oracle, frames, outs, 1000, (0, 1000), [f"c2_seed{100 + i}" for i in range(64)])
    assert total > 60000


def test_c4_shard_as_benched(pkg, oracle, synth):
    """C4's per-GPU shard: 32 frames of 1280x720 (seeds 1000..1031), 4 handles in flight."""
    import torch
    frames = np.stack([synth.polygon_frame(1280, 720, seed=1000 + i) for i in range(32)])
    outs = _run_in_flight(pkg, torch.from_numpy(frames).cuda(), 1000, 1280, 720, (0, 1000), stamps=False)
    _check_against_oracle(pkg, oracle, frames, outs, 1000, (0, 1000), [f"c4_seed{1000 + i}" for i in range(4)])


def _rmse(a, b):
    return float(np.sqrt(np.mean((np.asarray(a) - np.asarray(b)) ** 2)))


@pytest.mark.parametrize("n_kf,n_points,stereo_frac", [(82, 3200, 0.0), (82, 3200, 0.5), (202, 6000, 0.0)],
                         ids=["80free_mono", "80free_mixed", "200free_mono"])
def test_local_ba_large_window(pkg, oracle, synth, n_kf, n_points, stereo_frac):
    """Local windows above C5's 48 free keyframes (the reference's window is every covisible
    keyframe, src/Optimizer.cc:1752-1760, and is unbounded)."""
    prob = synth.local_ba_problem(n_kf=n_kf, n_points=n_points, obs_per_point=6, stereo_frac=stereo_frac, seed=17)
    solver = pkg.LocalBA()
    pose, point, chi2, depth, res = solver.optimize(prob, 10)
    rpose, rpoint, rchi2, rdepth, rres = oracle.local_ba(prob, 10)
    for k in ("iterations", "trials", "terminated", "stopped"):
        assert res[k] == rres[k], f"{k}: {res[k]} vs oracle {rres[k]}"
    assert _rmse(pose[:, :3], rpose[:, :3]) < 1e-6
    q, rq = pose[:, 3:], rpose[:, 3:]
    q = np.where((np.sum(q * rq, axis=1) < 0)[:, None], -q, q)
    assert _rmse(q, rq) < 1e-6
    assert _rmse(point, rpoint) < 1e-6
    assert np.array_equal(depth, rdepth)
    if stereo_frac == 0:
        assert np.allclose(chi2, rchi2, rtol=1e-9, atol=1e-12)
    else:
        assert np.allclose(chi2, rchi2, rtol=1e-6, atol=1e-3)
    assert res["final_chi2"] < res["initial_chi2"]
