"""Calls on different handles and streams running at the same time (the ABI is re-entrant across
handles: Tracking and LocalMapping call it from their own threads, and bench.py keeps several batches
in flight).  Each concurrent result must equal the same call made alone; the per-call scratch of the
stereo, pose and BoW batch paths is stream-ordered, not shared."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EUROC_BF, EUROC_B = 47.90639384423901, 0.110074


def test_stereo_batches_on_two_streams(pkg, synth):
    import torch
    sets = []
    for k in range(2):
        pairs = [synth.stereo_pair(752, 480, seed=500 + 10 * k + i) for i in range(4)]
        L = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
        R = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
        exl = pkg.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480, max_batch=4)
        exr = pkg.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480, max_batch=4)
        sets.append((L, R, exl, exr, torch.cuda.Stream()))

    def run(L, R, exl, exr, st):
        with torch.cuda.stream(st):
            ol = exl.extract_batch_device(L, (0, 0), stream=st)
            orr = exr.extract_batch_device(R, (0, 0), stream=st)
            return ol[2], pkg.compute_stereo_matches_batch_device(exl, exr, ol, orr, EUROC_BF, EUROC_B, stream=st)

    def host(res):  # (per frame: u_right and depth bits of the frame's keypoints, kept)
        u, d, kept = [t.cpu().numpy() for t in res[1]]
        counts = res[0].cpu().numpy()
        return [(u[f, :counts[f, 0]].view(np.uint32).copy(), d[f, :counts[f, 0]].view(np.uint32).copy(), int(kept[f]))
                for f in range(len(counts))]
    alone = []
    for s in sets:
        r = run(*s)
        torch.cuda.synchronize()
        alone.append(host(r))
    for _ in range(3):
        both = [run(*s) for s in sets]  # enqueued back to back on the two streams
        torch.cuda.synchronize()
        for a, b in zip(alone, both):
            for (u0, d0, k0), (u1, d1, k1) in zip(a, host(b)):
                assert k0 == k1 and np.array_equal(u0, u1) and np.array_equal(d0, d1)


def test_pose_batches_on_two_streams(pkg, synth):
    import torch
    lib = pkg._lib.load()
    jobs = []
    for k in range(2):
        frames, edges, _ = synth.pose_opt_batch(16, 600 + 300 * k, stereo_frac=0.5, seed=60 + k)
        d_fr = torch.from_numpy(frames.view(np.uint8).reshape(-1)).cuda()
        d_ed = torch.from_numpy(edges.view(np.uint8).reshape(-1)).cuda()
        outs = (torch.empty((len(frames), 7), dtype=torch.float64, device="cuda"),
                torch.empty(len(edges), dtype=torch.uint8, device="cuda"),
                torch.empty(len(frames), dtype=torch.int32, device="cuda"))
        jobs.append((len(frames), d_fr, len(edges), d_ed, outs, torch.cuda.Stream()))

    def run(nf, d_fr, ne, d_ed, outs, st):
        pkg._lib.check(lib.orb_pose_optimization_device(nf, d_fr.data_ptr(), ne, d_ed.data_ptr(), outs[0].data_ptr(),
                                                        outs[1].data_ptr(), outs[2].data_ptr(),
                                                        ctypes.c_void_p(st.cuda_stream)), "pose")
    alone = []
    for j in jobs:
        run(*j)
        torch.cuda.synchronize()
        alone.append([t.cpu().numpy().copy() for t in j[4]])
    for _ in range(3):
        for j in jobs:
            run(*j)
        torch.cuda.synchronize()
        for a, j in zip(alone, jobs):
            for x, y in zip(a, j[4]):
                assert np.array_equal(x, y.cpu().numpy())
