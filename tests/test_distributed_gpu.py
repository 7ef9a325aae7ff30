"""GPU check of the sharded extractor's data path on one rank (RCCL group of size 1).

The gathered blocks must equal a direct batched extraction of the same frames, and the cross-frame
knn2 on the gathered descriptors must run on the device.  World sizes > 1 are covered by the gloo
tests in test_distributed_cpu.py and by bench.py --gpus N.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharded_extractor_single_rank(pkg, synth, oracle):
    import torch
    import torch.distributed as dist
    from orbslam3_amd import distributed as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        frames = torch.from_numpy(synth.frame_batch(4, 640, 480, seed0=500)).cuda()
        ex = pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=640, max_height=480, max_batch=4)
        sh = D.ShardedExtractor(ex, 4)
        assert sh.step(frames, (0, 1000)) is None
        g_kps, g_desc, g_cnt = sh.finish()
        kps, desc, cnt = ex.extract_batch_device(frames, (0, 1000), cap=sh.cap)
        torch.cuda.synchronize()
        assert torch.equal(g_cnt, cnt)
        for f in range(4):
            n = int(cnt[f, 0])
            assert torch.equal(g_desc[f, :n], desc[f, :n])
            # int fields (octave, class_id = -1) are punned into the float rows: compare bits
            assert torch.equal(g_kps[f, :n].view(torch.int32), kps[f, :n].view(torch.int32))
        # cross-frame matching against the gathered set: frame 0 vs frame 1
        q = D.frame_descriptors(g_desc, g_cnt, 0).contiguous()
        t = D.frame_descriptors(g_desc, g_cnt, 1).contiguous()
        idx, d1, d2 = pkg.ORBmatcher.knn2_device(q, t)
        qa, ta = q.cpu().numpy(), t.cpu().numpy()
        D_ = np.unpackbits(qa[:16, None, :] ^ ta[None, :, :], axis=2).sum(axis=2)
        assert np.array_equal(d1.cpu().numpy()[:16], D_.min(axis=1))
        # cross-frame matching of every frame against its predecessor, one launch over the gathered
        # blocks (match=True), equals the oracle scan pair by pair
        shm = D.ShardedExtractor(ex, 4, match=True)
        shm.step(frames, (0, 1000))
        shm.step(frames, (0, 1000))  # matches the first step's gather
        torch.cuda.synchronize()
        idx, d1, d2 = (t.cpu().numpy() for t in shm.matches)
        cnt_h = cnt.cpu().numpy()
        for f in range(4):
            pf = (f - 1) % 4
            n, nt = int(cnt_h[f, 0]), int(cnt_h[pf, 0])
            ri, r1, r2 = oracle.hamming_knn2(desc[f, :n].cpu().numpy(), desc[pf, :nt].cpu().numpy())
            assert np.array_equal(idx[f, :n], ri) and np.array_equal(d1[f, :n], r1) and np.array_equal(d2[f, :n], r2)
            assert (idx[f, n:] == -1).all() and (d1[f, n:] == 257).all()
        first = shm.matches[0]
        shm.finish()  # the last step's gather is matched too, into the next buffer
        torch.cuda.synchronize()
        assert shm.matches[0] is not first and torch.equal(shm.matches[0], first)
        # two extractor handles in flight on their own streams (bench.py --in-flight 2): every step's
        # gathered blocks equal the direct extraction of that step's frames
        exs = [ex, pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=640, max_height=480, max_batch=4)]
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        sh2 = D.ShardedExtractor(exs, 4)
        batches = [torch.from_numpy(synth.frame_batch(4, 640, 480, seed0=600 + 10 * i)).cuda() for i in range(5)]
        got = []
        for i, b in enumerate(batches):
            r = sh2.step(b, (0, 1000), stream=streams[i % 2])
            if r is not None:
                got.append(r)
        got.append(sh2.finish(streams[1]))
        torch.cuda.synchronize()
        for b, (g_kps, g_desc, g_cnt) in zip(batches, got):
            kps, desc, cnt = ex.extract_batch_device(b, (0, 1000), cap=sh2.cap)
            torch.cuda.synchronize()
            assert torch.equal(g_cnt, cnt)
            for f in range(4):
                n = int(cnt[f, 0])
                assert torch.equal(g_desc[f, :n], desc[f, :n])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cap", [40, 1128])
def test_knn2_frames_device_vs_oracle(pkg, oracle, cap):
    """orb_hamming_knn2_frames_device: many (query frame, train frame) pairs of one block batch in one
    launch, equal to the oracle's scan per pair; empty query / train frames, a frame matched against
    itself (distance 0 at its own index), duplicated rows (first index on ties), counts at cap."""
    import torch
    rng = np.random.default_rng(cap)
    F = 6
    desc = rng.integers(0, 256, (F, cap, 32), dtype=np.uint8)
    desc[2, 7] = desc[2, 3]  # a tie inside frame 2
    cnt = np.array([[cap, 0], [cap // 2, 0], [cap - 3, 0], [0, 0], [1, 0], [cap, 0]], np.int32)
    pairs = np.array([[0, 1], [1, 0], [2, 2], [3, 0], [0, 3], [4, 5], [5, 4], [2, 0]], np.int32)
    idx, d1, d2 = pkg.ORBmatcher.knn2_frames_device(torch.from_numpy(desc).cuda(), torch.from_numpy(cnt).cuda(),
                                                   torch.from_numpy(pairs).cuda())
    torch.cuda.synchronize()
    idx, d1, d2 = idx.cpu().numpy(), d1.cpu().numpy(), d2.cpu().numpy()
    for p, (qf, tf) in enumerate(pairs):
        n, nt = cnt[qf, 0], cnt[tf, 0]
        if n:
            ri, r1, r2 = oracle.hamming_knn2(desc[qf, :n], desc[tf, :nt])
            if nt == 0:
                ri, r1, r2 = np.full(n, -1), np.full(n, 257), np.full(n, 257)
            assert np.array_equal(idx[p, :n], ri) and np.array_equal(d1[p, :n], r1) and np.array_equal(d2[p, :n], r2), p
        assert (idx[p, n:] == -1).all() and (d1[p, n:] == 257).all() and (d2[p, n:] == 257).all()
    assert (d1[2, : cnt[2, 0]] == 0).all()
