"""World-size-2 gloo tests of the multi-GPU path on CPU: frame sharding and the feature all-gather.

The extraction itself needs the GPU; here each rank fills its blocks with a deterministic function
of the global frame index.  The test checks that after all_gather_features every rank holds every
frame's blocks in global frame order, and that shard_range covers the batch exactly once.
"""
from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fill(frame, cap):
    g = torch.Generator().manual_seed(1000 + frame)
    desc = torch.randint(0, 256, (cap, 32), generator=g, dtype=torch.uint8)
    kps = torch.randn((cap, 7), generator=g)
    cnt = torch.tensor([cap - frame % 7, frame], dtype=torch.int32)
    return kps, desc, cnt


def _worker(rank, world, port, total, cap, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from conftest import load_package
        pkg = load_package()
        from orbslam3_amd import distributed as D
        b, e = D.shard_range(total, world, rank)
        per = -(-total // world)  # blocks are padded to the largest shard
        kps = torch.zeros((per, cap, 7))
        desc = torch.zeros((per, cap, 32), dtype=torch.uint8)
        cnt = torch.full((per, 2), -1, dtype=torch.int32)
        for i, f in enumerate(range(b, e)):
            kps[i], desc[i], cnt[i] = _fill(f, cap)
        g_kps, g_desc, g_cnt = D.all_gather_features(kps, desc, cnt)
        ok = True
        for r in range(world):
            rb, re_ = D.shard_range(total, world, r)
            for i, f in enumerate(range(rb, re_)):
                k, d, c = _fill(f, cap)
                j = r * per + i
                ok &= bool(torch.equal(g_desc[j], d) and torch.equal(g_kps[j], k) and torch.equal(g_cnt[j], c))
                ok &= bool(torch.equal(D.frame_descriptors(g_desc, g_cnt, j), d[: int(c[0])]))
        # async form returns the same data
        a_kps, a_desc, a_cnt, works = D.all_gather_features(kps, desc, cnt, async_op=True)
        for w in works:
            w.wait()
        ok &= bool(torch.equal(a_desc, g_desc) and torch.equal(a_cnt, g_cnt))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("total", [8, 11])
def test_all_gather_features_gloo_world2(pkg, total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, total, 24, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


def test_shard_range(pkg):
    from orbslam3_amd import distributed as D
    for total in (1, 7, 64, 256, 257):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                b, e = D.shard_range(total, world, r)
                assert 0 <= e - b <= -(-total // world)
                seen.extend(range(b, e))
            assert seen == list(range(total))


def _reducer_worker(rank, world, port, q):
    import ctypes

    import numpy as np
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from conftest import load_package
        load_package()
        from orbslam3_amd import optimizer as O
        cb = O.make_host_reducer()
        a = np.arange(5, dtype=np.float64) * (rank + 1)
        rc1 = cb(None, a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), 5, O.BA_SUM)
        b = np.array([rank, -rank, 0.5], dtype=np.float64)
        rc2 = cb(None, b.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), 3, O.BA_MAX)
        s = sum(r + 1 for r in range(world))
        ok = rc1 == 0 and rc2 == 0 and np.array_equal(a, np.arange(5) * s) and \
            np.array_equal(b, [world - 1, 0, 0.5])
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_ba_host_reducer_gloo_world2(pkg):
    """The orb_ba_host_reduce_fn callback the sharded LocalBA uses on gloo groups: in-place SUM and
    MAX of the library's float64 host buffer, called through ctypes as the library calls it."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_reducer_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


def _np_knn2(query, train):
    """Reference scan (src/ORBmatcher.cc:1160-1175 order): best, first index of it, second smallest."""
    import numpy as np
    q, t = query.numpy(), train.numpy()
    n = q.shape[0]
    if n == 0:
        z = torch.zeros(0, dtype=torch.int32)
        return z, z.clone(), z.clone()
    pc = np.unpackbits(np.arange(256, dtype=np.uint8)[:, None], axis=1).sum(1).astype(np.int32)
    D = pc[q[:, None, :] ^ t[None, :, :]].sum(axis=2)
    srt = np.sort(D, axis=1)
    second = srt[:, 1] if t.shape[0] > 1 else np.full(n, 257)
    return (torch.from_numpy(np.argmin(D, axis=1).astype(np.int32)), torch.from_numpy(srt[:, 0].astype(np.int32)),
            torch.from_numpy(second.astype(np.int32)))


def _knn_worker(rank, world, port, nq, nt, q_out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from conftest import load_package
        load_package()
        from orbslam3_amd import distributed as D
        g = torch.Generator().manual_seed(77)
        query = torch.randint(0, 256, (nq, 32), generator=g, dtype=torch.uint8)
        train = torch.randint(0, 256, (nt, 32), generator=g, dtype=torch.uint8)
        train[5] = query[min(3, nq - 1)]
        try:
            idx, d1, d2 = D.distributed_knn2(query, train, local_fn=_np_knn2)
            ridx, rd1, rd2 = _np_knn2(query, train)
            q_out.put((rank, bool(torch.equal(idx, ridx) and torch.equal(d1, rd1) and torch.equal(d2, rd2))))
        except Exception as e:  # noqa: BLE001 -- reported, not left to the queue timeout
            q_out.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("nq,nt", [(1000, 300), (7, 50), (1, 20)])
def test_distributed_knn2_query_split_gloo_world2(pkg, nq, nt):
    """SURVEY.md 8(e) Hamming matching: the query rows split over 2 ranks (one rank may get none) and
    the per-query (best index, best, second) all-gathered equal the single-device scan on every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_knn_worker, args=(r, 2, port, nq, nt, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


def _np_knn2_any(query, train):
    """_np_knn2 with an empty train set allowed (no match: -1, 257, 257)."""
    if train.shape[0] == 0:
        n = query.shape[0]
        return (torch.full((n,), -1, dtype=torch.int32), torch.full((n,), 257, dtype=torch.int32),
                torch.full((n,), 257, dtype=torch.int32))
    return _np_knn2(query, train)


def _match_worker(rank, world, port, total, cap, q_out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from conftest import load_package
        load_package()
        from orbslam3_amd import distributed as D
        per = total // world
        b = rank * per
        kps = torch.zeros((per, cap, 7))
        desc = torch.zeros((per, cap, 32), dtype=torch.uint8)
        cnt = torch.zeros((per, 2), dtype=torch.int32)
        for i in range(per):
            kps[i], desc[i], cnt[i] = _fill(b + i, cap)
        g_kps, g_desc, g_cnt = D.all_gather_features(kps, desc, cnt)
        pairs = D.frame_pairs(b, per, total)
        idx, d1, d2 = D.match_gathered(g_desc, g_cnt, pairs, local_fn=_np_knn2_any)
        ok = True
        for i in range(per):  # the single-process scan of frame f against its predecessor
            f = b + i
            _, qd, qc = _fill(f, cap)
            _, td, tc = _fill((f - 1) % total, cap)
            n = int(qc[0])
            ri, r1, r2 = _np_knn2_any(qd[:n], td[: int(tc[0])])
            ok &= bool(torch.equal(idx[i, :n], ri) and torch.equal(d1[i, :n], r1) and torch.equal(d2[i, :n], r2))
            ok &= bool((idx[i, n:] == -1).all() and (d1[i, n:] == 257).all())
        ok &= pairs.tolist() == [[b + i, (b + i - 1) % total] for i in range(per)]
        q_out.put((rank, ok))
    except Exception as e:  # noqa: BLE001 -- reported, not left to the queue timeout
        q_out.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_gather_then_cross_frame_match_gloo_world2(pkg):
    """C4 with matching: each rank extracts (here: fills) its frames, all-gathers every rank's blocks,
    then matches its own frames against their predecessors in the gathered set; the result equals the
    single-process scan of the same pairs (frame 0's predecessor, the last frame, lives on the other rank)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_match_worker, args=(r, 2, port, 8, 24, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}
