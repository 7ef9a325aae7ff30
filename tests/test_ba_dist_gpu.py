"""GPU check of the landmark-sharded LocalBA (orb_ba_dist_init_host + orb_ba_optimize).

W processes share the one GPU of the box, each attached to a gloo group with the host reducer;
every rank solves the SAME problem with 1/W of the landmarks and the partial Schur systems are
all-reduced.  The bar is the single-GPU bar against the oracle: same LM path (iterations, trials,
termination), poses and points within 1e-6 RMSE, edge chi2 and the culling decisions equal; and
all ranks return the same state.  The RCCL transport needs one GPU per rank and runs in
bench.py --gpus N.
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


def _worker(rank, world, port, kw, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from conftest import load_package
        pkg = load_package()
        from orbslam3_amd import synth
        prob = synth.local_ba_problem(**kw)
        ba = pkg.LocalBA().attach(transport="host")
        pose, point, chi2, depth, res = ba.optimize(prob, 10)
        q.put((rank, (pose, point, chi2, depth, res)))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def _run(world, kw):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kw, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r, v in out.items():
        assert not isinstance(v, str), f"rank {r}: {v}"
    return out


def _rmse(a, b):
    return float(np.sqrt(np.mean((np.asarray(a) - np.asarray(b)) ** 2)))


@pytest.mark.parametrize("world,stereo_frac,seed", [(2, 0.0, 7), (3, 0.0, 11), (2, 0.5, 8)])
def test_sharded_local_ba_matches_oracle(oracle, synth, world, stereo_frac, seed):
    kw = dict(n_kf=20, n_points=800, obs_per_point=5, stereo_frac=stereo_frac, seed=seed)
    out = _run(world, kw)
    prob = synth.local_ba_problem(**kw)
    rpose, rpoint, rchi2, rdepth, rres = oracle.local_ba(prob, 10)
    for r in range(world):
        pose, point, chi2, depth, res = out[r]
        for k in ("iterations", "trials", "terminated", "stopped"):
            assert res[k] == rres[k], f"rank {r} {k}: {res[k]} vs oracle {rres[k]}"
        assert _rmse(pose[:, :3], rpose[:, :3]) < 1e-6
        assert _rmse(point, rpoint) < 1e-6
        tol = dict(rtol=1e-9, atol=1e-12) if stereo_frac == 0 else dict(rtol=1e-6, atol=1e-3)
        assert np.allclose(chi2, rchi2, **tol)
        assert np.array_equal(depth, rdepth)
        # every rank holds the same result
        assert np.array_equal(pose, out[0][0]) and np.array_equal(point, out[0][1])
        assert np.array_equal(chi2, out[0][2])


def _rccl_one_rank_worker(port, kw, q):
    """One rank with an RCCL communicator forced onto the sharded path (ORBGPU_BA_DIST_FORCE=1): the
    device LM loop with its all-reduces as real RCCL calls, next to a plain single-GPU handle running the
    6-launch unit the sharded loop shares its arithmetic with (ORBGPU_BA_FAST_UNIT=0; the default fast
    unit sums in another order and is checked against the oracle by tests/test_ba_gpu.py)."""
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ORBGPU_BA_DIST_FORCE="1",
                      ORBGPU_BA_FAST_UNIT="0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        from conftest import load_package
        pkg = load_package()
        from orbslam3_amd import synth
        prob = synth.local_ba_problem(**kw)
        sharded = pkg.LocalBA().attach(transport="rccl")
        a = sharded.optimize(prob, 10)
        b = pkg.LocalBA().optimize(prob, 10)
        q.put((0, (a, b)))
    except Exception as e:  # noqa: BLE001
        q.put((0, repr(e)))
    finally:
        dist.destroy_process_group()


def test_rccl_one_rank_sharded_device_loop(oracle, synth):
    """The sharded device-driven LM loop with RCCL (stream-ordered all-reduces between the unit's
    launches, the build / trial controllers after them) on one rank: the same state as the
    single-GPU solve bit for bit, and the oracle's LM path."""
    import torch.multiprocessing as mp
    kw = dict(n_kf=20, n_points=800, obs_per_point=5, stereo_frac=0.3, seed=12)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_one_rank_worker, args=(_port(), kw, q))
    p.start()
    import queue
    import time
    t0 = time.time()
    v = None
    while v is None:  # a crashed worker fails the test instead of blocking on the queue
        try:
            _, v = q.get(timeout=5)
        except queue.Empty:
            assert p.is_alive(), f"worker exited with {p.exitcode}"
            assert time.time() - t0 < 150, "worker timed out"
    p.join(timeout=60)
    assert not isinstance(v, str), v
    (pose, point, chi2, depth, res), (pose1, point1, chi21, depth1, res1) = v
    for k in ("iterations", "trials", "terminated", "stopped"):
        assert res[k] == res1[k], k
    assert np.array_equal(pose, pose1) and np.array_equal(point, point1)
    assert np.array_equal(chi2, chi21) and np.array_equal(depth, depth1)
    prob = synth.local_ba_problem(**kw)
    rpose, rpoint, _, _, rres = oracle.local_ba(prob, 10)
    assert res["iterations"] == rres["iterations"] and res["trials"] == rres["trials"]
    assert _rmse(pose[:, :3], rpose[:, :3]) < 1e-6 and _rmse(point, rpoint) < 1e-6
