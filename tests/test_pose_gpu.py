"""GPU parity of Optimizer::PoseOptimization (orb_pose_optimization*, HIP) against the CPU oracle
(oracle/orb_pose_oracle.cpp).  Bar: 1e-6 pose RMSE (the north star's BA bar), identical
mvbOutlier flags and inlier counts."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check(pkg, oracle, frames, edges, tol=1e-6):
    P, O, I = pkg.pose_optimization(frames, edges)
    RP, RO, RI = oracle.pose_optimization(frames, edges)
    rmse = np.sqrt(np.mean((P - RP) ** 2, axis=1))
    assert (rmse < tol).all(), rmse.max()
    assert np.array_equal(I, RI), np.flatnonzero(I != RI)
    assert np.array_equal(O, RO), np.flatnonzero(O != RO)[:10]
    return P, O, I


@pytest.mark.parametrize("stereo_frac,seed", [(0.0, 41), (0.5, 42), (1.0, 43)])
def test_pose_optimization_parity(pkg, oracle, synth, stereo_frac, seed):
    frames, edges, truth = synth.pose_opt_batch(32, 500, stereo_frac=stereo_frac, seed=seed)
    P, O, I = _check(pkg, oracle, frames, edges)
    t0 = np.linalg.norm(frames["pose"][:, :3] - truth[:, :3], axis=1)
    t1 = np.linalg.norm(P[:, :3] - truth[:, :3], axis=1)
    assert np.median(t1) < 0.2 * np.median(t0)


def test_pose_optimization_ragged_and_edge_cases(pkg, oracle, synth):
    # < 3 edges (returns 0), < 10 edges (a single round), large frames (several edges per thread),
    # heavy outliers and a poor initial pose
    counts = [0, 2, 3, 7, 9, 10, 11, 64, 255, 256, 257, 1500, 3000]
    frames, edges, _ = synth.pose_opt_batch(len(counts), 0, seed=77, points_per_frame=counts, outlier_frac=0.3,
                                            rot_err=0.03, trans_err=0.1)
    _check(pkg, oracle, frames, edges)
    # empty batch
    P, O, I = pkg.pose_optimization(frames[:0], edges[:0])
    assert len(P) == 0 and len(I) == 0


@pytest.mark.parametrize("stereo_frac,seed", [(0.0, 44), (0.5, 45)])
def test_pose_optimization_two_frames_per_cu(pkg, oracle, synth, monkeypatch, stereo_frac, seed):
    """The batch form (two frames per CU: a 1024-edge LDS room, frames beyond ~900 edges read the rest
    from memory each pass), forced on small batches incl. the ragged frames, and taken by itself at 512
    frames: the oracle's poses, outlier flags and inlier counts."""
    monkeypatch.setenv("ORBGPU_POSE_DUAL", "1")
    counts = [0, 2, 3, 9, 10, 64, 256, 895, 896, 897, 1023, 1024, 1025, 1500, 3000]
    frames, edges, _ = synth.pose_opt_batch(len(counts), 0, seed=seed, points_per_frame=counts, outlier_frac=0.3,
                                            rot_err=0.03, trans_err=0.1, stereo_frac=stereo_frac)
    _check(pkg, oracle, frames, edges)
    monkeypatch.delenv("ORBGPU_POSE_DUAL")
    frames, edges, _ = synth.pose_opt_batch(512, 300, stereo_frac=stereo_frac, seed=seed + 10)
    _check(pkg, oracle, frames, edges)
