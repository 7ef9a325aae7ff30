"""GPU parity of SearchByProjection(CurrentFrame, LastFrame, th, bMono) (k_proj_candidates +
k_proj_resolve) against the oracle: bit-exact assignments and match counts, including contested
keypoints (the in-order 'already holds an observed map point' rule), mono/stereo, forward/backward
motion and the orientation filter."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed,th,mono,ori,stereo,forward", [
    (31, 7, False, True, True, 0.02), (32, 15, True, True, False, 0.02), (33, 7, False, False, True, 0.3),
    (34, 7, False, True, True, -0.3), (35, 3, False, True, True, 0.0)])
def test_search_by_projection_frame_parity(pkg, oracle, synth, seed, th, mono, ori, stereo, forward):
    cur, last = synth.tracking_pair(seed=seed, stereo=stereo, forward=forward, dup_frac=0.08)
    C, L = pkg.Frame(**cur), pkg.Frame(**last)
    m = pkg.ORBmatcher(0.9, ori)
    n, got = m.SearchByProjectionFrame(C, L, th, mono)
    rn, exp = oracle.search_by_projection_frame(C, L, th, mono, ori)
    assert n == rn, f"{n} vs oracle {rn}"
    assert np.array_equal(got, exp), f"{int((got != exp).sum())} differing assignments"
    assert n > 50


def test_search_by_projection_frame_edge_cases(pkg, oracle, synth):
    cur, last = synth.tracking_pair(n_points=300, clutter=50, seed=36)
    C, L = pkg.Frame(**cur), pkg.Frame(**last)
    m = pkg.ORBmatcher(0.9, True)
    # no valid last-frame map point
    mp = dict(L.map_points, valid=np.zeros(L.N, np.uint8))
    L0 = pkg.Frame(**dict(last, map_points=mp))
    n, got = m.SearchByProjectionFrame(C, L0, 7, False)
    assert n == 0 and (got == -1).all()
    # huge radius: many candidates per point (capacity growth path)
    n, got = m.SearchByProjectionFrame(C, L, 60, False)
    rn, exp = oracle.search_by_projection_frame(C, L, 60, False, True)
    assert n == rn and np.array_equal(got, exp)


@pytest.mark.parametrize("seed,th,far,ratio,taken_frac", [(51, 1, False, 0.8, 0.0), (52, 3, False, 0.9, 0.05),
                                                           (53, 5, True, 0.6, 0.1), (54, 10, False, 0.8, 0.0)])
def test_search_by_projection_local_parity(pkg, oracle, synth, seed, th, far, ratio, taken_frac):
    cur, _ = synth.tracking_pair(seed=seed)
    F = pkg.Frame(**cur)
    P = pkg.LocalMapPoints(**synth.local_map_points(cur, seed=seed + 100))
    taken = (np.random.default_rng(seed).random(F.N) < taken_frac).astype(np.uint8)
    m = pkg.ORBmatcher(ratio, True)
    n, got = m.SearchByProjection(F, P, th, far, 10.0, taken)
    rn, exp = oracle.search_by_projection_local(F, P, th, far, 10.0, ratio, taken)
    assert n == rn, f"{n} vs oracle {rn}"
    assert np.array_equal(got, exp), f"{int((got != exp).sum())} differing assignments"
    assert n > 50


def test_search_by_projection_large_paths(pkg, oracle, synth):
    """The resolve's memory-resident paths: more than 2,048 local map points whose answer an earlier
    point can change (the rounds read their state from memory instead of registers), and a current
    frame of more than 16,384 keypoints (claims in global memory instead of LDS)."""
    cur, _ = synth.tracking_pair(seed=61)
    F = pkg.Frame(**cur)
    P = pkg.LocalMapPoints(**synth.local_map_points(cur, n_points=9000, seed=161))
    taken = np.zeros(F.N, np.uint8)
    m = pkg.ORBmatcher(0.8, True)
    n, got = m.SearchByProjection(F, P, 10, False, 10.0, taken)
    rn, exp = oracle.search_by_projection_local(F, P, 10, False, 10.0, 0.8, taken)
    assert n == rn and np.array_equal(got, exp), f"{n} vs {rn}, {int((got != exp).sum())} differing"
    cur, last = synth.tracking_pair(n_points=1500, clutter=17000, seed=62)
    C, L = pkg.Frame(**cur), pkg.Frame(**last)
    assert C.N > 16384
    mf = pkg.ORBmatcher(0.9, True)
    n, got = mf.SearchByProjectionFrame(C, L, 7, False)
    rn, exp = oracle.search_by_projection_frame(C, L, 7, False, True)
    assert n == rn and np.array_equal(got, exp), f"{n} vs {rn}, {int((got != exp).sum())} differing"
