"""The matcher calls of bench.py's `matchers` section (C3 calls, knn2, ComputeDistinctiveDescriptors), 50 times each, for rocprofv3 kernel traces:
    rocprofv3 --kernel-trace --stats -d OUT -o m -- python3 tools/matcher_time.py
Prints the host-side median per call."""
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from conftest import load_package  # noqa: E402

pkg = load_package()
from orbslam3_amd import synth  # noqa: E402


def med(fn, reps=50):
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append((time.perf_counter() - t0) * 1e3)
    return float(np.median(t))


kfs = [pkg.KeyFrame(**k) for k in synth.keyframe_scene(n_kf=11, n_points=1500, seed=201)]
m = pkg.ORBmatcher(0.6, False)
geoms = [m.pair_geometry(kfs[0], k) for k in kfs[1:]]
print("SFT ms", med(lambda: m.SearchForTriangulationMany(kfs[0], kfs[1:], False, False, geoms=geoms)), flush=True)
cur, last = synth.tracking_pair(seed=31, stereo=True, forward=0.02, dup_frac=0.08)
C, L = pkg.Frame(**cur), pkg.Frame(**last)
mp = pkg.ORBmatcher(0.9, True)
print("SBP frame ms", med(lambda: mp.SearchByProjectionFrame(C, L, 7, False)), flush=True)
P = pkg.LocalMapPoints(**synth.local_map_points(cur, n_points=3000, seed=151))
ml = pkg.ORBmatcher(0.8, True)
print("SBP local ms", med(lambda: ml.SearchByProjection(C, P, 3, False, 50.0)), flush=True)
rng = np.random.default_rng(5)
import torch  # noqa: E402
q = torch.from_numpy(rng.integers(0, 256, (1000, 32), dtype=np.uint8)).cuda()
t = torch.from_numpy(rng.integers(0, 256, (1000, 32), dtype=np.uint8)).cuda()
print("knn2 ms", med(lambda: (pkg.ORBmatcher.knn2_device(q, t), torch.cuda.synchronize())), flush=True)
nobs = rng.integers(2, 13, 2000).astype(np.int32)
offs = np.concatenate([[0], np.cumsum(nobs)]).astype(np.int32)
dd = rng.integers(0, 256, (int(offs[-1]), 32), dtype=np.uint8)
print("distinctive ms", med(lambda: ml.ComputeDistinctiveDescriptors(dd, offs)), flush=True)
