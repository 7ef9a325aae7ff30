"""Local BA solve time against the window size (free keyframes), GPU only.

  python tools/ba_sizes.py [n_kf ...]     (default 50 82 130 202)
Prints ms per solve and per LM iteration for each window; ORBGPU_BA_CHOL=rows forces the tile-row
Cholesky at n <= 288 as well.
"""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from conftest import load_package  # noqa: E402

pkg = load_package()
from orbslam3_amd import synth  # noqa: E402

sizes = [int(a) for a in sys.argv[1:]] or [50, 82, 130, 202]
for n_kf in sizes:
    prob = synth.local_ba_problem(n_kf=n_kf, n_points=40 * n_kf, obs_per_point=6, seed=7)
    ba = pkg.LocalBA()
    for _ in range(2):
        ba.optimize(prob, 10)
    reps = 10
    t = time.perf_counter()
    for _ in range(reps):
        _, _, _, _, res = ba.optimize(prob, 10)
    dt = (time.perf_counter() - t) / reps * 1e3
    print(f"n_kf {n_kf} (n = {6 * (n_kf - 2)}): {dt:.3f} ms/solve, {dt / max(1, res['iterations']):.4f} ms/iter "
          f"({res['iterations']} it, {res['trials']} trials)", flush=True)
