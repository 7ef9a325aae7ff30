"""LocalBA solves at several window sizes (free keyframes -> S of 6 x nf rows), for a rocprofv3 kernel
trace: how k_ba_chol_mf2's duration scales with n.
    rocprofv3 --kernel-trace --output-format csv -d OUT -o c -- python3 tools/chol_size_probe.py [N_KF ...]
Prints the order of the sizes; the trace's dispatches come in the same order."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from conftest import load_package  # noqa: E402

pkg = load_package()
from orbslam3_amd import synth  # noqa: E402

for n_kf in [int(a) for a in sys.argv[1:]] or (14, 26, 38, 50):
    prob = synth.local_ba_problem(n_kf=n_kf, n_points=40 * n_kf, obs_per_point=6, stereo_frac=0.0, seed=7)
    ba = pkg.LocalBA()
    for _ in range(5):
        _, _, _, _, res = ba.optimize(prob, 10)
    print(f"n_kf {n_kf}: n = {6 * (n_kf - 2)}, {res['iterations']} it, {res['trials']} trials", flush=True)
