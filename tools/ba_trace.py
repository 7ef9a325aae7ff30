"""Phase stamps of the MFMA Cholesky (ORBGPU_BA_TRACE=1): one C5 solve, stamps printed to stderr
by the library as `MFTRACE k=.. w=.. panel_start update_start update_end/diag_start diag_end`."""
import os
import pathlib
import sys

os.environ["ORBGPU_BA_TRACE"] = "1"
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from conftest import load_package  # noqa: E402

pkg = load_package()
from orbslam3_amd import synth  # noqa: E402

prob = synth.local_ba_problem()
ba = pkg.LocalBA()
ba.optimize(prob, 1)
# steady state: the host phases of a few optimize(10) solves ([ba] lines on stderr)
for _ in range(6):
    ba.optimize(prob, 10)
