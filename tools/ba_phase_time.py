"""Host-side phases of orb_ba_optimize (ORBGPU_BA_TRACE=1 prints `[ba] structure .. upload+LM .. results`
per solve on stderr): 6 warm solves of the C5 problem, plus the Python-side packing time."""
import os
import pathlib
import sys
import time

os.environ["ORBGPU_BA_TRACE"] = "1"
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from conftest import load_package  # noqa: E402

pkg = load_package()
from orbslam3_amd import synth  # noqa: E402

prob = synth.local_ba_problem()
ba = pkg.LocalBA()
for _ in range(6):
    t0 = time.perf_counter()
    ba.optimize(prob, 10)
    print(f"optimize wall {(time.perf_counter() - t0) * 1e3:.3f} ms", file=sys.stderr, flush=True)
