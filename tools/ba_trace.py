import os, pathlib, sys
os.environ["ORBGPU_BA_TRACE"] = "1"
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
from conftest import load_package
pkg = load_package()
from orbslam3_amd import synth
prob = synth.local_ba_problem()
ba = pkg.LocalBA()
ba.optimize(prob, 2)
