"""Solve the C5 problem (mono and 50 % stereo) once and save poses / points / summary to an .npz:
    tools/ba_dump.py OUT.npz
Run under different ORBGPU_BA_* switches and compare the files (tools/ab_w.sh)."""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from conftest import load_package  # noqa: E402

pkg = load_package()
from orbslam3_amd import synth  # noqa: E402

out = {}
for st in (0.0, 0.5):
    prob = synth.local_ba_problem(stereo_frac=st)
    res = pkg.LocalBA().optimize(prob, 10)
    for i, a in enumerate(res[:4]):
        out[f"s{int(st * 10)}_{i}"] = np.asarray(a)
    out[f"s{int(st * 10)}_it"] = np.array([res[4]["iterations"], res[4]["trials"]])
np.savez(sys.argv[1], **out)
