"""The LocalBA Cholesky shapes are one computation: 7 or 11 tile waves, diagonal factor and backward
chain broadcast by v_readlane or by DPP (orb_ba.hip k_ba_chol_mf2) must give bitwise identical
solutions.  The switches are read once per process, so each variant solves in a child process
(tools/ba_dump.py) and the files are compared."""
import os
import pathlib
import subprocess
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _solve(tmp_path, name, env_extra):
    out = tmp_path / f"{name}.npz"
    env = dict(os.environ)
    env.pop("ORBGPU_BA_MF_W", None)
    env.pop("ORBGPU_BA_DIAG_READLANE", None)
    env.update(env_extra)
    subprocess.run([sys.executable, str(ROOT / "tools" / "ba_dump.py"), str(out)], env=env, check=True,
                   timeout=100)
    return np.load(out)


@pytest.mark.gpu
def test_cholesky_variants_bitwise_identical(tmp_path):
    ref = _solve(tmp_path, "w7_readlane", {"ORBGPU_BA_MF_W": "7", "ORBGPU_BA_DIAG_READLANE": "1"})
    for name, env in (("default", {}), ("w7_dpp", {"ORBGPU_BA_MF_W": "7"}),
                      ("w11_readlane", {"ORBGPU_BA_MF_W": "11", "ORBGPU_BA_DIAG_READLANE": "1"})):
        got = _solve(tmp_path, name, env)
        for k in ref.files:
            assert np.array_equal(ref[k], got[k]), f"{name}: {k} differs from the 7-wave readlane kernel"
