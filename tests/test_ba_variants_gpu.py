"""The LocalBA paths a plain C5 solve does not take, each against the CPU oracle at the 1e-6 bar:
  * ORBGPU_BA_CHOL=rows: the tile-row multi-workgroup Cholesky (k_ba_chol_rows), which windows above
    48 free keyframes use, here at n = 288;
  * ORBGPU_BA_HOST_LM=1: the host-driven LM loop the sharded (multi-GPU) solve uses, on one process;
  * both together;
  * ORBGPU_BA_FAST_UNIT=0: the 6-launch LM unit (the sharded solve's) on one process;
  * ORBGPU_BA_FUSED_TRIAL=0: the round-5 back-substitution + error launches (k_u_backsub_update +
    k_u_edges_trial) instead of k_u_land_trial;
  * ORBGPU_BA_UNITS=1 / 8: one and eight LM trials per graph launch.
The switches are read once per process, so each variant solves in a child process (tools/ba_dump.py:
the C5 problem, mono and 50 % stereo) and the saved results are compared here."""
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
    for k in ("ORBGPU_BA_CHOL", "ORBGPU_BA_HOST_LM", "ORBGPU_BA_TRACE", "ORBGPU_BA_FAST_UNIT", "ORBGPU_BA_FUSED_TRIAL",
              "ORBGPU_BA_UNITS"):
        env.pop(k, None)
    env.update(env_extra)
    subprocess.run([sys.executable, str(ROOT / "tools" / "ba_dump.py"), str(out)], env=env, check=True,
                   timeout=100)
    return np.load(out)


def _rmse(a, b):
    return float(np.sqrt(np.mean((np.asarray(a) - np.asarray(b)) ** 2)))


@pytest.mark.gpu
@pytest.mark.parametrize("name,env", [("rows", {"ORBGPU_BA_CHOL": "rows"}), ("host_lm", {"ORBGPU_BA_HOST_LM": "1"}),
                                      ("rows_host_lm", {"ORBGPU_BA_CHOL": "rows", "ORBGPU_BA_HOST_LM": "1"}),
                                      ("unit6", {"ORBGPU_BA_FAST_UNIT": "0"}),
                                      ("unfused", {"ORBGPU_BA_FUSED_TRIAL": "0"}),
                                      ("units1", {"ORBGPU_BA_UNITS": "1"}), ("units8", {"ORBGPU_BA_UNITS": "8"})])
def test_ba_variant_against_oracle(tmp_path, oracle, synth, name, env):
    got = _solve(tmp_path, name, env)
    for st in (0.0, 0.5):
        tag = f"s{int(st * 10)}"
        prob = synth.local_ba_problem(stereo_frac=st)
        rpose, rpoint, rchi2, rdepth, rres = oracle.local_ba(prob, 10)
        pose, point, chi2, depth = (got[f"{tag}_{i}"] for i in range(4))
        it, trials = got[f"{tag}_it"]
        assert (it, trials) == (rres["iterations"], rres["trials"]), f"{name} {tag}: LM path"
        assert _rmse(pose[:, :3], rpose[:, :3]) < 1e-6
        q = np.where((np.sum(pose[:, 3:] * rpose[:, 3:], axis=1) < 0)[:, None], -pose[:, 3:], pose[:, 3:])
        assert _rmse(q, rpose[:, 3:]) < 1e-6
        assert _rmse(point, rpoint) < 1e-6
        assert np.array_equal(depth, rdepth)
        if st == 0.0:
            assert np.allclose(chi2, rchi2, rtol=1e-9, atol=1e-12)
        else:
            assert np.allclose(chi2, rchi2, rtol=1e-6, atol=1e-3)
