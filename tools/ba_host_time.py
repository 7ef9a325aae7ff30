"""Per-solve wall time of LocalBA.optimize on the C5 problem, split into the Python packing
(make_problem_struct) and the library call; with ORBGPU_BA_TRACE=1 the library adds its own
phase line per solve on stderr."""
import sys
import time

sys.path.insert(0, ".")
import importlib

pkg = importlib.import_module("orb-slam3_byzyh_amd")
synth = importlib.import_module("orb-slam3_byzyh_amd.synth")
opt_mod = importlib.import_module("orb-slam3_byzyh_amd.optimizer")

prob = synth.local_ba_problem(n_kf=50, n_points=2000, obs_per_point=6, stereo_frac=0.0, seed=7)
ba = pkg.LocalBA()
for _ in range(3):
    ba.optimize(prob, 10)
t_pack = []
for _ in range(10):
    t0 = time.perf_counter()
    opt_mod.make_problem_struct(prob)
    t_pack.append((time.perf_counter() - t0) * 1e6)
t_call = []
for _ in range(10):
    t0 = time.perf_counter()
    ba.optimize(prob, 10)
    t_call.append((time.perf_counter() - t0) * 1e6)
t_pack.sort(); t_call.sort()
print(f"pack median {t_pack[5]:.0f} us, optimize median {t_call[5]:.0f} us", flush=True)
