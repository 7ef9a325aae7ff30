"""Single-frame PoseOptimization time (device-resident, ms per call) against the frame's edge count:
how much of a frame's time is the per-trial serial part (thread 0's solve, barriers) and how much
the per-edge linearisation."""
import ctypes
import os
import sys
import time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from tests.conftest import load_package  # noqa: E402
pkg = load_package()
from orbslam3_amd import synth  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402
dev = torch.device("cuda", 0)
lib = pkg._lib.load()
for ne_f in (30, 100, 250, 500, 1000):
    frames, edges, _ = synth.pose_opt_batch(1, ne_f, stereo_frac=0.5, seed=4242)
    ne = int(frames["n_edges"][0])
    d_fr = torch.from_numpy(frames.view(np.uint8).reshape(-1)).to(dev)
    d_ed = torch.from_numpy(edges[:ne].view(np.uint8).reshape(-1)).to(dev)
    d_pose = torch.empty((1, 7), dtype=torch.float64, device=dev)
    d_out = torch.empty(ne, dtype=torch.uint8, device=dev)
    d_inl = torch.empty(1, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev)

    def step():
        pkg._lib.check(lib.orb_pose_optimization_device(1, d_fr.data_ptr(), ne, d_ed.data_ptr(), d_pose.data_ptr(),
                                                        d_out.data_ptr(), d_inl.data_ptr(), ctypes.c_void_p(st.cuda_stream)),
                       "pose")
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    reps = 50
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
        torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / reps
    print(f"edges {ne}: {ms:.4f} ms per frame", flush=True)
