"""PoseOptimization timing on device-resident inputs: the bench's 256-frame batch and tracking's
single frame (one 500-edge frame per call), ms per call."""
import ctypes
import json
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
for nf in (256, 1):
    frames, edges, _ = synth.pose_opt_batch(256, 500, stereo_frac=0.5, seed=4242)
    frames = frames[:nf]
    ne = int(frames["edge_begin"][-1] + frames["n_edges"][-1])
    edges = edges[:ne]
    d_fr = torch.from_numpy(frames.view(np.uint8).reshape(-1)).to(dev)
    d_ed = torch.from_numpy(edges.view(np.uint8).reshape(-1)).to(dev)
    d_pose = torch.empty((nf, 7), dtype=torch.float64, device=dev)
    d_out = torch.empty(ne, dtype=torch.uint8, device=dev)
    d_inl = torch.empty(nf, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev)

    def step():
        pkg._lib.check(lib.orb_pose_optimization_device(nf, d_fr.data_ptr(), ne, d_ed.data_ptr(), d_pose.data_ptr(),
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
    print(json.dumps({"frames": nf, "ms_per_call": round(ms, 4), "frames_per_ms": round(nf / ms, 2)}), flush=True)
