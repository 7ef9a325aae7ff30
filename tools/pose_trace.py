"""Phase stamps of one PoseOptimization frame (frame 0 of the bench batch, k_pose_opt, orb_debug_pose_trace):
per LM trial the pass, its reduction to the totals, thread 0's decision + solve, and the closing barrier,
in s_memtime cycles; plus the single-frame call time as the bench measures it."""
import ctypes
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from conftest import load_package  # noqa: E402

pkg = load_package()
import torch  # noqa: E402
from orbslam3_amd import synth  # noqa: E402

NPTS = int(sys.argv[1]) if len(sys.argv) > 1 else 500
frames, edges, _ = synth.pose_opt_batch(4, NPTS, stereo_frac=0.5, seed=4242)
lib = pkg._lib.load()
dev = torch.device("cuda", 0)
d_fr = torch.from_numpy(frames.view(np.uint8).reshape(-1)).to(dev)
d_ed = torch.from_numpy(edges.view(np.uint8).reshape(-1)).to(dev)
d_pose = torch.empty((4, 7), dtype=torch.float64, device=dev)
d_out = torch.empty(len(edges), dtype=torch.uint8, device=dev)
d_inl = torch.empty(4, dtype=torch.int32, device=dev)
n1 = int(frames["n_edges"][0])
st = torch.cuda.current_stream(dev)


def call():
    pkg._lib.check(lib.orb_pose_optimization_device(1, d_fr.data_ptr(), n1, d_ed.data_ptr(), d_pose.data_ptr(),
                                                    d_out.data_ptr(), d_inl.data_ptr(), ctypes.c_void_p(st.cuda_stream)),
                   "orb_pose_optimization_device")


for _ in range(5):
    call()
torch.cuda.synchronize()
reps = 50
t0 = time.perf_counter()
for _ in range(reps):
    call()
torch.cuda.synchronize()
print(f"single frame ({n1} edges): {(time.perf_counter() - t0) / reps * 1e3:.4f} ms per call")
cap = 128
buf = torch.zeros(16 * cap, dtype=torch.int64, device=dev)
pkg._lib.check(lib.orb_debug_pose_trace(buf.data_ptr(), cap), "trace on")
call()
torch.cuda.synchronize()
pkg._lib.check(lib.orb_debug_pose_trace(None, 0), "trace off")
t = buf.cpu().numpy().reshape(cap, 16)
t = t[t[:, 0] != 0]
d = np.diff(t[:, :5], axis=1)
sv = t[t[:, 5] != 0]
print(f"solve: decide {np.median(sv[:, 5] - sv[:, 2]):.0f}, ldlt {np.median(sv[:, 6] - sv[:, 5]):.0f}, "
      f"oplus {np.median(sv[:, 7] - sv[:, 6]):.0f}, to end {np.median(sv[:, 3] - sv[:, 7]):.0f}")
nxt = t[1:, 0] - t[:-1, 4]
print(f"{len(t)} trials; median cycles: pass {np.median(d[:, 0]):.0f}, totals {np.median(d[:, 1]):.0f}, "
      f"decide+solve {np.median(d[:, 2]):.0f}, barrier {np.median(d[:, 3]):.0f}, between trials {np.median(nxt):.0f}; "
      f"trial span median {np.median(t[:, 4] - t[:, 0]):.0f}, first-to-last {t[-1, 4] - t[0, 0]}")
pz = t[t[:, 8] != 0]
print(f"pass detail (wave 0): T+rt {np.median(pz[:, 8] - pz[:, 0]):.0f}, slot0 {np.median(pz[:, 9] - pz[:, 8]):.0f}, "
      f"slot1 {np.median(pz[:, 10] - pz[:, 9]):.0f}, lds/mem slots {np.median(pz[:, 11] - pz[:, 10]):.0f}, "
      f"butterfly {np.median(pz[:, 12] - pz[:, 11]):.0f}, barrier {np.median(pz[:, 13] - pz[:, 12]):.0f}, "
      f"wave sums {np.median(pz[:, 1] - pz[:, 13]):.0f}")

# cost probe (a library built with -DORB_POSE_PROBE): the kernel time with the block solve / the
# exponential run twice on the dependent path
if lib.orb_debug_pose_extra(0) == 0:
    ntr = len(t)

    def timed():
        for _ in range(5):
            call()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            call()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3

    base = timed()
    for mode, name in ((1, "block solve"), (2, "exponential"), (3, "solve + exponential")):
        lib.orb_debug_pose_extra(mode)
        ms = timed()
        lib.orb_debug_pose_extra(0)
        print(f"probe: {name} once more per trial adds {(ms - base) * 1e3:.1f} us = "
              f"{(ms - base) * 1e-3 * 2.4e9 / max(ntr, 1):.0f} cycles per trial (at 2.4 GHz, {ntr} trials)")
