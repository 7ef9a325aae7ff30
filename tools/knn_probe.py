"""knn2 (1000 x 1000, device-resident) through the C ABI with preallocated outputs: GPU time per call
(events around back-to-back calls) next to the host's enqueue time, to tell kernel- from host-bound."""
import ctypes, sys, time, pathlib
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
from conftest import load_package
pkg = load_package()
import numpy as np, torch
from orbslam3_amd import _lib
lib = _lib.load()
rng = np.random.default_rng(5)
q = torch.from_numpy(rng.integers(0, 256, (1000, 32), dtype=np.uint8)).cuda()
t = torch.from_numpy(rng.integers(0, 256, (1000, 32), dtype=np.uint8)).cuda()
idx = torch.empty(1000, dtype=torch.int32, device="cuda"); d1 = torch.empty_like(idx); d2 = torch.empty_like(idx)
st = torch.cuda.current_stream()
def call():
    lib.orb_hamming_knn2_device(q.data_ptr(), 1000, t.data_ptr(), 1000, idx.data_ptr(), d1.data_ptr(), d2.data_ptr(), ctypes.c_void_p(st.cuda_stream))
for _ in range(20): call()
torch.cuda.synchronize()
for reps in (200, 2000):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter(); e0.record()
    for _ in range(reps): call()
    e1.record(); t1 = time.perf_counter(); torch.cuda.synchronize()
    print(f"reps {reps}: gpu {e0.elapsed_time(e1)/reps*1e3:.2f} us/call, host enqueue {(t1-t0)/reps*1e6:.2f} us/call")
