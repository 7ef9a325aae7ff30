"""One 64-frame C2 batch with ORBGPU_FAST_STAMPS set: per-launch mean phase clocks of k_fast_cells
(printed by the library to stderr)."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
os.environ["ORBGPU_FAST_STAMPS"] = "1"
from tests.conftest import load_package  # noqa: E402
pkg = load_package()
from orbslam3_amd import synth  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402
nfr = 64
frames = np.stack([synth.polygon_frame(640, 480, seed=100 + i) for i in range(nfr)])
imgs = torch.from_numpy(frames).to(torch.device("cuda", 0))
ex = pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=640, max_height=480, max_batch=nfr)
for i in range(3):
    print(f"--- batch {i}", file=sys.stderr, flush=True)
    ex.extract_batch_device(imgs, (0, 1000))
    torch.cuda.synchronize()
