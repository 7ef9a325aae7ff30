"""Exclusive pyramid launch durations (one 64-frame C2 batch at a time, event pair per dispatch) for
the two-level passes (ORBGPU_PYR_PAIR=1) and the level passes (=0), and the pyramid stage time of one
batch alone (stage events).  ORBGPU_PYR_PAIR is read when a handle is created."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bench import load_package  # noqa: E402

pkg = load_package()
from orbslam3_amd import synth  # noqa: E402

nfr = 64
imgs = torch.from_numpy(np.stack([synth.polygon_frame(640, 480, seed=100 + i) for i in range(nfr)])).cuda()
exs = {}
for v in ("1", "0"):
    os.environ["ORBGPU_PYR_PAIR"] = v
    exs[v] = pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=640, max_height=480, max_batch=nfr)
    exs[v].set_overlap(False)
for rep in range(2):
    for v, ex in exs.items():
        for _ in range(3):
            ex.extract_batch_device(imgs, (0, 1000))
        torch.cuda.synchronize()
        ex.profile("pyramid_launches")
        for _ in range(10):
            ex.extract_batch_device(imgs, (0, 1000))
            torch.cuda.synchronize()
        d = {k: ex.launch_durations(k) for k in ex.LAUNCH_KERNELS}
        ex.profile(False)
        ex.profile(True)
        for _ in range(10):
            ex.extract_batch_device(imgs, (0, 1000))
            torch.cuda.synchronize()
        st, n, _ = ex.stage_ms()
        ex.profile(False)
        pyr = d["k_pyramid_level"]
        per = len(pyr) // 10
        lv = [round(1e3 * sum(pyr[i::per]) / 10, 1) for i in range(per)]
        print(f"PYR_PAIR={v}: pyramid launches per batch {per}, us each {lv}, sum {sum(lv):.1f} us; "
              f"fast {1e3 * sum(d['k_fast_cells']) / 10:.1f} us; stages per batch (ms) "
              f"{ {k: round(x / max(1, n), 4) for k, x in st.items()} }", flush=True)
