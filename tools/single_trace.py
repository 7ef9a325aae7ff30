"""ORBextractor::operator() on one host 640x480 frame, 30 calls (for a rocprofv3 kernel trace of the
single-frame path: python3 tools/timeline.py <db> 20)."""
import os
import sys
import time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from tests.conftest import load_package  # noqa: E402
pkg = load_package()
from orbslam3_amd import synth  # noqa: E402
import numpy as np  # noqa: E402
img = synth.polygon_frame(640, 480, seed=7)
ex = pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=640, max_height=480)
t = []
for _ in range(30):
    t0 = time.perf_counter()
    ex(img, None, (0, 0))
    t.append((time.perf_counter() - t0) * 1e3)
print("median ms", float(np.median(t)))
