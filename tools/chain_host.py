"""Host cost of one TrackingChain.track call: enqueue time of back-to-back calls without a sync
(the launch path alone) and with a sync after each (latency), for rocprofv3 --hip-trace runs.
    python tools/chain_host.py [N]"""
import sys
import time

sys.path.insert(0, ".")
import bench  # noqa: E402

pkg = bench.load_package()
import numpy as np  # noqa: E402
import torch  # noqa: E402

from orbslam3_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dev = torch.device("cuda:0")
sc, C, L, cur, last, local = bench._chain_inputs(pkg, synth, dev, 4400)
ch = pkg.TrackingChain(cur.cap, device=dev, th_motion=7, th_local=1)
st = torch.cuda.Stream(dev)
for _ in range(3):
    ch.track(cur, last, local, sc["pose7_pred"], stream=st)
st.synchronize()
enq = []
for _ in range(n):
    t0 = time.perf_counter()
    ch.track(cur, last, local, sc["pose7_pred"], stream=st)
    enq.append((time.perf_counter() - t0) * 1e3)
st.synchronize()
lat = []
for _ in range(n):
    t0 = time.perf_counter()
    ch.track(cur, last, local, sc["pose7_pred"], stream=st)
    st.synchronize()
    lat.append((time.perf_counter() - t0) * 1e3)
print(f"enqueue back-to-back median {np.median(enq):.4f} ms, min {np.min(enq):.4f}; "
      f"track + sync median {np.median(lat):.4f} ms")
