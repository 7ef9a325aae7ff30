import sys, time, json
sys.path.insert(0, '/root/repo')
from tests.conftest import load_package
pkg = load_package()
from orbslam3_amd import synth
import numpy as np, torch
nfr = 64
frames = np.stack([synth.polygon_frame(640, 480, seed=100 + i) for i in range(nfr)])
dev = torch.device('cuda', 0)
imgs = torch.from_numpy(frames).to(dev)
cap = 1000 + 16 * 8
def mk():
    ex = pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=640, max_height=480, max_batch=nfr)
    out = (torch.empty((nfr, cap, 7), dtype=torch.float32, device=dev), torch.empty((nfr, cap, 32), dtype=torch.uint8, device=dev),
           torch.empty((nfr, 2), dtype=torch.int32, device=dev))
    return ex, out
for nh in (1, 2, 3):
    hs = [mk() for _ in range(nh)]
    streams = [torch.cuda.Stream(dev) for _ in range(nh)]
    def step(i):
        ex, out = hs[i % nh]
        ex.extract_batch_device(imgs, (0, 1000), cap=cap, out=out, stream=streams[i % nh])
    for i in range(6): step(i)
    torch.cuda.synchronize()
    K = 40
    t0 = time.perf_counter()
    for i in range(K): step(i)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / K
    n = int(hs[0][1][2][:, 0].sum())
    print(json.dumps({"handles": nh, "ms_per_step": round(ms, 4), "features_per_ms": round(n / ms, 1)}), flush=True)
