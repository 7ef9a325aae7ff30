"""C2 step time with stage launches left out (ORBGPU_ABLATE, timing study only: the skipped stages'
outputs stay from the warm-up steps, which ran on the same frames).  What each stage costs the
overlapped step, as opposed to its own launch durations.

    python3 tools/c2_ablate.py 0 1 3 4 8 16   (masks; each in a child process, alternated twice)"""
import json
import os
import subprocess
import sys
import time

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import numpy as np
    import torch
    from bench import load_package, throughput_mode
    pkg = load_package()
    from orbslam3_amd import synth
    dev = torch.device("cuda", 0)
    nfr, H, W, Hh = 64, 4, 640, 480
    imgs = torch.from_numpy(np.stack([synth.polygon_frame(W, Hh, seed=100 + i) for i in range(nfr)])).to(dev)
    exs = throughput_mode([pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=W, max_height=Hh, max_batch=nfr)
                           for _ in range(H)])
    cap = 1000 + 16 * 8
    outs = [(torch.empty((nfr, cap, 7), dtype=torch.float32, device=dev),
             torch.empty((nfr, cap, 32), dtype=torch.uint8, device=dev),
             torch.empty((nfr, 2), dtype=torch.int32, device=dev)) for _ in range(H)]
    sts = [torch.cuda.Stream(dev) for _ in range(H)]
    mask = int(sys.argv[2])
    # warm-up with every stage, so the stale outputs a skipped stage leaves are the real ones
    for i in range(16):
        exs[i % H].extract_batch_device(imgs, (0, 1000), cap=cap, out=outs[i % H], stream=sts[i % H])
    torch.cuda.synchronize()
    os.environ["ORBGPU_ABLATE"] = str(mask)  # read by every batch call from here on
    res = {}
    for rep in range(3):
        t_end = time.perf_counter() + 0.3
        n = 0
        while time.perf_counter() < t_end:
            exs[n % H].extract_batch_device(imgs, (0, 1000), cap=cap, out=outs[n % H], stream=sts[n % H])
            n += 1
        torch.cuda.synchronize()
        steps = 200
        t0 = time.perf_counter()
        for i in range(steps):
            exs[i % H].extract_batch_device(imgs, (0, 1000), cap=cap, out=outs[i % H], stream=sts[i % H])
        torch.cuda.synchronize()
        res[rep] = (time.perf_counter() - t0) * 1e3 / steps
    print(json.dumps({"mask": mask, "ms_per_step": sorted(res.values())[1]}))
    sys.exit(0)

for rnd in range(2):
    for m in sys.argv[1:]:
        env = {k: v for k, v in os.environ.items() if k != "ORBGPU_ABLATE"}
        out = subprocess.run([sys.executable, __file__, "--child", m], env=env, capture_output=True, text=True,
                             timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        print(line[-1] if line else f"mask {m} failed: {out.stderr[-400:]}", flush=True)
