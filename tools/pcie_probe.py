"""Host-input C2 pipeline variants (H2D -> extract -> D2H) on the GPU box: which stream layout lets the
copies overlap the extraction.  python3 tools/pcie_probe.py"""
import os
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

dev = torch.device("cuda", 0)
N = 64
frames = np.stack([synth.polygon_frame(640, 480, seed=100 + i) for i in range(N)])
host = torch.from_numpy(frames).pin_memory()
cap = 1128


def run(layout, H, copy_first, env=None):
    for k, v in (env or {}).items():
        os.environ[k] = v
    up = down = None
    if copy_first:
        up, down = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    exs = [pkg.ORBextractor(1000, 1.2, 8, 20, 7, max_width=640, max_height=480, max_batch=N) for _ in range(H)]
    if not copy_first:
        up, down = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    sts = [torch.cuda.Stream(dev) for _ in range(H)]
    dimg = [torch.empty_like(host, device=dev) for _ in range(H)]
    outs = [(torch.empty((N, cap, 7), dtype=torch.float32, device=dev), torch.empty((N, cap, 32), dtype=torch.uint8, device=dev),
             torch.empty((N, 2), dtype=torch.int32, device=dev)) for _ in range(H)]
    houts = [tuple(torch.empty(o.shape, dtype=o.dtype).pin_memory() for o in outs[h]) for h in range(H)]
    ev = [[torch.cuda.Event() for _ in range(3)] for _ in range(H)]
    started = [False] * H

    def step(i):
        h = i % H
        if layout == "own":
            with torch.cuda.stream(sts[h]):
                dimg[h].copy_(host, non_blocking=True)
                exs[h].extract_batch_device(dimg[h], (0, 1000), cap=cap, out=outs[h], stream=sts[h])
                for d, o in zip(houts[h], outs[h]):
                    d.copy_(o, non_blocking=True)
            return
        with torch.cuda.stream(up):
            if started[h]:
                up.wait_event(ev[h][1])
            dimg[h].copy_(host, non_blocking=True)
            ev[h][0].record(up)
        with torch.cuda.stream(sts[h]):
            sts[h].wait_event(ev[h][0])
            if started[h]:
                sts[h].wait_event(ev[h][2])
            exs[h].extract_batch_device(dimg[h], (0, 1000), cap=cap, out=outs[h], stream=sts[h])
            ev[h][1].record(sts[h])
        with torch.cuda.stream(down):
            down.wait_event(ev[h][1])
            for d, o in zip(houts[h], outs[h]):
                d.copy_(o, non_blocking=True)
            ev[h][2].record(down)
        started[h] = True

    for i in range(3 * H):
        step(i)
    torch.cuda.synchronize()
    reps = 20
    t = time.perf_counter()
    for i in range(reps):
        step(i)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1e3 / reps
    nf = int(houts[0][2][:, 0].sum())
    print(f"{layout:5s} H={H} copies-first={copy_first} env={env}: {ms:.3f} ms/step, {nf / ms:.0f} features/ms", flush=True)
    for k in (env or {}):
        del os.environ[k]


run("own", 3, False)
run("own", 2, False)
run("split", 2, False)
run("split", 2, True)
run("split", 1, True)
run("split", 2, True, {"ORBGPU_FAST_SPLIT": "0"})
run("own", 3, False, {"ORBGPU_FAST_SPLIT": "0"})
run("split", 3, True)
