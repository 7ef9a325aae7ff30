"""C3 stereo bench (bench.bench_stereo) with 1, 2 and 3 extractor sets in flight."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
import bench
from tests.conftest import load_package
pkg = load_package()
from orbslam3_amd import synth
import torch
dev = torch.device('cuda', 0)
for ns in (1, 2, 3, 2):
    r = bench.bench_stereo(pkg, synth, dev, 20, False, n_sets=ns)
    print(ns, r['stereo_frames_per_ms'], r['ms_per_step'], flush=True)
