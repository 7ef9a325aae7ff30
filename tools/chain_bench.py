"""Run only bench.py's tracking_chain measurement (quick iteration on the device tracking chain)."""
import json
import sys

sys.path.insert(0, ".")
import bench  # noqa: E402

pkg = bench.load_package()
import torch  # noqa: E402

from orbslam3_amd import synth  # noqa: E402

cpu = "--cpu" in sys.argv
import os  # noqa: E402
ns = int(os.environ.get("ORB_CHAIN_STREAMS", "4"))
nb = int(os.environ.get("ORB_CHAIN_BATCH", "32"))
out = bench.bench_tracking_chain(pkg, synth, torch.device("cuda:0"), 20, cpu, batch=nb, n_streams=ns)
print(json.dumps(out, indent=1))
if "--pose" in sys.argv:
    print(json.dumps(bench.bench_pose(pkg, synth, torch.device("cuda:0"), 20, cpu), indent=1))
