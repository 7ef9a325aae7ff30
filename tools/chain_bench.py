"""Run only bench.py's tracking_chain measurement (quick iteration on the device tracking chain)."""
import json
import sys

sys.path.insert(0, ".")
import bench  # noqa: E402

pkg = bench.load_package()
import torch  # noqa: E402

from orbslam3_amd import synth  # noqa: E402

cpu = "--cpu" in sys.argv
out = bench.bench_tracking_chain(pkg, synth, torch.device("cuda:0"), 20, cpu)
print(json.dumps(out, indent=1))
if "--pose" in sys.argv:
    print(json.dumps(bench.bench_pose(pkg, synth, torch.device("cuda:0"), 20, cpu), indent=1))
