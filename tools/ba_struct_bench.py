"""Write the C5 local BA problem for tools/ba_struct_bench.cpp (binary: np nq ne, pose, pose_id,
pose_fixed, point, point_id, edges)."""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from conftest import load_package  # noqa: E402

load_package()
from orbslam3_amd import synth  # noqa: E402

prob = synth.local_ba_problem()
with open(sys.argv[1] if len(sys.argv) > 1 else "/tmp/c5.bin", "wb") as f:
    f.write(np.array([len(prob["pose"]), len(prob["point"]), len(prob["edges"])], np.int32).tobytes())
    for k, dt in (("pose", np.float64), ("pose_id", np.int64), ("pose_fixed", np.uint8), ("point", np.float64),
                  ("point_id", np.int64)):
        f.write(np.ascontiguousarray(prob[k], dtype=dt).tobytes())
    f.write(np.ascontiguousarray(prob["edges"]).tobytes())
