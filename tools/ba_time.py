"""Time the local BA solve (C5) on the GPU and the oracle on the CPU."""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from conftest import load_package  # noqa: E402

pkg = load_package()
from orbslam3_amd import synth  # noqa: E402
from oracle import oracle  # noqa: E402

for st in (0.0, 0.5):
    prob = synth.local_ba_problem(stereo_frac=st)
    ba = pkg.LocalBA()
    for _ in range(3):
        ba.optimize(prob, 10)
    t = time.perf_counter()
    reps = 20
    for _ in range(reps):
        _, _, _, _, res = ba.optimize(prob, 10)
    dt = (time.perf_counter() - t) / reps * 1e3
    if "--gpu-only" in sys.argv:
        # the marginal cost of an iteration: solves capped at 2 and at the full count
        t = time.perf_counter()
        for _ in range(reps):
            _, _, _, _, r2 = ba.optimize(prob, 2)
        dt2 = (time.perf_counter() - t) / reps * 1e3
        di = res["iterations"] - r2["iterations"]
        marg = (dt - dt2) / di if di > 0 else float("nan")
        print(f"stereo {st}: gpu {dt:.3f} ms/solve ({res['iterations']} it, {res['trials']} trials); "
              f"{dt2:.3f} ms at {r2['iterations']} it: {marg:.4f} ms per added iteration, "
              f"fixed part {dt - marg * res['iterations']:.3f} ms", flush=True)
        continue
    t = time.perf_counter()
    _, _, _, _, rres = oracle.local_ba(prob, 10)
    dto = (time.perf_counter() - t) * 1e3
    print(f"stereo {st}: gpu {dt:.3f} ms/solve, {dt / res['iterations']:.3f} ms/iter ({res['iterations']} it, "
          f"{res['trials']} trials); oracle {dto:.1f} ms, {dto / rres['iterations']:.2f} ms/iter", flush=True)
