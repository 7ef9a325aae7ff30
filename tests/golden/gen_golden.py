#!/usr/bin/env python3
"""Write the golden fixtures (tests/golden/fixtures.py describes them) from the CPU oracle on the seeded
synthetic workloads.  Run once in the build container after a deliberate oracle / generator change:

    python3 tests/golden/gen_golden.py

and commit the diff with the reason.  Takes ~20 s on one core."""
from __future__ import annotations

import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from conftest import load_package  # noqa: E402
from golden import fixtures as fx  # noqa: E402
from oracle import oracle, tracking_chain  # noqa: E402


def main() -> int:
    pkg = load_package()
    from orbslam3_amd import synth
    oracle.load()
    out = fx.HERE

    # extraction
    recs = {}
    for name, img, nf, lap in fx.extract_cases(synth):
        k, d, m = oracle.OracleExtractor(nf, 1.2, 8, 20, 7)(img, lap)
        recs[name] = dict(fx.extract_record(img, k, d, m), nfeatures=nf, lapping=list(lap),
                          width=int(img.shape[1]), height=int(img.shape[0]))
        if name == "c1_seed1":
            np.savez_compressed(out / "c1_seed1.npz", kps=k.view(np.uint8).reshape(-1, 28), desc=d, mono=np.int64(m))
    (out / "extract.json").write_text(json.dumps(recs, indent=1, sort_keys=True) + "\n")

    # SearchForTriangulation on the C3 keyframe chain
    kfs, _ = fx.c3_keyframes(pkg, synth, oracle)
    (out / "sft_c3.json").write_text(json.dumps(fx.sft_records(pkg, oracle, kfs), indent=1, sort_keys=True) + "\n")

    # LocalBA
    arrays = {}
    meta = {}
    for name, kw in fx.BA_CASES.items():
        prob = synth.local_ba_problem(**kw)
        pose, point, chi2, depth, res = oracle.local_ba(prob, 10)
        meta[name] = {"problem_sha256": fx.problem_sha(prob), "kwargs": kw}
        arrays[f"{name}__pose"] = pose
        arrays[f"{name}__point"] = point
        arrays[f"{name}__chi2"] = chi2
        arrays[f"{name}__depth"] = np.asarray(depth, np.uint8)
        arrays[f"{name}__path"] = fx.ba_path(res)
        arrays[f"{name}__chi2_final"] = np.float64(res["final_chi2"])
    small = synth.local_ba_problem(**fx.BA_SMALL)
    for k, v in small.items():
        if isinstance(v, np.ndarray):
            if v.dtype.names:  # structured records: keep the bytes and the dtype description
                arrays[f"small_problem__{k}__bytes"] = v.view(np.uint8).reshape(len(v), -1)
                meta[f"small_problem__{k}__dtype"] = v.dtype.descr
            else:
                arrays[f"small_problem__{k}"] = v
    pose, point, chi2, depth, res = oracle.local_ba(small, 10)
    arrays.update(small__pose=pose, small__point=point, small__chi2=chi2, small__depth=np.asarray(depth, np.uint8),
                  small__path=fx.ba_path(res))
    meta["small"] = {"problem_sha256": fx.problem_sha(small), "kwargs": fx.BA_SMALL}
    arrays["meta_json"] = np.frombuffer(json.dumps(meta, sort_keys=True).encode(), np.uint8)
    np.savez_compressed(out / "ba_c5.npz", **arrays)

    # tracking chain
    tr = {}
    for name, kw in fx.TRACK_SCENES.items():
        sc = synth.tracking_chain_scene(**kw)
        C, L = pkg.Frame(**sc["cur"]), pkg.Frame(**sc["last"])
        o = tracking_chain.track(pkg, C, L, sc["local"], sc["pose7_pred"], sc["level_sigma2"], fx.track_th(kw), 1)
        tr[name] = fx.tracking_record(o)
    (out / "tracking.json").write_text(json.dumps(tr, indent=1, sort_keys=True) + "\n")
    for f in sorted(out.glob("*")):
        if f.suffix in (".json", ".npz"):
            print(f"{f.name}: {f.stat().st_size} B")
    return 0


if __name__ == "__main__":
    sys.exit(main())
