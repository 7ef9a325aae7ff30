"""Frame::SetPose (src/Optimizer.cc:390-395, src/Frame.cc:533-599, Thirdparty/Sophus/sophus/so3.hpp:229-231,
297-303,358-367, se3.hpp:208-211): the product's float restatement (csrc/orb_pose_frame.h, compiled into
the device tracking chain) against the oracle's independent one (oracle/orb_tracking_oracle.cpp), bit for
bit on 140k poses (tests/native/pose_frame_check.cpp).  The oracle shares no source with the product."""
from __future__ import annotations

import pathlib
import subprocess

ROOT = pathlib.Path(__file__).resolve().parents[1]


def test_oracle_shares_no_product_source():
    """Apart from the checksum-pinned rBRIEF pattern table (tests/test_oracle_kat.py), nothing under
    oracle/ includes or names a product source file."""
    offenders = []
    for f in sorted((ROOT / "oracle").glob("*")):
        if f.suffix not in (".cpp", ".h", ".py") and f.name != "Makefile":
            continue
        for i, line in enumerate(f.read_text().splitlines(), 1):
            if "orb-slam3_byzyh_amd" in line and "orb_pattern31.inc" not in line:
                offenders.append(f"{f.name}:{i}: {line.strip()}")
    assert not offenders, offenders


def test_pose_frame_product_equals_oracle():
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)
    out = ROOT / "build" / "tests"
    out.mkdir(parents=True, exist_ok=True)
    exe = out / "pose_frame_check"
    lib = ROOT / "oracle" / "_build"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", str(ROOT / "tests" / "native" / "pose_frame_check.cpp"),
                    "-o", str(exe), f"-L{lib}", "-lorb_oracle", f"-Wl,-rpath,{lib}"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("OK "), r.stdout + r.stderr
