"""CPU tests of the native pieces: the C-ABI library loads and exports every symbol of
include/orbgpu.h (no compute without a GPU), the device-side introsort port equals libstdc++ std::sort,
and the rBRIEF sin/cos exception table reproduces glibc's steering offsets for every angle."""
from __future__ import annotations

import ctypes
import pathlib
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
BUILD = ROOT / "build" / "tests"


def _ensure_lib():
    lib = ROOT / "orb-slam3_byzyh_amd" / "lib" / "liborbgpu.so"
    if not lib.exists():
        subprocess.run(["make", "-s", "-C", str(ROOT), "orb-slam3_byzyh_amd/lib/liborbgpu.so"], check=True)
    return lib


def test_library_exports_header_symbols(pkg):
    from orbslam3_amd import _lib
    _ensure_lib()
    names = _lib.header_symbols()
    assert len(names) >= 11
    lib = ctypes.CDLL(str(_lib.LIB_PATH))
    for n in names:
        assert hasattr(lib, n), f"missing export {n}"
    assert set(names) == set(_lib.PROTOTYPES), "ctypes prototypes out of sync with include/orbgpu.h"


def test_no_silent_cpu_fallback(pkg):
    from orbslam3_amd import _lib
    _ensure_lib()
    lib = _lib.load()
    if lib.orb_device_count() > 0:
        pytest.skip("a GPU is visible; the no-device path is exercised on CPU hosts only")
    p = _lib.OrbParams(1000, 1.2, 8, 20, 7)
    h = ctypes.c_void_p()
    assert lib.orb_extractor_create(ctypes.byref(p), 640, 480, 1, ctypes.byref(h)) == _lib.ORB_ERR_DEVICE
    with pytest.raises(_lib.OrbGpuError):
        pkg.ORBextractor(1000, 1.2, 8, 20, 7)


def test_host_descriptor_distance(pkg):
    import numpy as np
    from orbslam3_amd import _lib
    _ensure_lib()
    lib = _lib.load()
    rng = np.random.default_rng(3)
    for _ in range(100):
        a = rng.integers(0, 256, 32, dtype=np.uint8)
        b = rng.integers(0, 256, 32, dtype=np.uint8)
        assert lib.orb_descriptor_distance(a.ctypes.data, b.ctypes.data) == int(np.unpackbits(a ^ b).sum())


def _compile(src: pathlib.Path, out: pathlib.Path, extra=()):
    BUILD.mkdir(parents=True, exist_ok=True)
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-pthread", *extra, str(src), "-o", str(out)],
                   check=True)
    return out


def test_introsort_port_matches_libstdcxx():
    exe = _compile(ROOT / "tests" / "native" / "sort_port_check.cpp", BUILD / "sort_port_check")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "\nOK " in "\n" + r.stdout, r.stdout + r.stderr


def test_local_ba_shim_on_mock_graph():
    """include/orbgpu_optimizer.hpp (Optimizer::LocalBundleAdjustment drop-in): window, vertex ids,
    edge order, stop flag, cull order and write-back on a mock KeyFrame/MapPoint graph."""
    exe = _compile(ROOT / "tests" / "native" / "local_ba_shim_check.cpp", BUILD / "local_ba_shim_check",
                   ("-I" + str(ROOT / "include"), "-Wall", "-Werror"))
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "OK local_ba_shim_check" in r.stdout, r.stdout + r.stderr


def test_matcher_shim_on_mock_objects():
    """include/orbgpu_matcher.hpp (ORBmatcher drop-in): the flat views built from KeyFrame / Frame /
    MapPoint objects and the writes back into vMatchedPairs and mvpMapPoints, against ABI test doubles."""
    exe = _compile(ROOT / "tests" / "native" / "matcher_shim_check.cpp", BUILD / "matcher_shim_check",
                   ("-I" + str(ROOT / "include"), "-Wall", "-Werror"))
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "OK matcher_shim_check" in r.stdout, r.stdout + r.stderr


def test_extractor_shim_on_mock_opencv():
    """include/orbgpu_cv.hpp (ORBextractor drop-in) compiled against a minimal OpenCV stand-in
    (tests/native/mock_cv) and ABI test doubles: parameters, getters, keypoint / descriptor conversion,
    the capacity retry, errors, and mvImagePyramid downloaded lazily on the first operator[]."""
    exe = _compile(ROOT / "tests" / "native" / "cv_shim_check.cpp", BUILD / "cv_shim_check",
                   ("-I" + str(ROOT / "include"), "-I" + str(ROOT / "tests" / "native" / "mock_cv"),
                    "-Wall", "-Werror"))
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "OK cv_shim_check" in r.stdout, r.stdout + r.stderr


@pytest.mark.slow
def test_sincos_exception_table_exhaustive():
    """All 1,135,869,952 float angles in [0, 360): deterministic sincos + table == glibc offsets."""
    exe = _compile(ROOT / "tools" / "gen_sincos_exceptions.cpp", BUILD / "sincos_check", ("-DORB_CHECK_TABLE",))
    r = subprocess.run([str(exe), "--check"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "\nOK: " in "\n" + r.stdout, r.stdout + r.stderr


def test_tracking_chain_abi_host_side(pkg):
    """The tracking chain entry points' host side, no device work: scratch sizes (the batch's grow with
    the frame count and cover one chain's per frame) and argument rejection with ORB_ERR_ARG."""
    from orbslam3_amd import _lib
    _ensure_lib()
    lib = _lib.load()
    one = lib.orb_tracking_chain_scratch_bytes(1850, 1855, 1800)
    b1 = lib.orb_tracking_chain_batch_scratch_bytes(1, 1850, 1855, 1800)
    b8 = lib.orb_tracking_chain_batch_scratch_bytes(8, 1850, 1855, 1800)
    assert one > 0 and b1 >= one and b8 >= 8 * one
    assert lib.orb_tracking_chain_scratch_bytes(0, 10, 10) == 0
    assert lib.orb_tracking_chain_batch_scratch_bytes(0, 1850, 10, 10) == 0
    assert lib.orb_tracking_chain_batch_device(None, None, 0, None, None, None, None) == _lib.ORB_ERR_ARG
    assert lib.orb_tracking_chain_device(None, None, None, None, None, None, None, None, None, None, None, None, None,
                                         None, None, None) == _lib.ORB_ERR_ARG
