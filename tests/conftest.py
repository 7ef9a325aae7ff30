"""Shared pytest setup: markers, package loader (the package dir has a hyphen), oracle access."""
from __future__ import annotations

import importlib.util
import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
PKG_DIR = ROOT / "orb-slam3_byzyh_amd"
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def load_package():
    """Import orb-slam3_byzyh_amd/ under the module name `orbslam3_amd`."""
    if "orbslam3_amd" in sys.modules:
        return sys.modules["orbslam3_amd"]
    spec = importlib.util.spec_from_file_location("orbslam3_amd", PKG_DIR / "__init__.py",
                                                  submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["orbslam3_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box with -m gpu)")
    config.addinivalue_line("markers", "slow: exhaustive CPU checks (seconds to a minute)")


@pytest.fixture(scope="session")
def pkg():
    return load_package()


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as o
    o.load()
    return o


@pytest.fixture(scope="session")
def synth(pkg):
    from orbslam3_amd import synth as s
    return s
