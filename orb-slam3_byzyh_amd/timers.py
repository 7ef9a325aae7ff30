"""REGISTER_TIMES-compatible stage timers of the library (csrc/orb_timers.hip): "ORB Extraction" and
"Stereo Matching" brackets inside the synchronous entry points, "LBA" around the host side of
LocalBundleAdjustment (the C++ shim, optimizer.local_bundle_adjustment), with ExecMean.txt output
(src/Tracking.cc:318-420).  Mode 2 leaves the per-call brackets off for callers that time a whole
Frame themselves (one "ORB Extraction" sample per stereo Frame, as src/Frame.cc:132-146 records it)."""
from __future__ import annotations

import ctypes

from . import _lib
from ._lib import check

STAGES = ("ORB Extraction", "Stereo Matching", "LBA")


def enable(on: bool | int = True) -> None:
    """True / 1: per-call brackets; 2: caller brackets only (add()); False / 0: off."""
    mode = int(on) if not isinstance(on, bool) else (1 if on else 0)
    check(_lib.load().orb_timers_enable(mode), "orb_timers_enable")


def enabled() -> int:
    return int(_lib.load().orb_timers_enabled())


def reset() -> None:
    check(_lib.load().orb_timers_reset(), "orb_timers_reset")


def add(name: str, ms: float) -> None:
    check(_lib.load().orb_timer_add(name.encode(), float(ms)), "orb_timer_add")


def stats(name: str) -> tuple[float, float, int]:
    """(mean ms, population std ms, count) of one stage."""
    m, s, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_longlong()
    check(_lib.load().orb_timer_stats(name.encode(), ctypes.byref(m), ctypes.byref(s), ctypes.byref(n)),
          "orb_timer_stats")
    return m.value, s.value, n.value


def write(path: str) -> None:
    """The ExecMean.txt lines, "Stage: mean$\\pm$std", of every stage with samples."""
    check(_lib.load().orb_timers_write(str(path).encode()), "orb_timers_write")
