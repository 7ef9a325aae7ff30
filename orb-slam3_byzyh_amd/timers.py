"""REGISTER_TIMES-compatible stage timers of the library (csrc/orb_timers.hip): "ORB Extraction",
"Stereo Matching" and "LBA" brackets inside the synchronous entry points, with ExecMean.txt output
(src/Tracking.cc:318-420)."""
from __future__ import annotations

import ctypes

from . import _lib
from ._lib import check

STAGES = ("ORB Extraction", "Stereo Matching", "LBA")


def enable(on: bool = True) -> None:
    check(_lib.load().orb_timers_enable(1 if on else 0), "orb_timers_enable")


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
