"""Per-unit timeline of the BA solve from a rocprofv3 kernel trace (rocpd sqlite db or the csv
`*_kernel_trace.csv`): kernel durations and the idle gaps between consecutive dispatches (median over
dispatches of each kernel)."""
import csv
import sqlite3
import sys
from collections import defaultdict
from statistics import median


def rows_of(path):
    if path.endswith(".csv"):
        with open(path) as f:
            r = csv.DictReader(f)
            out = [(d["Kernel_Name"], int(d["Start_Timestamp"]), int(d["End_Timestamp"])) for d in r]
        return sorted(out, key=lambda t: t[1])
    c = sqlite3.connect(path)
    return c.execute("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s "
                     "on d.kernel_id=s.id order by d.start").fetchall()


dur = defaultdict(list)
gap = defaultdict(list)
prev_end = None
for name, st, en in rows_of(sys.argv[1]):
    short = name.replace("(anonymous namespace)::", "").replace("_ZN12_GLOBAL__N_1", "")
    short = (short[5:] if short.startswith("void ") else short).split("(")[0][:40]
    dur[short].append((en - st) / 1e3)
    if prev_end is not None and 0 <= st - prev_end < 200e3:
        gap[short].append((st - prev_end) / 1e3)
    prev_end = en
print(f"{'kernel':42s} {'n':>5s} {'dur_med':>8s} {'gap_before_med':>15s}")
for k in dur:
    d = median(dur[k])
    g = median(gap[k]) if gap[k] else 0.0
    print(f"{k:42s} {len(dur[k]):5d} {d:8.2f} {g:15.2f}")
