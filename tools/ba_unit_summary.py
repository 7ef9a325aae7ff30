"""Median duration of each LocalBA unit kernel over its live launches, from a rocprofv3 kernel trace
(csv).  A launch is live when the Cholesky of its unit ran (the gated no-op units after a solve's end
return at once: their Cholesky takes a few microseconds, a live one ~100); the graph boundary gap is reported too."""
import csv
import re
import statistics
import sys

UNIT = ("k_u_land_build", "k_u_schur2", "k_u_edges_build", "k_u_reduce_build", "k_ba_schur_edges", "k_u_schur",
        "k_ba_chol_mf2", "k_u_pose_update", "k_u_backsub_update", "k_u_edges_trial", "k_u_land_trial", "k_u_land_trial8")
START = ("k_u_edges_build", "k_u_land_build")  # the first launch of a unit (6-launch / fast unit)


def short(name):
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name[:30]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ev = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
dur = {k: [] for k in UNIT}
gaps = []
live = False
for i, (k, s, e) in enumerate(ev):
    if k not in UNIT:
        continue
    if k in START:  # a unit starts: live if its Cholesky (next mf2 launch) ran
        nxt = next((x for x in ev[i:] if x[0] == "k_ba_chol_mf2"), None)
        live = nxt is not None and nxt[2] - nxt[1] > 30000  # a gated-off Cholesky launch is a few us
        if i and ev[i - 1][0] in UNIT and live:
            gaps.append((s - ev[i - 1][2]) / 1e3)
    if live:
        dur[k].append((e - s) / 1e3)
tot = 0.0
for k in UNIT:
    if dur[k]:
        m = statistics.median(dur[k])
        tot += m
        print(f"  {k:20s} n {len(dur[k]):4d} median {m:8.2f} us")
print(f"  sum of medians {tot:.1f} us; unit-start gaps: median {statistics.median(gaps) if gaps else 0:.2f} us "
      f"({sum(1 for g in gaps if g > 1)} of {len(gaps)} above 1 us)")
