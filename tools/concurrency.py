#!/usr/bin/env python3
"""Kernel concurrency in a window of a rocprofv3 kernel trace (csv): the fraction of the window with at
least one kernel running, the mean number running, and each kernel's share of the kernel-time.
    tools/concurrency.py TRACE.csv [FIRST_DISPATCH] [N_DISPATCHES]
(defaults: the middle 2000 dispatches of the trace)"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = len(rows)
cnt = int(sys.argv[3]) if len(sys.argv) > 3 else min(2000, n)
first = int(sys.argv[2]) if len(sys.argv) > 2 else max(0, n // 2 - cnt // 2)
if first < 0:
    first += n
win = rows[first:first + cnt]
t0 = int(win[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in win)
ev = []
per = collections.Counter()
for r in win:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    ev += [(s, 1), (e, -1)]
    nm = r["Kernel_Name"]
    per[nm[nm.find("k_"):].split("(")[0].split("<")[0][:40] if "k_" in nm else nm[:40]] += e - s
ev.sort()
busy = area = 0
cur, last = 0, t0
hist = collections.Counter()
for t, d in ev:
    if cur > 0:
        busy += t - last
    area += cur * (t - last)
    hist[cur] += t - last
    cur += d
    last = t
span = t1 - t0
print(f"window {cnt} dispatches, {span / 1e3:.1f} us: busy {busy / span:.3f}, mean concurrency {area / span:.2f}")
print("time at concurrency k:", {k: round(v / span, 3) for k, v in sorted(hist.items())})
tot = sum(per.values())
for k, v in per.most_common():
    print(f"  {k:40s} {v / tot:.3f} of kernel-time")
