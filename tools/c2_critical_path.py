#!/usr/bin/env python3
"""Critical path of the C2 step from a rocprofv3 kernel trace (csv) of bench.py: the extraction
kernels grouped into batches per stream (k_pyramid_pair / k_pyramid_level passes -> k_fast_cells -> k_quadtree_kp ->
k_describe on one handle's stream), then per batch its span (first start to last end), the kernel time
inside it, and the gaps between its kernels (the batch waiting for the device: other batches' kernels
hold the CUs, or the host had not enqueued the next launch).  With H batches in flight the step time
is about span / H when the batches overlap fully; the report says where each batch's span goes.
    tools/c2_critical_path.py TRACE.csv [N_BATCHES] [FIRST_BATCH]
(default: the N_BATCHES (20) consecutive batches with the shortest start-to-start period, i.e. the
bench's steady timed steps, not the warm-up or the instrumented second pass)
"""
import collections
import csv
import statistics as st
import sys

STAGES = ("k_pyramid_level", "k_fast_cells", "k_quadtree_kp", "k_describe")


def short(name):
    """Stage of a kernel (the two-level k_pyramid_pair passes count as the pyramid stage)."""
    if "k_pyramid_pair" in name:
        return "k_pyramid_level"
    for s in STAGES:
        if s in name:
            return s
    return None


rows = [r for r in csv.DictReader(open(sys.argv[1])) if short(r["Kernel_Name"])]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
by_stream = collections.defaultdict(list)
for r in rows:
    by_stream[(r["Queue_Id"], r["Stream_Id"])].append(r)
batches = []
for key, rs in by_stream.items():
    cur = []
    for r in rs:  # a batch starts at the first pyramid launch after a describe
        if short(r["Kernel_Name"]) == "k_pyramid_level" and cur and short(cur[-1]["Kernel_Name"]) == "k_describe":
            batches.append((key, cur))
            cur = []
        cur.append(r)
    if cur and short(cur[-1]["Kernel_Name"]) == "k_describe":
        batches.append((key, cur))
batches.sort(key=lambda b: int(b[1][0]["Start_Timestamp"]))
nsel = int(sys.argv[2]) if len(sys.argv) > 2 else 20
bstart = [int(rs[0]["Start_Timestamp"]) for _, rs in batches]
if len(sys.argv) > 3:
    first = int(sys.argv[3])
else:
    first = min(range(max(1, len(batches) - nsel)), key=lambda i: bstart[min(i + nsel, len(bstart) - 1)] - bstart[i])
sel = batches[first:first + nsel]
spans, busy, gaps = [], [], []
stage_t = collections.defaultdict(list)
gap_before = collections.defaultdict(list)
for _, rs in sel:
    t0 = int(rs[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in rs)
    spans.append((t1 - t0) / 1e3)
    k = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs)
    busy.append(k / 1e3)
    gaps.append((t1 - t0 - k) / 1e3)
    per = collections.Counter()
    prev_end = None
    for r in rs:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        nm = short(r["Kernel_Name"])
        per[nm] += e - s
        if prev_end is not None:
            gap_before[nm].append(max(0, s - prev_end) / 1e3)
        prev_end = max(prev_end or 0, e)
    for nm, v in per.items():
        stage_t[nm].append(v / 1e3)
starts = [int(rs[0]["Start_Timestamp"]) for _, rs in sel]
period = (starts[-1] - starts[0]) / 1e3 / max(1, len(starts) - 1)
print(f"{len(batches)} batches in the trace on {len(by_stream)} streams; batches {first}..{first + len(sel) - 1}:")
print(f"  batch span median {st.median(spans):.1f} us = kernels {st.median(busy):.1f} + gaps {st.median(gaps):.1f}")
print(f"  a batch starts every {period:.1f} us (step time per batch); span / period = {st.median(spans) / period:.2f} "
      "batches in flight")
for nm in STAGES:
    if stage_t[nm]:
        g = gap_before[nm]
        print(f"  {nm:16s} {st.median(stage_t[nm]):7.1f} us per batch"
              + (f", gaps before its launches {sum(g) / len(sel):6.1f} us per batch" if g else ""))
