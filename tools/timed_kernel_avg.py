#!/usr/bin/env python3
"""Average duration of a kernel's dispatches in bench.py's timed region, from a rocprofv3 kernel
trace (--kernel-trace --output-format csv) of an extraction-only bench run:
    tools/timed_kernel_avg.py TRACE.csv STEPS [KERNEL_SUBSTRING] [LAUNCHES_PER_STEP]
The timed region is the last STEPS steps of extraction work (LAUNCHES_PER_STEP dispatches each), so
its dispatches are the last STEPS * LAUNCHES_PER_STEP of the kernel in dispatch order.  This is the
number bench.py's roofline.launch_avg_us (per-block wall-clock spans) is compared with."""
import csv
import sys

path, steps = sys.argv[1], int(sys.argv[2])
name = sys.argv[3] if len(sys.argv) > 3 else "k_pyramid_level"
per = int(sys.argv[4]) if len(sys.argv) > 4 else 8
rows = [r for r in csv.DictReader(open(path)) if name in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
tail = rows[-steps * per:]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in tail]
print(f"{name}: {len(rows)} dispatches, timed region {len(tail)}: avg {sum(d) / len(d):.2f} us, "
      f"all dispatches avg {sum((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in rows) / len(rows):.2f} us")
