#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per kernel (mean per dispatch over the run)."""
import csv
import collections
import glob
import json
import re
import sys


def short(name):
    m = re.search(r"(k_[a-z0-9_]+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{d}/pass*_counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            k = short(row["Kernel_Name"])
            per[k][row["Counter_Name"]].append((int(row["Dispatch_Id"]), float(row["Counter_Value"])))
    out = {}
    for k, cs in per.items():
        out[k] = {}
        for c, vals in cs.items():
            by = collections.defaultdict(float)
            for d_id, v in vals:
                by[d_id] += v
            out[k][c] = sum(by.values()) / max(1, len(by))
    return out


if __name__ == "__main__":
    d = sys.argv[1]
    res = load(d)
    cols = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU",
            "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_LDS_BANK_CONFLICT",
            "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "FETCH_SIZE", "WRITE_SIZE"]
    print("kernel".ljust(24) + "".join(c.replace("SQ_", "")[:12].rjust(13) for c in cols))
    for k, cs in sorted(res.items()):
        print(k[:24].ljust(24) + "".join(f"{cs.get(c, float('nan')):13.4g}" for c in cols))
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"), indent=1)
