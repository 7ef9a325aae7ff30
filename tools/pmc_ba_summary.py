"""Per-kernel mean counters of the LocalBA PMC passes (tools/pmc_ba.sh), live launches only for the
unit kernels (a gated no-op launch issues no VALU): one table, counters as columns."""
import collections
import csv
import glob
import re
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_ba"
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{d}/pass*_counter_collection.csv")):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        per[(r["Dispatch_Id"], re.search(r"(k_\w+(<\d+>)?)", r["Kernel_Name"]).group(1))][r["Counter_Name"]] = float(r["Counter_Value"])
    for (_, k), cs in per.items():
        if cs.get("SQ_INSTS_VALU", 1) == 0 and k not in ("k_ba_restore",):
            continue  # a gated-off launch
        if cs.get("SQ_BUSY_CYCLES") is not None and "SQ_INSTS_VALU" not in cs and cs.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) == 0 \
                and k == "k_ba_chol_mf2<11>":
            continue
        for c, v in cs.items():
            vals[k][c].append(v)
cols = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_VALU_MFMA_F64", "SQ_INSTS_VALU_MFMA_MOPS_F64", "SQ_VALU_MFMA_BUSY_CYCLES",
        "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_LDS", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE"]
print(f"{'kernel':22s}" + "".join(f"{c.replace('SQ_', '').replace('INSTS_', '')[:14]:>15s}" for c in cols))
for k in sorted(vals):
    row = vals[k]
    print(f"{k:22s}" + "".join(f"{(sum(row[c]) / len(row[c]) if row.get(c) else float('nan')):15.1f}" for c in cols))
