#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py into profiles/pmc_latest.json.

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch.  Per MI355X_MICROARCH.md (HBM section) gfx950's
FETCH_SIZE counts half the bytes of wide coalesced reads, so it is doubled.  Totals are per step of
the stage, summed over the stage's launches, to match bench.py's roofline.achieved.
"""
import collections
import csv
import glob
import json
import re
import sys

STAGE_KERNELS = {"pyramid": ["k_pyramid_pair", "k_pyramid_level"], "fast": ["k_fast_cells"], "quadtree": ["k_quadtree_kp"],
                 "describe": ["k_describe"]}
# launches per step: 4 two-level pyramid passes (8 level passes with ORBGPU_PYR_PAIR=0); FAST two (levels 0-2, 3-7), quad-tree and describe one each (the bench's handles
# run one chain per batch, orb_extractor_set_overlap(h, 0); with the side-stream overlap they are two)
LAUNCHES = {"k_pyramid_pair": 4, "k_pyramid_level": 8, "k_fast_cells": 2, "k_quadtree_kp": 1, "k_describe": 1}


def main(d, out, frames=64):
    per = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        for row in csv.DictReader(open(f)):
            m = re.search(r"(k_[a-z0-9_]+)", row["Kernel_Name"])
            if not m:
                continue
            per[m.group(1)][row["Counter_Name"]][int(row["Dispatch_Id"])] += float(row["Counter_Value"])
    res = {"frames_per_launch": frames, "unit_note": "bytes per step of the stage (all its launches); "
           "FETCH_SIZE doubled for the gfx950 half-count of wide reads", "stages": {}}
    for stage, ks in STAGE_KERNELS.items():
        fetch = write = 0.0
        launches = 0
        for k in ks:
            cs = per.get(k, {})
            fd = cs.get("FETCH_SIZE", {})
            wd = cs.get("WRITE_SIZE", {})
            if not fd:
                continue
            # per-dispatch averages x launches per step
            nper = LAUNCHES.get(k, 1)
            fetch += 2 * 1024 * sum(fd.values()) / len(fd) * nper
            if wd:
                write += 1024 * sum(wd.values()) / len(wd) * nper
            launches += nper
        if launches:
            res["stages"][stage] = {"fetch_bytes": fetch, "write_bytes": write, "hbm_bytes": fetch + write,
                                    "launches_per_step": launches}
            # integer-VALU bound: a wave64 VALU instruction issues over 2 cycles
            # (MI355X_MICROARCH.md), 1024 SIMDs, GRBM_GUI_ACTIVE summed over the 8 XCDs:
            # frac = SQ_INSTS_VALU x 2 / (1024 x GRBM_GUI_ACTIVE / 8), over the stage's dispatches
            for k in ks:
                cs = per.get(k, {})
                vi, ga = cs.get("SQ_INSTS_VALU", {}), cs.get("GRBM_GUI_ACTIVE", {})
                common = sorted(set(vi) & set(ga))
                if common:
                    ins = sum(vi[d] for d in common) / len(common)
                    act = sum(ga[d] for d in common) / len(common)
                    st = res["stages"][stage]
                    st["valu_insts_per_launch"] = ins
                    st["grbm_gui_active_per_launch"] = act
                    st["valu_frac"] = ins * 2 / (1024 * act / 8) if act else None
                lds, bc = cs.get("SQ_INSTS_LDS", {}), cs.get("SQ_LDS_BANK_CONFLICT", {})
                if lds and bc:
                    res["stages"][stage]["lds_conflict_cycles_per_lds_inst"] = sum(bc.values()) / max(1.0, sum(lds.values()))
    dom = max(res["stages"], key=lambda s: res["stages"][s]["hbm_bytes"]) if res["stages"] else None
    res["kernel_stage"] = "pyramid" if "pyramid" in res["stages"] else dom
    if res["kernel_stage"]:
        n = res["stages"][res["kernel_stage"]]["launches_per_step"]
        res["hbm_bytes_per_step"] = res["stages"][res["kernel_stage"]]["hbm_bytes"]
        res["launches_per_step"] = n
        res["hbm_bytes_per_launch"] = res["hbm_bytes_per_step"] / n
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
