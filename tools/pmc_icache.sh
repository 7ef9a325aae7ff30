#!/bin/bash
# Instruction-cache counters of the LocalBA (C5) solve's kernels (one rocprofv3 --pmc pass).
set -u
export TMPDIR=/tmp
O=${1:-gpurun_out/pmc_ic}; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH --kernel-trace --output-format csv -d $O -o ic -- python3 tools/ba_time.py --gpu-only > $O/ic.log 2>&1 || { tail -5 $O/ic.log; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:40]; acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    print(k, {c: round(v / n[(k, c)]) for c, v in d.items()})
PY
