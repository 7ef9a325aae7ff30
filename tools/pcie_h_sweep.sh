#!/bin/bash
# PCIe-inclusive C2 (bench.py --pcie-only) at several handle counts (ORB_PCIE_H), alternating, two
# passes each: gpurun_out/pcie_h/sweep.txt
set -u
O=gpurun_out/pcie_h; mkdir -p $O
: > $O/sweep.txt
for pass in 1 2; do
  for h in ${@:-3 4 5 6}; do
    ORB_PCIE_H=$h timeout -k 10 120 python3 bench.py --pcie-only --steps 20 > $O/h$h.json 2> $O/h$h.err || { echo "H=$h failed"; tail -5 $O/h$h.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/h$h.json').read().strip().splitlines()[-1]); print('H=$h', d['features_per_ms'], d['ms_per_step'], d['frac_of_bound'])" | tee -a $O/sweep.txt
  done
done
