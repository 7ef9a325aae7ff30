#!/bin/bash
# LocalBA C5: units per graph launch (ORBGPU_BA_UNITS), alternating, tools/ba_time.py --gpu-only.
set -u
O=gpurun_out/baunits
mkdir -p $O
for i in 1 2; do
  for u in 2 3 4 8; do
    timeout -k 10 120 env ORBGPU_BA_UNITS=$u python3 tools/ba_time.py --gpu-only > $O/u${u}_$i.txt 2>&1 || { cat $O/u${u}_$i.txt; exit 1; }
    echo "units $u run $i"; grep stereo $O/u${u}_$i.txt
  done
done
