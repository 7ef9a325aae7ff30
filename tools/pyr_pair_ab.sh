#!/bin/bash
# A/B of the two-level pyramid pass (ORBGPU_PYR_PAIR=1, default) against level by level (=0): the C2
# step time (tools/c2_ablate.py, no stage skipped), alternated.
set -u
for r in 1 2; do
  for v in ${MODES:-1 0}; do
    echo "PYR_PAIR=$v: $(ORBGPU_PYR_PAIR=$v timeout -k 10 200 python3 tools/c2_ablate.py 0 | tr '\n' ' ')" || exit 1
  done
done
