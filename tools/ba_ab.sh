#!/bin/bash
# A/B of BA solve timing on the GPU box: the host phases of a few solves (ORBGPU_BA_TRACE) and
# tools/ba_time.py under each "VAR=value" given (plus the default).  tools/ba_ab.sh tag [VAR=v ...]
set -u
export TMPDIR=/tmp
T=${1:-x}; shift
O=gpurun_out
ORBGPU_BA_TRACE=1 timeout -k 10 120 python3 tools/ba_trace.py > $O/ab_${T}_trace.log 2>&1 || exit 1
grep "^\[ba\]" $O/ab_${T}_trace.log | tail -6
echo "default:"; timeout -k 10 120 python3 tools/ba_time.py --gpu-only 2>&1 | grep stereo || exit 1
for kv in "$@"; do
  echo "$kv:"; env "$kv" timeout -k 10 120 python3 tools/ba_time.py --gpu-only 2>&1 | grep stereo || exit 1
done
