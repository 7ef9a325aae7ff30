#!/bin/bash
# Kernel durations of the BA unit under rocprofv3 for Cholesky variants (run on the GPU box):
#   tools/ba_chol_prof.sh  -> gpurun_out/bacp_<variant>/ + summary lines in gpurun_out/bacp.txt
set -e
export TMPDIR=/tmp
: > gpurun_out/bacp.txt
for v in "7 1" "11 0"; do
  set -- $v
  if [ "$2" = 1 ]; then export ORBGPU_BA_DIAG_READLANE=1; else unset ORBGPU_BA_DIAG_READLANE; fi
  ORBGPU_BA_MF_W=$1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bacp_$1_$2 -o k -- python3 tools/ba_time.py --gpu-only > gpurun_out/bacp_$1_$2.log 2>&1
  echo "W=$1 readlane=$2" >> gpurun_out/bacp.txt
  head -12 gpurun_out/bacp_$1_$2/k_kernel_stats.csv | cut -d, -f1-8 >> gpurun_out/bacp.txt
done
