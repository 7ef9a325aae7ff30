#!/bin/bash
# A/B the two Cholesky paths of the BA solve under rocprofv3 (run on the GPU box).
set -e
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_single -o ba -- python3 tools/ba_time.py --gpu-only > gpurun_out/ab_single.log 2>&1
ORBGPU_BA_COOP=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_coop -o ba -- python3 tools/ba_time.py --gpu-only > gpurun_out/ab_coop.log 2>&1
