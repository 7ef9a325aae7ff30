#!/bin/bash
# A/B of the MFMA Cholesky variants (tile-wave count ORBGPU_BA_MF_W, diagonal/backward broadcast by
# readlane or DPP) on the C5 solve: timing, bitwise result comparison, trace; run on the GPU box.
set -e
for w in 7 11; do
  ORBGPU_BA_MF_W=$w ORBGPU_BA_DIAG_READLANE=1 timeout -k 10 120 python3 tools/ba_time.py --gpu-only > gpurun_out/abw_${w}_rl.log 2>&1
  ORBGPU_BA_MF_W=$w timeout -k 10 120 python3 tools/ba_time.py --gpu-only > gpurun_out/abw_${w}_dpp.log 2>&1
  ORBGPU_BA_MF_W=$w ORBGPU_BA_DIAG_READLANE=1 timeout -k 10 120 python3 tools/ba_dump.py gpurun_out/abw_${w}_rl.npz
  ORBGPU_BA_MF_W=$w timeout -k 10 120 python3 tools/ba_dump.py gpurun_out/abw_${w}_dpp.npz
done
ORBGPU_BA_MF_W=11 timeout -k 10 120 python3 tools/ba_trace.py > gpurun_out/abw_trace.log 2>&1
ORBGPU_BA_MF_W=11 timeout -k 10 200 python -u -m pytest tests/test_ba_gpu.py tests/test_ba_dist_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/abw_test.log 2>&1
