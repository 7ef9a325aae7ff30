export TMPDIR=/tmp
timeout -k 10 120 python3 tools/ba_time.py --gpu-only > gpurun_out/rows_mf2_time.txt 2>&1 || exit 1
ORBGPU_BA_CHOL=rows timeout -k 10 120 python3 tools/ba_time.py --gpu-only > gpurun_out/rows_rows_time.txt 2>&1 || exit 1
ORBGPU_BA_CHOL=rows timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/rows_kt -o k -- python3 tools/ba_time.py --gpu-only > /dev/null 2>&1 || exit 1
python3 tools/ba_gaps.py gpurun_out/rows_kt/k_kernel_trace.csv > gpurun_out/rows_kernels.txt
