#!/bin/bash
# BA iteration on the GPU box: parity tests, the Cholesky phase trace, solve timing and a kernel trace.
#   tools/ba_check.sh [tag]  -> gpurun_out/ba_<tag>_*.{log,txt}
set -u
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py tests/test_ba_variants_gpu.py tests/test_shims_gpu.py \
  tests/test_workloads_gpu.py -k "ba or BA or local" -x -q --timeout 200 --timeout-method thread > $O/ba_${T}_tests.log 2>&1
rc=$?
tail -3 $O/ba_${T}_tests.log
[ $rc -eq 0 ] || exit $rc
ORBGPU_BA_TRACE=1 timeout -k 10 120 python3 tools/ba_trace.py > $O/ba_${T}_trace.log 2>&1 || exit 1
python3 tools/chol_trace_summary.py $O/ba_${T}_trace.log > $O/ba_${T}_trace_summary.txt || exit 1
head -3 $O/ba_${T}_trace_summary.txt
grep "^\[ba\]" $O/ba_${T}_trace.log | tail -3
timeout -k 10 120 python3 tools/ba_time.py --gpu-only > $O/ba_${T}_time.txt 2>&1 || exit 1
cat $O/ba_${T}_time.txt
timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $PWD/$O/ba_${T}_kt -o k -- python3 tools/ba_time.py --gpu-only > /dev/null 2>&1 || exit 1
python3 tools/ba_gaps.py $O/ba_${T}_kt/k_kernel_trace.csv > $O/ba_${T}_kernels.txt
cat $O/ba_${T}_kernels.txt
