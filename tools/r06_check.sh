#!/bin/bash
# Round-6 iteration check on the GPU box: the changed parity tests, then the LocalBA timing and the
# Cholesky phase trace.  Outputs under gpurun_out/r06/.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest ${TESTS:-tests/test_tracking_chain_gpu.py tests/test_shims_gpu.py tests/test_ba_gpu.py tests/test_ba_dist_gpu.py tests/test_workloads_gpu.py} -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python3 tools/ba_time.py --gpu-only > $O/ba_time.txt 2>&1 || { echo "ba_time failed"; tail -5 $O/ba_time.txt; exit 1; }
cat $O/ba_time.txt
timeout -k 10 200 python3 tools/ba_trace.py > $O/ba_trace.log 2>&1 || { echo "ba_trace failed"; tail -5 $O/ba_trace.log; exit 1; }
python3 tools/chol_trace_summary.py $O/ba_trace.log > $O/chol_trace_summary.txt && head -3 $O/chol_trace_summary.txt
