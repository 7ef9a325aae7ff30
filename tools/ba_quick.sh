#!/bin/bash
# LocalBA on the GPU box: every BA parity test, then tools/ba_time.py --gpu-only twice.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/baq
timeout -k 10 400 python3 -u -m pytest tests/test_ba_gpu.py tests/test_ba_variants_gpu.py tests/test_ba_dist_gpu.py tests/test_shims_gpu.py "tests/test_workloads_gpu.py::test_local_ba_large_window" -x -q --timeout 200 --timeout-method thread > gpurun_out/baq/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/baq/tests.log; exit 1; }
tail -1 gpurun_out/baq/tests.log
for i in 1 2; do timeout -k 10 120 python3 tools/ba_time.py --gpu-only 2>&1 | grep stereo; done
