set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/bafuse
timeout -k 10 400 python3 -u -m pytest tests/test_ba_gpu.py tests/test_ba_variants_gpu.py tests/test_ba_dist_gpu.py tests/test_shims_gpu.py "tests/test_workloads_gpu.py::test_local_ba_large_window" -x -q --timeout 200 --timeout-method thread > gpurun_out/bafuse/tests3.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/bafuse/tests3.log; exit 1; }
tail -2 gpurun_out/bafuse/tests3.log
bash tools/ba_unit_trace.sh ORBGPU_BA_FAST_UNIT=0 ORBGPU_BA_FUSED_TRIAL=0
