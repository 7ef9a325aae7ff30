export TMPDIR=/tmp
ORBGPU_BA_TRACE=1 timeout -k 10 120 python3 tools/ba_trace.py > gpurun_out/ba_t7.log 2>&1
