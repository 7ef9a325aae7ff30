#!/bin/bash
# Round-end evidence in one GPU call: the GPU parity suite, smoke(), then tools/round_profile.sh
# (bench line, rocprofv3 kernel stats, PMC passes).  Outputs under gpurun_out/round/.
set -u
export TMPDIR=/tmp
O=gpurun_out/round
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/round_profile.sh
