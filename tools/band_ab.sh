#!/bin/bash
# A/B of the pyramid paths on the GPU box: extraction parity tests (default config and hybrid),
# then bench (stage times) for several pyramid configurations.
set -u
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_extract_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { echo "tests failed"; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
ORBGPU_PYR_BAND_FROM=3 timeout -k 10 300 python -u -m pytest tests/test_extract_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t3.log 2>&1 || { echo "hybrid tests failed"; tail -30 $O/t3.log; exit 1; }
tail -1 $O/t3.log
for cfg in "ORBGPU_PYR_BAND=0" "ORBGPU_PYR_BAND_FROM=0" "ORBGPU_PYR_BAND_FROM=2" "ORBGPU_PYR_BAND_FROM=3" "ORBGPU_PYR_BAND_FROM=4" "ORBGPU_PYR_BAND_FROM=3 ORBGPU_PYR_BAND_R=8" "ORBGPU_PYR_BAND_R=8 ORBGPU_PYR_WG_PER_CU=2" "ORBGPU_PYR_BAND_FROM=3 ORBGPU_PYR_BAND_R=8 ORBGPU_PYR_WG_PER_CU=2"; do
  env $cfg timeout -k 10 120 python bench.py --no-cpu-baseline --no-ba --steps 20 > $O/bench.json 2>$O/bench.err || { echo "bench failed $cfg"; tail $O/bench.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench.json')); print('$cfg', d['value'], d['ms_per_step'], d['stages_ms'])"
done
