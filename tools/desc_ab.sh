#!/bin/bash
# Describe-kernel A/B: extraction parity (default path), then bench stage times per variant
# (ORBGPU_DESC_FLAT=0 is the one-chunk-per-block kernel; ORBGPU_DESC_BLOCKS sets blocks per frame).
set -u
O=gpurun_out/dab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_extract_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { echo "tests failed"; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
run() {
  env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --no-ba --no-stereo --no-pose --no-bow --no-single --no-c4 --no-matchers --steps 30 > $O/bench.json 2>$O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench.json')); print(sys.argv[1:], d['value'], d['ms_per_step'], d['stages_ms'])" "$@"
}
for v in "${@:-ORBGPU_DESC_FLAT=1}"; do run $v; done
