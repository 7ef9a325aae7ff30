#!/bin/bash
# Extraction parity + bench stage times (default path), for pyramid/FAST kernel iterations.
set -u
O=gpurun_out/pab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_extract_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { echo "tests failed"; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2; do
timeout -k 10 120 python bench.py --no-cpu-baseline --no-ba --no-stereo --no-pose --no-bow --no-single --no-c4 --no-matchers --steps 30 > $O/bench.json 2>$O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['stages_ms'], d['roofline']['frac'])"
done
